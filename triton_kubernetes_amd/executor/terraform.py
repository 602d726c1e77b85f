"""Terraform executor (reference ``shell/run_terraform.go:11-80``, ``get/*.go``).

Per call: a fresh ``triton-kubernetes-*`` temp dir holding ``main.tf.json``,
``terraform init -force-copy`` and then ``apply -auto-approve`` /
``destroy <flags> -target=…`` / ``output``; the dir is removed afterwards.

Version awareness (the reference pins 0.11.2):

==================  ======================  ==========================================
Terraform           destroy                 module outputs
==================  ======================  ==========================================
< 0.12              ``destroy -force``      ``terraform output -module <key>``
0.12 – 0.14         ``destroy -force``      root outputs ``<key>__<name>`` (rendered)
>= 0.15             ``destroy -auto-approve``  root outputs ``<key>__<name>`` (rendered)
==================  ======================  ==========================================

The document Terraform sees (:func:`render`) differs from the persisted one in three
version-dependent ways; the persisted ``main.tf.json`` keeps the reference's layout:

* for >= 0.12 one root ``output`` per catalog output of every module, so ``get
  manager|cluster`` keep working.  An output the module declares ``sensitive`` (the
  Rancher secret key, the registration token — ``terraform/generate.py`` is the single
  source, read through ``catalog.sensitive_outputs``) is rendered ``sensitive = true``:
  from 0.15 Terraform rejects the whole configuration otherwise ("Output refers to
  sensitive values").  ``terraform output -json`` still prints the values;
* a state backend Terraform no longer has (``manta`` was removed in 1.3, reference
  ``backend/manta/backend.go:196-205``) is replaced by a ``local`` backend inside the
  work dir, and the CLI carries ``terraform.tfstate`` itself: downloaded from the state
  backend before every command, uploaded after ``apply``/``destroy`` (also after a
  failed one: Terraform records what it created before failing), all under the
  backend's lock (the Manta conditional-PUT lock, ``backend/manta.py``);
* modules from a local directory (the packaged tree) are checked against their
  ``required_version`` before ``init``, so a too-old Terraform gets one clear error;
* ``tk::`` module sources (``terraform/catalog.py``) become this install's module
  directories, the backend block becomes the running operator's, and modules that take
  ``tk_operation`` get it from a root variable, which ``destroy`` sets to ``destroy``.

``-parallelism`` is configurable (the reference leaves it at Terraform's default of 10,
which bounds node fan-out).
"""

import contextlib
import copy
import json
import os
import re
import shutil
import tempfile
from dataclasses import dataclass
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

from ..backend.base import Backend
from ..errors import ExecutorError
from ..state import MANAGER_KEY, State
from ..terraform import constraints
from ..terraform.catalog import (check_sources, declared_variables, is_packaged_source, local_module_dir,
                                 module_from_source, outputs_for_source, resolve_source, sensitive_outputs)
from ..parallel.hostkeys import HostKeys, keys_for, preferred_key
from ..utils.jsonenc import dumps_go
from .base import Executor, outputs_from_tfstate
from .shell import ShellOptions, capture_command, run_shell_command

_VERSION_RE = re.compile(r"Terraform v(\d+)\.(\d+)\.(\d+)")
WORKDIR_TFSTATE = "terraform.tfstate"


def parse_version(text: str) -> Tuple[int, int, int]:
    m = _VERSION_RE.search(text)
    if not m:
        try:
            data = json.loads(text)
            return tuple(int(x) for x in data["terraform_version"].split(".")[:3])  # type: ignore[return-value]
        except (ValueError, KeyError, TypeError):
            raise ExecutorError(f"could not determine terraform version from {text!r}")
    return int(m.group(1)), int(m.group(2)), int(m.group(3))


@dataclass
class Rendered:
    body: bytes
    # the state backend is one this Terraform lacks: the CLI carries terraform.tfstate
    managed_state: bool = False
    backend_kind: str = ""
    # the root variable tk_operation is declared (some module takes it): -var may set it
    operation_var: bool = False


# The root variable through which the executor tells the modules' data sources which CLI
# operation runs them (terraform/generate.py, ``tk_operation``): ``apply`` finds or
# creates, ``destroy`` / ``read`` only find and tolerate hosts that are gone.
OPERATION_VAR = "tk_operation"
# ... and the one carrying the manager's pinned SSH host keys to their SSH reads
KNOWN_HOSTS_VAR = "tk_known_hosts"
# module output of the keys those reads pinned (merged back into the store after an apply)
KNOWN_HOSTS_OUTPUT = "tk_ssh_known_hosts"
# the manager's pinned Rancher CA for the modules' Rancher calls (rancher/trust.py) ...
RANCHER_CA_VAR = "tk_rancher_ca"
# ... the manager module output it is first pinned from (read on the manager host)
RANCHER_CA_OUTPUT = "tk_rancher_ca_certs"
# the random first-login password (rancher/bootstrap_secret.py), a sensitive root variable
# rendered into the manager modules' rancher_bootstrap_password
BOOTSTRAP_VAR = "tk_rancher_bootstrap_password"
# the staged prebuilt MI355X node tools (node/tools.py), uploaded by the MI355X host modules
PREBUILT_VAR = "tk_prebuilt_tools"
PREBUILT_SUBDIR = "tk-prebuilt-tools"


def _backend_kind(doc: Dict) -> str:
    block = ((doc.get("terraform") or {}).get("backend") or {})
    return next(iter(block), "") if isinstance(block, dict) else ""


def check_module_versions(state: State, version: Tuple[int, int, int]) -> None:
    """Raise when a module from a local directory declares a ``required_version`` that
    ``version`` does not meet (Terraform's own init error, reported up front), when a
    ``tk::`` source is pinned to another CLI version, or when an absolute-path source
    written by another install (a pre-``tk::`` document) does not exist here."""
    check_sources(state.modules())
    seen = set()
    for key, mod in state.modules().items():
        local = local_module_dir(str(mod.get("source", "")))
        if local is None or local in seen:
            continue
        seen.add(local)
        bad = constraints.unsupported_by(version, local)
        if bad is not None:
            raise ExecutorError(
                f"module.{key} ({os.path.basename(local.rstrip('/'))}) requires Terraform {bad}; "
                f"found v{constraints.fmt(version)}. Install a newer Terraform, or point source_url/source_ref "
                "at modules written for this version.")


def resolve_sources(doc: Dict) -> Dict:
    """``doc`` (copied when anything changes) with every ``tk::`` module source replaced
    by this install's module directory (``terraform/catalog.py:resolve_source``)."""
    modules = doc.get("module") or {}
    if not any(is_packaged_source(str((m or {}).get("source", ""))) for m in modules.values()):
        return doc
    doc = dict(doc)
    doc["module"] = {k: (dict(m, source=resolve_source(str(m["source"]), k))
                         if is_packaged_source(str((m or {}).get("source", ""))) else m)
                     for k, m in modules.items()}
    return doc


def render(state: State, version: Tuple[int, int, int], backend: Optional[Backend] = None,
           known_hosts: str = "", rancher_ca: str = "", bootstrap_password: str = "",
           prebuilt_tools: str = "") -> Rendered:
    """The document Terraform sees (see module docstring).

    With ``backend`` the backend block is this operator's (``state_terraform_config``),
    when it is of the same kind as the persisted one: a shared document carries the key
    path of whoever wrote it (``key_material``, reference ``backend/manta/backend.go:199``).
    ``known_hosts``: the manager's pinned SSH host keys (``parallel/hostkeys.py``), for the
    modules' SSH reads (root variable) and their provisioner connections (``host_key``,
    ``bastion_host_key`` of each pinned host).  ``rancher_ca``: its pinned Rancher CA
    (``tk_rancher_ca`` of the cluster and add-on modules).  ``bootstrap_password``: the
    random first-login password (``rancher_bootstrap_password`` of a manager module that
    does not set one; a sensitive root variable).  ``prebuilt_tools``: the directory of staged
    node tools (``tk_prebuilt_tools`` of the MI355X host modules)."""
    doc = resolve_sources(state.doc)
    kind = _backend_kind(doc)
    if backend is not None and kind:
        path, block = backend.state_terraform_config(state.name)
        if path == f"terraform.backend.{kind}" and block != doc["terraform"]["backend"][kind]:
            doc = dict(doc, terraform=dict(doc["terraform"], backend={kind: block}))
    managed = bool(kind) and constraints.backend_removed(kind, version)
    if version < (0, 12, 0) and not managed:
        return Rendered(dumps_go(doc), False, kind)
    doc = copy.deepcopy(doc)
    if managed:
        doc["terraform"]["backend"] = {"local": {"path": WORKDIR_TFSTATE}}
    root_vars: Dict[str, str] = {}
    if version >= (0, 12, 0):
        for mod in (doc.get("module") or {}).values():
            local = local_module_dir(str(mod.get("source", "")))
            declared = declared_variables(local) if local else frozenset()
            for var, default in ((OPERATION_VAR, "apply"), (KNOWN_HOSTS_VAR, known_hosts),
                                 (RANCHER_CA_VAR, rancher_ca), (PREBUILT_VAR, prebuilt_tools)):
                if var in declared and var not in mod:
                    mod[var] = f"${{var.{var}}}"
                    root_vars[var] = default
            if bootstrap_password and "rancher_bootstrap_password" in declared and \
                    not mod.get("rancher_bootstrap_password"):
                mod["rancher_bootstrap_password"] = f"${{var.{BOOTSTRAP_VAR}}}"
                root_vars[BOOTSTRAP_VAR] = bootstrap_password
            for var, addr in (("host_key", mod.get("host")), ("bastion_host_key", mod.get("bastion_host"))):
                pinned = keys_for(known_hosts, str(addr or "")) if known_hosts and addr else []
                if var in declared and var not in mod and pinned:
                    mod[var] = preferred_key(pinned)  # the type Terraform's Go client negotiates
        for var, default in root_vars.items():
            doc.setdefault("variable", {})[var] = {"type": "string", "default": default}
            if var == BOOTSTRAP_VAR and version >= (0, 14, 0):
                doc["variable"][var]["sensitive"] = True
        outputs = doc.setdefault("output", {})
        for key, mod in state.modules().items():
            source = str(mod.get("source", ""))
            info = module_from_source(source)
            secret = set(sensitive_outputs(info.name)) if info else set()
            for out in outputs_for_source(source):
                block = {"value": f"${{module.{key}.{out}}}"}
                if out in secret:
                    block["sensitive"] = True
                outputs[f"{key}__{out}"] = block
        if not outputs:
            doc.pop("output")
    return Rendered(dumps_go(doc), managed, kind, OPERATION_VAR in root_vars)


def _takes(state: State, var: str) -> bool:
    """Some module of ``state`` declares ``var`` and does not set it itself."""
    for mod in (resolve_sources(state.doc).get("module") or {}).values():
        local = local_module_dir(str(mod.get("source", "")))
        if local and var in declared_variables(local) and var not in mod:
            return True
    return False


def render_document(state: State, version: Tuple[int, int, int]) -> bytes:
    return render(state, version).body


class TerraformExecutor(Executor):
    name = "terraform"

    def __init__(
        self,
        binary: str = "terraform",
        parallelism: Optional[int] = None,
        env: Optional[Dict[str, str]] = None,
        timeout: Optional[float] = None,
        version: Optional[Tuple[int, int, int]] = None,
        keep_workdir: bool = False,
        ca_file: str = "",
        stage_tools: bool = True,
    ):
        self.binary = binary
        self.parallelism = parallelism
        self.env = dict(env or {})
        self.timeout = timeout
        self._version = version
        self.keep_workdir = keep_workdir
        self.last_workdir: Optional[str] = None
        self.last_rendered: Optional[Rendered] = None
        self.host_keys: Optional[HostKeys] = None
        # the manager's pinned Rancher CA (rancher/trust.py); ca_file re-pins
        self.trust = None
        self.ca_file = ca_file
        # stage the prebuilt MI355X node tools for the host modules that upload them
        self.stage_tools = stage_tools
        self.last_staged: Dict[str, str] = {}

    # --- helpers -------------------------------------------------------------------------
    def version(self) -> Tuple[int, int, int]:
        if self._version is None:
            res = capture_command(self.binary, "version", env=self.env or None)
            self._version = parse_version(res.stdout)
        return self._version

    def _opts(self, workdir: str) -> ShellOptions:
        return ShellOptions(working_dir=workdir, env=self.env or None, timeout=self.timeout)

    def _run(self, workdir: str, *args: str) -> None:
        run_shell_command(self._opts(workdir), self.binary, *args)

    @contextlib.contextmanager
    def workdir(self, state: State, backend: Optional[Backend] = None, write_back: bool = False,
                stage: bool = False) -> Iterator[str]:
        """Temp dir with the rendered document, initialised.  With CLI-managed state the
        tfstate comes from ``backend`` first and (``write_back``) goes back to it after the
        body, under ``backend.lock``.  ``stage`` (apply): the prebuilt node tools go into the
        dir for the MI355X host modules to upload (``node/tools.py``)."""
        version = self.version()
        check_module_versions(state, version)
        keys = self.host_keys = HostKeys(backend, state.name) if backend is not None else None
        ca, boot = "", ""
        if backend is not None:
            from ..rancher import bootstrap_secret, trust as rtrust

            self.trust = rtrust.load(backend, state.name)
            if self.ca_file:
                self.trust = rtrust.from_file(self.ca_file)
                rtrust.save(backend, state.name, self.trust)
            ca = self.trust.pem if self.trust is not None else ""
            src = str((state.module(MANAGER_KEY) or {}).get("source", ""))
            local = local_module_dir(resolve_source(src, MANAGER_KEY) if is_packaged_source(src) else src) \
                if src else None
            if local and "rancher_bootstrap_password" in declared_variables(local):
                boot = bootstrap_secret.ensure(backend, state.name)
        tmp = tempfile.mkdtemp(prefix="triton-kubernetes-")
        self.last_workdir = tmp
        keep = self.keep_workdir
        try:
            prebuilt = ""
            if stage and version >= (0, 12, 0) and self.stage_tools and _takes(state, PREBUILT_VAR):
                from ..node import tools
                prebuilt = os.path.join(tmp, PREBUILT_SUBDIR)
                self.last_staged = tools.stage(prebuilt)
            rendered = render(state, version, backend, keys.text() if keys is not None else "", ca, boot, prebuilt)
            self.last_rendered = rendered
            if rendered.managed_state and backend is None:
                raise ExecutorError(f"the {rendered.backend_kind} state backend needs the CLI to carry terraform.tfstate")
            with open(os.path.join(tmp, "main.tf.json"), "wb") as fh:
                fh.write(rendered.body)
            if not rendered.managed_state:
                self._run(tmp, "init", "-force-copy", "-input=false")
                yield tmp
                return
            lock = backend.lock(state.name) if write_back else contextlib.nullcontext()
            with lock:
                prior = backend.read_tfstate(state.name)
                path = os.path.join(tmp, WORKDIR_TFSTATE)
                if prior:
                    with open(path, "wb") as fh:
                        fh.write(prior)
                try:
                    self._run(tmp, "init", "-force-copy", "-input=false")
                    yield tmp
                finally:
                    if write_back and os.path.exists(path):
                        with open(path, "rb") as fh:
                            after = fh.read()
                        if after != (prior or b""):
                            try:
                                backend.write_tfstate(state.name, after)
                            except Exception as exc:
                                keep = True
                                raise ExecutorError(
                                    f"could not upload terraform.tfstate to the {rendered.backend_kind} backend "
                                    f"({exc}); it is kept at {path}") from exc
        finally:
            if not keep:
                shutil.rmtree(tmp, ignore_errors=True)

    # --- Executor API ---------------------------------------------------------------------
    def apply(self, state: State, backend: Backend) -> None:
        with self.workdir(state, backend, write_back=True, stage=True) as wd:
            args: List[str] = ["apply", "-auto-approve", "-input=false"]
            if self.parallelism:
                args.append(f"-parallelism={self.parallelism}")
            self._run(wd, *args)
            self._pin_learned_keys(state, wd, backend)

    def _pin_learned_keys(self, state: State, wd: str, backend: Optional[Backend] = None) -> None:
        """Merge the SSH host keys the modules' reads pinned on first contact (their
        ``tk_ssh_known_hosts`` outputs) into the manager's store, and pin the Rancher CA the
        manager module read on its host (``rancher_ca_certs``) when none is pinned yet."""
        if self.host_keys is None or self.version() < (0, 12, 0):
            return
        if not any(KNOWN_HOSTS_OUTPUT in outputs_for_source(str(m.get("source", "")))
                   for m in state.modules().values()):
            return
        res = capture_command(self.binary, "output", "-json", working_dir=wd, env=self.env or None)
        outs = json.loads(res.stdout or "{}") or {}
        for name, out in outs.items():
            if name.endswith("__" + KNOWN_HOSTS_OUTPUT) and isinstance(out, dict) and out.get("value"):
                self.host_keys.add(str(out["value"]))
        self.host_keys.save()
        ca = outs.get(f"{MANAGER_KEY}__{RANCHER_CA_OUTPUT}")
        key = outs.get(f"{MANAGER_KEY}__rancher_access_key")
        # pinned only from a read that worked: read_api_key.sh yields empty keys (and an empty
        # bundle) for a manager it could not reach outside an apply, and a bundle is either a
        # PEM or empty because the server's cacerts setting is (a public certificate)
        read_ok = isinstance(key, dict) and bool(key.get("value"))
        value = ca.get("value") if isinstance(ca, dict) else None
        if value and "BEGIN CERTIFICATE" not in str(value):
            value = None
        if backend is not None and self.trust is None and read_ok and value is not None:
            from ..rancher import trust as rtrust

            mgr = state.module(MANAGER_KEY) or {}
            self.trust = rtrust.RancherTrust(rtrust.normalize(str(value)), f"ssh:{mgr.get('host', '')}")
            rtrust.save(backend, state.name, self.trust)

    def destroy_flags(self) -> List[str]:
        return ["-auto-approve"] if self.version() >= (0, 15, 0) else ["-force"]

    def destroy(self, state: State, backend: Backend, targets: Sequence[str]) -> None:
        """``terraform destroy`` of ``targets`` (all without).  The state is authoritative
        for a destroy: ``-refresh=false`` skips the pre-destroy refresh, which would re-run
        the create-side data sources (the API-key read over SSH from a manager host that may
        be gone; the find-or-create of a Rancher cluster removed out of band, reference
        ``terraform/modules/triton-rancher/main.tf:128-144``, ``rancher_cluster.sh:17-42``).
        Should Terraform still read one, ``tk_operation=destroy`` makes it find-only."""
        with self.workdir(state, backend, write_back=True) as wd:
            args = ["destroy", *self.destroy_flags(), "-refresh=false"]
            if self.last_rendered is not None and self.last_rendered.operation_var:
                args.append(f"-var={OPERATION_VAR}=destroy")
            if self.parallelism:
                args.append(f"-parallelism={self.parallelism}")
            self._run(wd, *args, *[f"-target={t}" for t in targets])

    def outputs(self, state: State, backend: Backend, module_key: str) -> Dict[str, str]:
        with self.workdir(state, backend) as wd:
            if self.version() < (0, 12, 0):
                res = capture_command(self.binary, "output", "-json", f"-module={module_key}",
                                      working_dir=wd, env=self.env or None)
                data = json.loads(res.stdout or "{}")
                return {k: str(v.get("value", "")) for k, v in data.items()}
            res = capture_command(self.binary, "output", "-json", working_dir=wd, env=self.env or None)
            data = json.loads(res.stdout or "{}")
        raw = json.dumps({"outputs": data}).encode()
        return outputs_from_tfstate(raw, module_key)

    def print_outputs(self, state: State, backend: Backend, module_key: str, out) -> None:
        if self.version() < (0, 12, 0):
            # exactly the reference's behaviour: stream `terraform output -module`
            with self.workdir(state, backend) as wd:
                self._run(wd, "output", "-module", module_key)
            return
        super().print_outputs(state, backend, module_key, out)
