"""DirectExecutor: native execution of the bare-metal module family.

Implements, without a Terraform binary, the semantics of

* ``bare-metal-rancher`` (T5): install docker + run ``rancher/server`` over SSH
  (S1, S2), then bootstrap the API (S3) — from the operator side by default, or
  on the host like the reference (``rancher_bootstrap: remote``).  A manager
  ``host`` of the form ``rancher+https://…`` adopts an already running server;
* ``bare-metal-rancher-k8s`` (T10): find-or-create the RKE cluster, its
  registration token and CA checksum (S4) through the Rancher client;
* ``bare-metal-rancher-k8s-host`` (T16) and ``bare-metal-mi355x-rancher-k8s-host``:
  a :class:`~..node.plan.BootstrapPlan` per node, delivered by a transport
  (SSH / node agent / local);
* ``rancher-k8s-mi355x-addons``: wait for the cluster, then apply the ROCm
  device plugin / labeller / RCCL manifests through Rancher's k8s proxy.

Scheduling is a dependency-driven DAG walk over the ``${module.X.Y}``
interpolations: every module whose inputs are available starts immediately,
up to ``parallelism`` (default 64, vs Terraform's 10) in flight — so all N nodes
of a cluster bootstrap concurrently and the add-on step overlaps them.

State: a tfstate-compatible document (root outputs ``<module>__<output>`` plus
per-module config hashes) written to the backend after *every* module, so a
failed apply keeps completed modules and a re-run resumes (unchanged, already
applied modules are skipped — the whole document is re-applied exactly like the
reference's ``terraform apply`` of ``main.tf.json``).
"""

import concurrent.futures as cf
import copy
import hashlib
import json
import re
import threading
import time
import uuid
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Set, Tuple

from .. import __version__
from ..backend.base import Backend
from ..cloud.http import HTTPError
from ..errors import ExecutorError
from ..node.plan import TOOLS_DIR, build_host_plan
from ..parallel.transport import HostRef, Transport, TransportRouter
from ..rancher.client import RancherClient, wait_until
from ..state import MANAGER_KEY, State
from ..terraform.catalog import ModuleInfo, check_sources, module_from_source
from ..terraform import hcl
from ..utils.trace import span
from ..versions import DEFAULT_DISTRIBUTION, default_version
from .base import Executor, outputs_from_tfstate
from .tfstate import CODEC

INTERP_RE = re.compile(r"\$\{module\.([A-Za-z0-9_.-]+?)\.([A-Za-z0-9_]+)\}")
SUPPORTED = {"bare-metal-rancher", "bare-metal-rancher-k8s", "bare-metal-rancher-k8s-host",
             "bare-metal-mi355x-rancher-k8s-host", "rancher-k8s-mi355x-addons"}


def config_hash(cfg: Any) -> str:
    return hashlib.sha256(json.dumps(cfg, sort_keys=True).encode()).hexdigest()[:16]


def fingerprint(cfg: Any) -> Tuple[str, Set[str]]:
    """``(config_hash(cfg), module_deps(cfg))`` from ONE C-encoder pass over ``cfg``.

    Every apply re-plans every module of the manager, so this runs once per module per
    create.  The interpolation pattern holds no ``"`` or ``\\``, so its matches in the
    encoded text are exactly its matches in the document's strings.
    """
    text = json.dumps(cfg, sort_keys=True)
    return hashlib.sha256(text.encode()).hexdigest()[:16], {m.group(1) for m in INTERP_RE.finditer(text)}


def module_deps(cfg: Any) -> Set[str]:
    deps: Set[str] = set()

    def walk(v: Any) -> None:
        if isinstance(v, str):
            deps.update(m.group(1) for m in INTERP_RE.finditer(v))
        elif isinstance(v, dict):
            for x in v.values():
                walk(x)
        elif isinstance(v, list):
            for x in v:
                walk(x)

    walk(cfg)
    return deps


def resolve(cfg: Any, outputs: Dict[str, Dict[str, str]]) -> Any:
    def sub(m: "re.Match") -> str:
        mod, out = m.group(1), m.group(2)
        try:
            return str(outputs[mod][out])
        except KeyError:
            raise ExecutorError(f"module.{mod}.{out} is not available (module not applied?)") from None

    if isinstance(cfg, str):
        return INTERP_RE.sub(sub, cfg)
    if isinstance(cfg, dict):
        return {k: resolve(v, outputs) for k, v in cfg.items()}
    if isinstance(cfg, list):
        return [resolve(v, outputs) for v in cfg]
    return cfg


@dataclass
class ModuleRun:
    key: str
    info: ModuleInfo
    cfg: Dict[str, Any]
    deps: Set[str]
    hash: str = ""
    status: str = "pending"  # pending | skipped | ok | failed | blocked
    error: Optional[str] = None
    start: float = 0.0
    end: float = 0.0
    detail: Any = None
    # module-private state kept in the tfstate between applies (what a Terraform module keeps
    # in its resources' state, e.g. the add-ons' tls_* certificate)
    prev_private: Optional[Dict[str, Any]] = None
    # add-on modules: the injector certificate, started when the walk starts (_prefetch_tls)
    tls: Optional[cf.Future] = None


@dataclass
class ApplyReport:
    runs: Dict[str, ModuleRun] = field(default_factory=dict)
    wall: float = 0.0

    @property
    def ok(self) -> bool:
        return all(r.status in ("ok", "skipped") for r in self.runs.values())

    def summary(self) -> Dict[str, Any]:
        return {k: {"status": r.status, "seconds": round(r.end - r.start, 4) if r.end else None,
                    "error": r.error} for k, r in self.runs.items()}


class DirectExecutor(Executor):
    name = "direct"

    def __init__(self, transport: Optional[Transport] = None, parallelism: int = 64,
                 rancher_factory: Optional[Callable[..., RancherClient]] = None, rancher_bootstrap: str = "operator",
                 node_timeout: float = 3600.0, cluster_wait: float = 1800.0, upload_tools: bool = True,
                 node_cleanup: bool = True, on_event: Optional[Callable[[str, Dict[str, Any]], None]] = None,
                 host_retries: int = 0, retry_backoff: float = 2.0, ca_file: str = ""):
        self.transport = transport or TransportRouter()
        self.parallelism = max(1, parallelism)
        # the manager's pinned Rancher CA (rancher/trust.py), loaded per apply; every client
        # this executor makes verifies the server against it
        self.trust: Optional[Any] = None
        self.ca_file = ca_file
        self._trust_store: Optional[Tuple[Backend, str]] = None
        self.rancher_factory = rancher_factory or (
            lambda url, ak="", sk="": RancherClient(url, ak, sk, trust=self.trust))
        self.rancher_bootstrap = rancher_bootstrap
        self.node_timeout = node_timeout
        self.cluster_wait = cluster_wait
        self.upload_tools = upload_tools
        self.node_cleanup = node_cleanup
        self.on_event = on_event
        # a host module whose bootstrap fails is re-run this many times (plans are idempotent:
        # find-or-create cluster, runtime installed only when absent, agent re-registration)
        self.host_retries = max(0, host_retries)
        self.retry_backoff = retry_backoff
        self.last_report: Optional[ApplyReport] = None
        # host key -> the cleanup report of the last destroy (node/cleanup.py)
        self.last_cleanup: Dict[str, Dict[str, Any]] = {}
        self._mu = threading.Lock()

    # --- tfstate ---------------------------------------------------------------------------------
    @staticmethod
    def _load_tfstate(backend: Backend, name: str) -> Dict[str, Any]:
        doc = CODEC.load(name, backend.read_tfstate(name))
        if doc is not None:
            return doc
        return {"version": 4, "terraform_version": f"tk-direct-{__version__}", "serial": 0,
                "lineage": str(uuid.uuid4()), "resources": [], "module_outputs": {}, "module_state": {}}

    def _save_tfstate(self, backend: Backend, name: str, doc: Dict[str, Any]) -> None:
        # executor/tfstate.py: only new or replaced entries are encoded; the root
        # "outputs" (<key>__<output>) are derived from module_outputs there
        with self._mu:
            doc["serial"] = int(doc.get("serial", 0)) + 1
            backend.write_tfstate(name, CODEC.dumps(name, doc))

    # --- planning -------------------------------------------------------------------------------------
    def plan(self, state: State) -> Dict[str, ModuleRun]:
        check_sources(state.modules())  # a document pinned to other modules is refused, as by Terraform
        runs: Dict[str, ModuleRun] = {}
        for key, cfg in state.modules().items():
            source = str(cfg.get("source", ""))
            info = module_from_source(source)
            if info is None or info.name not in SUPPORTED:
                raise ExecutorError(f"the direct executor does not implement module '{cfg.get('source')}' "
                                    f"(module.{key}); use `executor: terraform`")
            # the module's identity, not where its source lives, is part of the hash: the same
            # document applied from another install (another tk:: directory) re-applies nothing
            h, deps = fingerprint(dict(cfg, source=info.name))
            runs[key] = ModuleRun(key, info, cfg, deps, h)
        # An add-on module is applied after every host of its cluster (Terraform
        # would need an explicit depends_on): a failed node then blocks it
        # instead of leaving it waiting for a cluster that cannot turn active.
        hosts_of: Dict[str, Set[str]] = {}  # module key -> the host modules that reference it
        for k, h in runs.items():
            if h.info.kind == "host":
                for d in h.deps:
                    hosts_of.setdefault(d, set()).add(k)
        for r in runs.values():
            if r.info.kind == "addon":
                for d in [d for d in r.deps if runs.get(d) and runs[d].info.kind == "cluster"]:
                    r.deps |= hosts_of.get(d, set())
        for r in runs.values():
            missing = r.deps - set(runs)
            if missing:
                raise ExecutorError(f"module.{r.key} references unknown module(s): {', '.join(sorted(missing))}")
        return runs

    @staticmethod
    def supports(state: State) -> bool:
        for cfg in state.modules().values():
            info = module_from_source(str(cfg.get("source", "")))
            if info is None or info.name not in SUPPORTED:
                return False
        return bool(state.modules())

    def _event(self, kind: str, **data: Any) -> None:
        if self.on_event is not None:
            self.on_event(kind, data)

    # --- apply -------------------------------------------------------------------------------------------
    def apply(self, state: State, backend: Backend) -> None:
        report = self.apply_report(state, backend)
        if not report.ok:
            failed = [f"module.{k}: {r.error}" for k, r in report.runs.items() if r.status == "failed"]
            raise ExecutorError("apply failed: " + "; ".join(failed))

    def _bind_host_keys(self, backend: Backend, name: str):
        """The manager's pinned SSH host keys for this run's SSH connections (they stay bound:
        the readiness waiter's process gate reaches the same hosts)."""
        from ..parallel.hostkeys import HostKeys

        keys = HostKeys(backend, name)
        self.transport.bind_host_keys(keys)
        return keys

    def apply_report(self, state: State, backend: Backend) -> ApplyReport:
        keys = self._bind_host_keys(backend, state.name)
        try:
            self._load_trust(state, backend)
            return self._apply_report(state, backend)
        finally:
            keys.save()  # first-contact keys pinned by this run

    # --- the Rancher server's CA (rancher/trust.py) ----------------------------------------------
    def _load_trust(self, state: State, backend: Backend) -> None:
        """The manager's pinned CA for this run's clients.  ``rancher_ca_file`` re-pins (an
        operator's deliberate act).  A manager created before pinning existed, installed
        over SSH and already applied, is pinned now from its host (host-key-pinned SSH)."""
        from ..rancher import trust as rtrust

        self._trust_store = (backend, state.name)
        self.trust = rtrust.load(backend, state.name)
        if self.ca_file:
            self._pin(rtrust.from_file(self.ca_file))
            return
        mgr = state.module(MANAGER_KEY) or {}
        host = str(mgr.get("host", ""))
        applied = (self._load_tfstate(backend, state.name)["module_state"].get(MANAGER_KEY) or {}).get("status") == "ok"
        if self.trust is None and applied and host and not host.startswith("rancher+"):
            self._pin(self._read_host_ca(mgr))

    def _pin(self, trust: Any) -> None:
        from ..rancher import trust as rtrust

        self.trust = trust
        if self._trust_store is not None:
            rtrust.save(self._trust_store[0], self._trust_store[1], trust)

    def _read_host_ca(self, cfg: Dict[str, Any]) -> Any:
        """The CA bundle the manager host's install saved from ``https://127.0.0.1/cacerts``,
        read over the host-key-pinned SSH session -- fetched there from the loopback first
        when an older install never saved it (``trust.HOST_CA_READ``)."""
        from ..rancher.trust import HOST_CA_FILE, HOST_CA_READ, RancherTrust, normalize

        host = str(cfg.get("host", ""))
        ref = HostRef(host, cfg.get("ssh_user") or "ubuntu", cfg.get("key_path") or "~/.ssh/id_rsa",
                      cfg.get("bastion_host") or "")
        try:
            pem = self.transport.run_script(ref, HOST_CA_READ, timeout=120)
        except ExecutorError as exc:
            raise ExecutorError(f"{host}: cannot read the Rancher CA on the manager host ({exc}); give "
                                f"rancher_ca_file to pin it") from None
        if pem.strip() and "BEGIN CERTIFICATE" not in pem:
            raise ExecutorError(f"{host}: {HOST_CA_FILE} holds no PEM certificate")
        return RancherTrust(normalize(pem), f"ssh:{host}")

    def _apply_report(self, state: State, backend: Backend) -> ApplyReport:
        t0 = time.time()
        runs = self.plan(state)
        tf = self._load_tfstate(backend, state.name)
        outputs: Dict[str, Dict[str, str]] = {k: dict(v) for k, v in tf["module_outputs"].items() if k in runs}
        report = ApplyReport(runs)
        pending = set(runs)
        futures: Dict[cf.Future, str] = {}
        from ..parallel.fanout import shared_pool

        pool = shared_pool(f"tk-direct-{self.parallelism}", self.parallelism)
        tls_pool = self._prefetch_tls(runs, tf)
        rehashed = False
        with span("direct.apply", modules=len(runs)):
            while pending or futures:
                # to a fixed point: a module blocked (or skipped) in this pass can decide one
                # that sorted before it (a chain of dependents of a failed module), before
                # "nothing running and nothing startable" may be read as a cycle
                progress = True
                while progress:
                    progress = False
                    for key in sorted(pending):
                        run = runs[key]
                        if any(runs[d].status in ("failed", "blocked") for d in run.deps):
                            run.status, run.error = "blocked", "dependency failed"
                            pending.discard(key)
                            progress = True
                            continue
                        if all(runs[d].status in ("ok", "skipped") for d in run.deps):
                            pending.discard(key)
                            progress = True
                            prev = tf["module_state"].get(key)
                            if self._unchanged(run, prev) and key in outputs:
                                run.status = "skipped"
                                if prev.get("hash") != run.hash:  # a pre-r4 hash: stored in today's form
                                    tf["module_state"][key] = dict(prev, hash=run.hash)
                                    rehashed = True
                                continue
                            run.start = time.time()
                            run.prev_private = (prev or {}).get("private")
                            futures[pool.submit(self._apply_module, run, dict(outputs), state.name)] = key
                if not futures:
                    for key in pending:  # nothing running and nothing startable: a cycle
                        runs[key].status, runs[key].error = "failed", "dependency cycle"
                    pending.clear()
                    break
                done, _ = cf.wait(list(futures), return_when=cf.FIRST_COMPLETED)
                # one save per batch of finished modules (entries are replaced, never edited:
                # executor/tfstate.py caches their encoding by identity)
                keys_done: Dict[cf.Future, str] = {}
                for fut in done:
                    key = keys_done[fut] = futures.pop(fut)
                    run = runs[key]
                    run.end = time.time()
                    try:
                        outs, detail = fut.result()
                        run.status, run.detail = "ok", detail
                        outputs[key] = outs
                        tf["module_outputs"][key] = outs
                        tf["module_state"][key] = {"hash": run.hash, "status": "ok",
                                                   "applied_at": run.end, "seconds": run.end - run.start,
                                                   "source": run.cfg.get("source")}
                        if isinstance(detail, dict) and detail.get("private"):
                            tf["module_state"][key]["private"] = detail["private"]
                    except Exception as exc:  # noqa: BLE001 - recorded per module
                        run.status, run.error = "failed", str(exc)
                        tf["module_state"][key] = {"hash": run.hash, "status": "failed",
                                                   "error": str(exc), "applied_at": run.end}
                self._save_tfstate(backend, state.name, tf)
                for fut in done:
                    run = runs[keys_done[fut]]
                    self._event("module_done", key=run.key, status=run.status, seconds=run.end - run.start)
        if rehashed:
            self._save_tfstate(backend, state.name, tf)  # the upgraded hashes, whatever else ran
        if tls_pool is not None:
            tls_pool.shutdown(wait=False)  # an unused certificate (add-on blocked) finishes on its own
        report.wall = time.time() - t0
        self.last_report = report
        return report

    @staticmethod
    def _unchanged(run: ModuleRun, prev: Optional[Dict[str, Any]]) -> bool:
        """``prev`` (the module's tfstate entry) records a successful apply of this config.

        Since round 4 the hash covers the module's identity instead of its source string
        (``plan``).  A hash persisted before that covers the source the module was applied
        from, which the entry keeps: that form is accepted too (same module, same config), so
        the first apply after an upgrade or a ``migrate manager`` re-runs nothing -- above all
        no host bootstrap, whose full burn-in memtests a node that is in service."""
        if not prev or prev.get("status") != "ok":
            return False
        if prev.get("hash") == run.hash:
            return True
        src = prev.get("source")
        if not src:
            return False
        info = module_from_source(str(src))
        return info is not None and info.name == run.info.name and \
            fingerprint(dict(run.cfg, source=src))[0] == prev.get("hash")

    @staticmethod
    def _prefetch_tls(runs: Dict[str, ModuleRun], tf: Dict[str, Any]) -> Optional[cf.ThreadPoolExecutor]:
        """Start every add-on module's injector certificate when the walk starts.

        Terraform creates the module's ``tls_private_key`` / ``tls_*_cert`` resources as soon
        as the graph walk begins (they reference no other module), not after the hosts the
        module's manifests wait for; the three ``openssl`` runs (~27 ms) overlap the node
        bring-up the same way here.  Skipped for a module whose certificate is kept in the
        tfstate or that will be skipped as unchanged; an add-on whose injector switch is an
        interpolation makes its certificate itself (``_apply_addons``)."""
        from ..k8s import addons

        wanted = []
        for key, run in runs.items():
            if run.info.kind != "addon":
                continue
            prev = tf["module_state"].get(key) or {}
            if (prev.get("private") or {}).get("injector_tls"):
                continue
            if DirectExecutor._unchanged(run, prev):
                continue
            if addons.enabled("env", addons.module_cfg_defaults(run.cfg)):
                wanted.append(run)
        if not wanted:
            return None
        from ..k8s.tls import serving_cert

        pool = cf.ThreadPoolExecutor(max_workers=len(wanted), thread_name_prefix="tk-tls")
        for run in wanted:
            run.tls = pool.submit(serving_cert, addons.INJECTOR, "kube-system")
        return pool

    def _apply_module(self, run: ModuleRun, outputs: Dict[str, Dict[str, str]],
                      manager_name: str) -> Tuple[Dict[str, str], Any]:
        cfg = resolve(copy.deepcopy(run.cfg), outputs)
        kind = run.info.kind
        # what `terraform plan` would refuse about this call (unknown or missing arguments,
        # types, the variables' validation blocks), refused here too: the same document must
        # not apply through one executor and fail through the other
        problems = hcl.check_inputs(run.info.local_dir, cfg, cached=True)
        if problems:
            raise ExecutorError(f"module.{run.key} ({run.info.name}): " + "; ".join(problems[:3]))
        with span(f"module.{kind}", key=run.key, module=run.info.name):
            if kind == "manager":
                return self._apply_manager(cfg), None
            if kind == "cluster":
                return self._apply_cluster(cfg), None
            if kind == "host":
                for attempt in range(self.host_retries + 1):
                    try:
                        return self._apply_host(run.key, cfg, run.info.mi355x)
                    except ExecutorError as exc:
                        if attempt == self.host_retries:
                            raise
                        self._event("module_retry", key=run.key, attempt=attempt + 1, error=str(exc))
                        time.sleep(self.retry_backoff * (2 ** attempt))
            if kind == "addon":
                outs, private = self._apply_addons(cfg, run.prev_private, run.tls)
                return outs, {"private": private}
        raise ExecutorError(f"unsupported module kind {kind}")

    # --- manager ---------------------------------------------------------------------------------------
    def _apply_manager(self, cfg: Dict[str, Any]) -> Dict[str, str]:
        host = str(cfg.get("host", ""))
        password = cfg.get("rancher_admin_password", "")
        # the server's first-login password (CATTLE_BOOTSTRAP_PASSWORD): given for an adopted
        # server, else the value every install path of this framework starts the server with
        from ..rancher import bootstrap_secret
        from ..rancher.trust import RancherTrust, normalize

        if host.startswith("rancher+"):
            # an adopted server: its first-login password as given (rancher_bootstrap_password,
            # kept in the state backend), or none -- a server already bootstrapped, which takes
            # the admin password.  The legacy derivation of the admin password is tried only
            # when the operator opted in (rancher_legacy_bootstrap): never sent otherwise
            store = self._trust_store
            initial = cfg.get("rancher_bootstrap_password") or (bootstrap_secret.load(*store) if store else "")
            legacy = bool(store) and bootstrap_secret.legacy_allowed(*store)
            url = host[len("rancher+"):]
            if self.trust is None:
                if url.startswith("https://"):
                    # adopted over HTTPS without rancher_ca_file: a publicly trusted
                    # certificate, verified by the system store (a private CA must be given)
                    self._pin(RancherTrust("", "public"))
                else:  # plain http (the in-process fake; loopback development): no TLS to pin
                    self._pin(RancherTrust(normalize(self.rancher_factory(url).http.request(
                        "GET", "/cacerts").body.decode()), f"server:{url}"))
            client = self.rancher_factory(url)
            if initial:
                return client.bootstrap(password, url, initial, timeout=self.cluster_wait)
            try:  # no bootstrap password: the server must already take the admin password
                return client.bootstrap(password, url, password, timeout=self.cluster_wait)
            except HTTPError as exc:
                if exc.status != 401:
                    raise
                if not legacy:
                    raise ExecutorError(
                        f"the adopted Rancher server {url} does not accept the admin password and no "
                        f"rancher_bootstrap_password was given: set rancher_bootstrap_password (the server's "
                        f"CATTLE_BOOTSTRAP_PASSWORD), or rancher_legacy_bootstrap: true for a server an "
                        f"earlier version of triton-kubernetes started") from None
            return client.bootstrap(password, url, bootstrap_secret.legacy_password(str(cfg.get("name", "")),
                                                                                    password),
                                    timeout=self.cluster_wait)
        # a server this framework starts: a random first-login password kept in the state
        # backend (rancher/bootstrap_secret.py), never derived from the admin password
        initial = cfg.get("rancher_bootstrap_password") or (
            bootstrap_secret.ensure(*self._trust_store) if self._trust_store is not None else "")
        if not initial:
            raise ExecutorError("no state backend to keep the Rancher bootstrap password in")
        ref = HostRef(host, cfg.get("ssh_user") or "ubuntu", cfg.get("key_path") or "~/.ssh/id_rsa",
                      cfg.get("bastion_host") or "")
        from ..node.manager import manager_install_script, manager_setup_script

        with span("manager.install", host=host):
            self.transport.run_script(ref, manager_install_script(cfg, initial), timeout=self.node_timeout)
        if not self.ca_file:
            # the CA the server serves on the host itself, over the pinned SSH session
            self._pin(self._read_host_ca(cfg))
        url = f"https://{host}"
        if self.rancher_bootstrap == "remote":
            with span("manager.setup_remote", host=host):
                out = self.transport.run_script(ref, manager_setup_script(cfg, url, initial),
                                                timeout=self.node_timeout)
            data = json.loads(out.strip().splitlines()[-1])
            return {"rancher_url": url, "rancher_access_key": data["name"],
                    "rancher_secret_key": data["token"].split(":", 1)[-1]}
        client = self.rancher_factory(url)
        return client.bootstrap(password, url, initial, timeout=self.cluster_wait)

    # --- cluster ---------------------------------------------------------------------------------------
    def _apply_cluster(self, cfg: Dict[str, Any]) -> Dict[str, str]:
        client = self.rancher_factory(cfg["rancher_api_url"], cfg.get("rancher_access_key", ""),
                                      cfg.get("rancher_secret_key", ""))
        dist = cfg.get("k8s_distribution") or ""
        info = client.ensure_cluster(cfg["name"], cfg.get("k8s_version") or default_version(dist or DEFAULT_DISTRIBUTION),
                                     cfg.get("k8s_network_provider") or ("canal" if dist != "rke1" else "flannel"), cfg.get("k8s_registry", ""),
                                     cfg.get("k8s_registry_username", ""), cfg.get("k8s_registry_password", ""),
                                     distribution=dist)
        return info.outputs()

    # --- host ------------------------------------------------------------------------------------------------
    def _apply_host(self, key: str, cfg: Dict[str, Any], mi355x: bool) -> Tuple[Dict[str, str], Any]:
        ref = HostRef(str(cfg.get("host", "")), cfg.get("ssh_user") or "ubuntu", cfg.get("key_path") or "",
                      cfg.get("bastion_host") or "")
        plan = build_host_plan(cfg, cfg["rancher_api_url"], cfg["rancher_cluster_registration_token"],
                               cfg["rancher_cluster_ca_checksum"], mi355x=mi355x, sequential=ref.scheme != "agent")
        if mi355x and self.upload_tools and ref.scheme == "ssh":
            self._upload_tools(ref)
        result = self.transport.run_plan(ref, plan, timeout=self.node_timeout)
        if not result.get("ok"):
            raise ExecutorError(f"{plan.hostname}: {result.get('error')}")
        outs: Dict[str, str] = {}
        if mi355x:
            outs["gpu_node_labels"] = json.dumps(result.get("labels", {}), sort_keys=True)
        return outs, result

    def _upload_tools(self, ref: HostRef) -> List[str]:
        """The prebuilt gfx950 node tools, each with its source stamp (``node/tools.py``,
        the same stamp the Terraform host module and the machine image install): a tool the
        host already has from these sources is not uploaded again.  Returns what was sent."""
        from ..node import tools
        from ..ops.native import executable

        have: Dict[str, str] = {}
        for line in (self.transport.run_script(ref, tools.REMOTE_STAMPS.format(tools=TOOLS_DIR)) or "").splitlines():
            name, _, stamp = line.strip().partition(" ")
            have[name] = stamp.strip()
        sent = []
        for tool in tools.TOOL_SOURCES:
            want = tools.node_stamp(tool)
            if have.get(tool) == want:
                continue
            self.transport.put_file(ref, executable(tool), f"{TOOLS_DIR}/{tool}")
            self.transport.run_script(ref, f"sudo mkdir -p {TOOLS_DIR}/.stamps && echo {want} | "
                                           f"sudo tee {TOOLS_DIR}/.stamps/{tool}.sha256 >/dev/null\n")
            sent.append(tool)
        return sent

    # --- addons -------------------------------------------------------------------------------------------
    def _apply_addons(self, cfg: Dict[str, Any],
                      private: Optional[Dict[str, Any]] = None,
                      tls: Optional[cf.Future] = None) -> Tuple[Dict[str, str], Dict[str, Any]]:
        """The Terraform add-on module's objects, rendered from its own template files
        (``k8s/addons.py``), with the injector's serving certificate made by ``openssl``
        (the module uses the ``tls`` provider) -- while the nodes still bootstrap (``tls``:
        the one :meth:`_prefetch_tls` started with the walk).  The
        certificate is kept in the module's private tfstate entry and reused by later
        applies, as Terraform keeps its ``tls_*`` resources, so re-applying never leaves
        running webhook pods with a certificate the new ``caBundle`` rejects."""
        from ..k8s import addons
        from ..k8s.manifests import apply_manifests

        client = self.rancher_factory(cfg["rancher_api_url"], cfg.get("rancher_access_key", ""),
                                      cfg.get("rancher_secret_key", ""))
        cid = cfg["rancher_cluster_id"]
        cert = None
        if addons.enabled("env", addons.module_cfg_defaults(cfg)):
            from ..k8s.tls import ServingCert, serving_cert

            kept = (private or {}).get("injector_tls")
            if kept:
                cert = ServingCert(**kept)
            else:
                with span("addons.tls", cluster=cid, prefetched=tls is not None):
                    cert = tls.result() if tls is not None else serving_cert(addons.INJECTOR, "kube-system")
        manifests = addons.rendered_addons(cfg, cert)
        with span("addons.wait_active", cluster=cid):
            wait_until(lambda: client.cluster_state(cid) == "active", self.cluster_wait, f"cluster {cid} active")
        with span("addons.apply", cluster=cid):
            applied = apply_manifests(client, cid, manifests)
        kept = {"injector_tls": {"ca_pem": cert.ca_pem, "cert_pem": cert.cert_pem, "key_pem": cert.key_pem}} \
            if cert else {}
        return {"addons_applied": str(len(applied))}, kept

    # --- destroy / outputs ------------------------------------------------------------------------------
    def destroy(self, state: State, backend: Backend, targets: List[str]) -> None:
        keys = self._bind_host_keys(backend, state.name) if self.node_cleanup else None
        try:
            self._destroy(state, backend, targets)
        finally:
            if keys is not None:
                keys.save()

    @staticmethod
    def cleanup_wanted(cfg: Dict[str, Any]) -> bool:
        """A host module's ``node_cleanup`` (default on: bare metal outlives its cluster)."""
        v = cfg.get("node_cleanup", True)
        return v if isinstance(v, bool) else str(v).strip().lower() not in ("false", "0", "no", "off", "")

    def _cleanup_hosts(self, state: State, keys: List[str]) -> Dict[str, Dict[str, Any]]:
        """Take every destroyed host out of its cluster, all hosts at once (node/cleanup.py):
        SSH hosts run the cleanup script, agent hosts their fixed-argv ``/v1/cleanup``.  A
        failure is reported (``last_cleanup``), not raised: a dead host must not pin the
        document, and the host's join record refuses a later join until it is cleaned.  A
        changed SSH host key is raised (nothing is destroyed): that host is not dead."""
        from ..parallel.hostkeys import HostKeyChanged

        work = []
        for key in keys:
            cfg = state.module(key) or {}
            info = module_from_source(str(cfg.get("source", "")))
            if info is None or info.kind != "host" or not self.cleanup_wanted(cfg):
                continue
            ref = HostRef(str(cfg.get("host", "")), cfg.get("ssh_user") or "ubuntu", cfg.get("key_path") or "",
                          cfg.get("bastion_host") or "")
            work.append((key, str(cfg.get("hostname", key)), ref))
        if not work:
            return {}
        from ..parallel.fanout import shared_pool

        def one(item):
            key, hostname, ref = item
            t0 = time.time()
            with span("destroy.cleanup", host=hostname, transport=ref.scheme):
                try:
                    rep = self.transport.cleanup_host(ref, timeout=600)
                except HostKeyChanged:
                    raise  # not a dead host: an impostor or a reinstall -- the destroy stops here
                except Exception as exc:  # noqa: BLE001 - reported per host
                    rep = {"ok": False, "error": f"{type(exc).__name__}: {exc}", "actions": []}
            rep = dict(rep, hostname=hostname, seconds=round(time.time() - t0, 3))
            self._event("host_cleanup", key=key, **{k: rep.get(k) for k in ("hostname", "ok", "error")})
            return key, rep

        pool = shared_pool(f"tk-direct-{self.parallelism}", self.parallelism)
        return dict(pool.map(one, work))

    def _destroy(self, state: State, backend: Backend, targets: List[str]) -> None:
        tf = self._load_tfstate(backend, state.name)
        keys = [t[len("module."):] if t.startswith("module.") else t for t in targets] or list(state.modules())
        self.last_cleanup = self._cleanup_hosts(state, keys) if self.node_cleanup else {}
        for key in keys:
            tf["module_outputs"].pop(key, None)
            tf["module_state"].pop(key, None)
        self._save_tfstate(backend, state.name, tf)

    def outputs(self, state: State, backend: Backend, module_key: str) -> Dict[str, str]:
        return outputs_from_tfstate(backend.read_tfstate(state.name), module_key)
