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

For >= 0.12 the rendered document gains one root ``output`` per catalog output
of every module, so ``get manager|cluster`` keep working; the persisted
document is unchanged.  ``-parallelism`` is configurable (the reference leaves
it at Terraform's default of 10, which bounds node fan-out).
"""

import contextlib
import copy
import json
import os
import re
import shutil
import tempfile
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

from ..backend.base import Backend
from ..errors import ExecutorError
from ..state import State
from ..terraform.catalog import outputs_for_source
from ..utils.jsonenc import dumps_go
from .base import Executor, outputs_from_tfstate
from .shell import ShellOptions, capture_command, run_shell_command

_VERSION_RE = re.compile(r"Terraform v(\d+)\.(\d+)\.(\d+)")


def parse_version(text: str) -> Tuple[int, int, int]:
    m = _VERSION_RE.search(text)
    if not m:
        try:
            data = json.loads(text)
            return tuple(int(x) for x in data["terraform_version"].split(".")[:3])  # type: ignore[return-value]
        except (ValueError, KeyError, TypeError):
            raise ExecutorError(f"could not determine terraform version from {text!r}")
    return int(m.group(1)), int(m.group(2)), int(m.group(3))


def render_document(state: State, version: Tuple[int, int, int]) -> bytes:
    """The document Terraform sees (see module docstring)."""
    if version < (0, 12, 0):
        return state.bytes()
    doc = copy.deepcopy(state.doc)
    outputs = doc.setdefault("output", {})
    for key, mod in state.modules().items():
        for out in outputs_for_source(str(mod.get("source", ""))):
            outputs[f"{key}__{out}"] = {"value": f"${{module.{key}.{out}}}"}
    if not outputs:
        doc.pop("output")
    return dumps_go(doc)


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
    ):
        self.binary = binary
        self.parallelism = parallelism
        self.env = dict(env or {})
        self.timeout = timeout
        self._version = version
        self.keep_workdir = keep_workdir
        self.last_workdir: Optional[str] = None

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
    def workdir(self, state: State) -> Iterator[str]:
        tmp = tempfile.mkdtemp(prefix="triton-kubernetes-")
        self.last_workdir = tmp
        try:
            with open(os.path.join(tmp, "main.tf.json"), "wb") as fh:
                fh.write(render_document(state, self.version()))
            self._run(tmp, "init", "-force-copy", "-input=false")
            yield tmp
        finally:
            if not self.keep_workdir:
                shutil.rmtree(tmp, ignore_errors=True)

    # --- Executor API ---------------------------------------------------------------------
    def apply(self, state: State, backend: Backend) -> None:
        with self.workdir(state) as wd:
            args: List[str] = ["apply", "-auto-approve", "-input=false"]
            if self.parallelism:
                args.append(f"-parallelism={self.parallelism}")
            self._run(wd, *args)

    def destroy_flags(self) -> List[str]:
        return ["-auto-approve"] if self.version() >= (0, 15, 0) else ["-force"]

    def destroy(self, state: State, backend: Backend, targets: Sequence[str]) -> None:
        with self.workdir(state) as wd:
            args = ["destroy", *self.destroy_flags()]
            if self.parallelism:
                args.append(f"-parallelism={self.parallelism}")
            self._run(wd, *args, *[f"-target={t}" for t in targets])

    def outputs(self, state: State, backend: Backend, module_key: str) -> Dict[str, str]:
        with self.workdir(state) as wd:
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
            with self.workdir(state) as wd:
                self._run(wd, "output", "-module", module_key)
            return
        super().print_outputs(state, backend, module_key, out)
