"""Executor interface: turns a ``main.tf.json`` document into real resources.

The reference has exactly one executor, ``shell/run_terraform.go`` (terraform
init + apply / destroy in a temp dir).  We keep that (:class:`TerraformExecutor`)
and add :class:`DirectExecutor`, a native implementation of the bare-metal
module semantics that needs no Terraform binary and fans out to hosts in
parallel.
"""

import json
import threading
from typing import Any, Dict, List, Optional

from ..backend.base import Backend
from ..state import State


class Executor:
    name = "abstract"

    def apply(self, state: State, backend: Backend) -> None:
        raise NotImplementedError

    def destroy(self, state: State, backend: Backend, targets: List[str]) -> None:
        """Destroy ``targets`` (``module.<key>`` addresses) or everything if empty."""
        raise NotImplementedError

    def outputs(self, state: State, backend: Backend, module_key: str) -> Dict[str, str]:
        raise NotImplementedError

    def print_outputs(self, state: State, backend: Backend, module_key: str, out) -> None:
        outs = self.outputs(state, backend, module_key)
        for k in sorted(outs):
            if not k.startswith("tk_"):  # the CLI's own bookkeeping (pinned host keys)
                out.write(f"{k} = {outs[k]}\n")
        out.flush()


_PARSED: List[Any] = [None, None]  # [raw, document] of the last tfstate parsed here
_PARSED_MU = threading.Lock()


def _parsed(raw: bytes) -> Any:
    """``json.loads(raw)``, reusing the last result for the same bytes (the readiness
    waiter reads the manager's and the cluster's outputs from one tfstate).  The document
    is shared: callers only read it."""
    with _PARSED_MU:
        if _PARSED[0] == raw:
            return _PARSED[1]
    try:
        doc = json.loads(raw)
    except ValueError:
        return None
    with _PARSED_MU:
        _PARSED[0], _PARSED[1] = bytes(raw), doc
    return doc


def outputs_from_tfstate(raw: Optional[bytes], module_key: str) -> Dict[str, str]:
    """Module outputs from a tfstate document.

    Supports Terraform 0.11 (v3: ``modules[].path == ["root", key]``), the root
    outputs written for Terraform >= 0.12 (``<key>__<output>``), and the
    DirectExecutor's documents (v4-shaped with ``module_outputs``).
    """
    if not raw:
        return {}
    doc = _parsed(raw)
    if not isinstance(doc, dict):
        return {}
    result: Dict[str, str] = {}
    for mod in doc.get("modules", []) or []:  # v3
        if mod.get("path") == ["root", module_key]:
            for k, v in (mod.get("outputs") or {}).items():
                result[k] = v.get("value") if isinstance(v, dict) else v
    direct = (doc.get("module_outputs") or {}).get(module_key)
    if isinstance(direct, dict):
        result.update(direct)
    prefix = f"{module_key}__"
    for k, v in (doc.get("outputs") or {}).items():  # v4 root outputs
        if k.startswith(prefix):
            result[k[len(prefix):]] = v.get("value") if isinstance(v, dict) else v
    return {k: ("" if v is None else str(v)) for k, v in result.items()}
