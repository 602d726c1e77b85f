"""In-memory backend: the test double for ``backend/mocks/Backend.go``.

It doubles as the reference's testify mock: canned ``states`` / ``state`` return
values can be given up front, and every call is recorded in :attr:`calls`.
"""

import threading
from typing import Any, Dict, List, Optional, Tuple

from ..state import State
from .base import Backend


class MemoryBackend(Backend):
    kind = "memory"

    def __init__(self, states: Optional[Dict[str, Any]] = None, state_names: Optional[List[str]] = None):
        self._docs: Dict[str, bytes] = {}
        self._blobs: Dict[Tuple[str, str], bytes] = {}
        self._canned_names = list(state_names) if state_names is not None else None
        self.calls: List[Tuple[str, tuple]] = []
        self._mu = threading.Lock()
        for name, doc in (states or {}).items():
            st = doc if isinstance(doc, State) else State(name, doc)
            self._docs[name] = st.bytes()

    def state(self, name: str) -> State:
        self.calls.append(("State", (name,)))
        with self._mu:
            raw = self._docs.get(name)
        return State(name, raw if raw is not None else b"{}")

    def delete_state(self, name: str) -> None:
        self.calls.append(("DeleteState", (name,)))
        with self._mu:
            self._docs.pop(name, None)
            for key in [k for k in self._blobs if k[0] == name]:
                del self._blobs[key]
            if self._canned_names is not None and name in self._canned_names:
                self._canned_names.remove(name)

    def persist_state(self, state: State) -> None:
        self.calls.append(("PersistState", (state.name,)))
        with self._mu:
            self._docs[state.name] = state.bytes()
            if self._canned_names is not None and state.name not in self._canned_names:
                self._canned_names.append(state.name)

    def states(self) -> List[str]:
        self.calls.append(("States", ()))
        with self._mu:
            if self._canned_names is not None:
                return list(self._canned_names)
            return sorted(self._docs)

    def state_terraform_config(self, name: str) -> Tuple[str, Any]:
        return "terraform.backend.local", {"path": f"/memory/{name}/terraform.tfstate"}

    def read_blob(self, name: str, filename: str) -> Optional[bytes]:
        with self._mu:
            return self._blobs.get((name, filename))

    def write_blob(self, name: str, filename: str, data: bytes) -> None:
        with self._mu:
            self._blobs[(name, filename)] = bytes(data)
