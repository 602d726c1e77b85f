"""State backend interface (reference ``backend/backend.go:7-27``).

A backend stores, per cluster manager ``<name>``:

* ``main.tf.json``      — the CLI-owned desired state (:class:`~..state.State`);
* ``terraform.tfstate`` — the executor-owned actual state (Terraform, or our
  :class:`~..executor.direct.DirectExecutor` which writes a tfstate-compatible
  document so ``get manager`` works without Terraform).

Additions over the reference: an advisory per-manager lock
around read-modify-write of ``main.tf.json`` (the reference has none: last
writer wins), and blob access for the tfstate.
"""

import contextlib
from typing import Any, Iterator, List, Optional, Tuple

from ..state import State

CONFIG_FILE = "main.tf.json"
TFSTATE_FILE = "terraform.tfstate"


class Backend:
    kind = "abstract"

    def state(self, name: str) -> State:
        """The named state; an empty ``{}`` document if it does not exist."""
        raise NotImplementedError

    def delete_state(self, name: str) -> None:
        raise NotImplementedError

    def persist_state(self, state: State) -> None:
        raise NotImplementedError

    def states(self) -> List[str]:
        raise NotImplementedError

    def state_terraform_config(self, name: str) -> Tuple[str, Any]:
        """``(json path, object)`` of the Terraform backend block for ``name``."""
        raise NotImplementedError

    # --- extensions -----------------------------------------------------------------
    def read_blob(self, name: str, filename: str) -> Optional[bytes]:
        raise NotImplementedError

    def write_blob(self, name: str, filename: str, data: bytes) -> None:
        raise NotImplementedError

    def read_tfstate(self, name: str) -> Optional[bytes]:
        return self.read_blob(name, TFSTATE_FILE)

    def write_tfstate(self, name: str, data: bytes) -> None:
        self.write_blob(name, TFSTATE_FILE, data)

    @contextlib.contextmanager
    def lock(self, name: str, timeout: float = 30.0) -> Iterator[None]:
        """Advisory lock on the manager's documents (no-op by default)."""
        yield
