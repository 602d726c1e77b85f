"""Local filesystem backend (reference ``backend/local/backend.go:1-132``).

Layout (byte-compatible with the reference)::

    ~/.triton-kubernetes/<name>/main.tf.json        CLI-owned
    ~/.triton-kubernetes/<name>/terraform.tfstate   executor-owned

``states()`` lists the sub-directories of the root.  The Terraform backend block
is ``terraform.backend.local = {"path": <abs tfstate path>}``.

Improvements: writes are atomic (temp file + ``rename``), and :meth:`lock`
takes an ``flock`` on ``<name>/.lock`` so two CLIs cannot interleave
read-modify-write cycles of the same manager.
"""

import contextlib
import errno
import fcntl
import os
import shutil
import tempfile
import threading
import time
from typing import Any, Iterator, List, Optional, Tuple

from ..errors import BackendError
from ..state import State
from .base import CONFIG_FILE, TFSTATE_FILE, Backend

DEFAULT_ROOT = "~/.triton-kubernetes"


def _atomic_write(path: str, data: bytes, mode: int = 0o644) -> None:
    directory = os.path.dirname(path)
    fd, tmp = tempfile.mkstemp(prefix=".tmp-", dir=directory)
    try:
        with os.fdopen(fd, "wb") as fh:
            fh.write(data)
        os.chmod(tmp, mode)
        os.replace(tmp, path)
    except BaseException:
        with contextlib.suppress(OSError):
            os.unlink(tmp)
        raise


class LocalBackend(Backend):
    kind = "local"

    def __init__(self, root: Optional[str] = None):
        root = root or os.environ.get("TRITON_KUBERNETES_HOME") or DEFAULT_ROOT
        self.root = os.path.abspath(os.path.expanduser(root))
        self._held = threading.local()
        try:
            os.makedirs(self.root, exist_ok=True)
        except OSError as exc:
            raise BackendError(f"mkdir {self.root}: {exc.strerror}") from exc

    def _dir(self, name: str) -> str:
        if not name or "/" in name or name in (".", ".."):
            raise BackendError(f"invalid cluster manager name '{name}'")
        return os.path.join(self.root, name)

    def state(self, name: str) -> State:
        path = os.path.join(self._dir(name), CONFIG_FILE)
        try:
            with open(path, "rb") as fh:
                return State(name, fh.read())
        except FileNotFoundError:
            return State(name, b"{}")

    def delete_state(self, name: str) -> None:
        shutil.rmtree(self._dir(name), ignore_errors=True)

    def persist_state(self, state: State) -> None:
        directory = self._dir(state.name)
        os.makedirs(directory, exist_ok=True)
        _atomic_write(os.path.join(directory, CONFIG_FILE), state.bytes())

    def states(self) -> List[str]:
        try:
            entries = sorted(os.listdir(self.root))
        except FileNotFoundError:
            return []
        return [e for e in entries if os.path.isdir(os.path.join(self.root, e)) and not e.startswith(".")]

    def state_terraform_config(self, name: str) -> Tuple[str, Any]:
        return "terraform.backend.local", {"path": os.path.join(self._dir(name), TFSTATE_FILE)}

    def read_blob(self, name: str, filename: str) -> Optional[bytes]:
        try:
            with open(os.path.join(self._dir(name), filename), "rb") as fh:
                return fh.read()
        except FileNotFoundError:
            return None

    def write_blob(self, name: str, filename: str, data: bytes) -> None:
        directory = self._dir(name)
        os.makedirs(directory, exist_ok=True)
        _atomic_write(os.path.join(directory, filename), data, 0o600)

    @contextlib.contextmanager
    def lock(self, name: str, timeout: float = 30.0) -> Iterator[None]:
        # Re-entrant within a thread (a workflow holds it around the executor, which may
        # take it again, e.g. to create the manager's node-agent PKI).  The lock lives next
        # to (not inside) the manager directory so that a lock taken before the first
        # persist does not make the name appear in states() (which lists directories).
        held = getattr(self._held, "names", None)
        if held is None:
            held = self._held.names = {}
        if held.get(name):
            held[name] += 1
            try:
                yield
            finally:
                held[name] -= 1
            return
        lock_path = os.path.join(self.root, f".{name}.lock")
        fd = os.open(lock_path, os.O_CREAT | os.O_RDWR, 0o600)
        deadline = time.monotonic() + timeout
        try:
            while True:
                try:
                    fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
                    break
                except OSError as exc:
                    if exc.errno not in (errno.EAGAIN, errno.EACCES):
                        raise
                    if time.monotonic() > deadline:
                        raise BackendError(f"timed out waiting for the state lock of '{name}' ({lock_path})")
                    time.sleep(0.05)
            held[name] = 1
            try:
                yield
            finally:
                held.pop(name, None)
        finally:
            with contextlib.suppress(OSError):
                fcntl.flock(fd, fcntl.LOCK_UN)
            os.close(fd)
