"""Manta object-store backend (reference ``backend/manta/backend.go:1-205``).

Layout: ``/stor/triton-kubernetes/<name>/{main.tf.json,terraform.tfstate}``.
Terraform backend block: ``terraform.backend.manta = {account, key_material,
key_id, path="/triton-kubernetes/<name>"}`` — kept in the persisted document for
format compatibility.  Terraform removed the ``manta`` backend in v1.3, so for
Terraform >= 1.3 the executor swaps it for a ``local`` backend in its work dir and
carries ``terraform.tfstate`` to and from this backend itself, under :meth:`lock`
(``executor/terraform.py``).

Deliberate fixes:

* Q9 — the reference passes the key *path* as ``key_material``.  Terraform's
  manta backend accepts either PEM text or a path in ``key_material``; we keep
  the path (byte-compatible documents) but expose ``embed_key_material`` to
  write the PEM instead;
* ``states()`` paginates instead of stopping at 100 entries;
* ``persist_state`` creates the manager directory first;
* :meth:`lock` implements a lock object ``<name>/.lock`` with an owner token and
  TTL (the reference's TODO at ``backend.go:32``), taken with Manta's conditional
  PUT — ``If-None-Match: *`` to create it, ``If-Match: <etag>`` to take over an
  expired one and to release it — so two writers can never both hold it;
* :meth:`delete_state` removes *every* object of the manager directory (state,
  tfstate, ``status.json``, backups, the lock) before the directory, as the
  reference removes each object it wrote before the directory
  (``backend.go:160-194``); Manta refuses to delete a non-empty directory.
"""

import contextlib
import json
import os
import threading
import time
import uuid
from typing import Any, Iterator, List, Optional, Tuple

from ..cloud.http import HTTPError
from ..cloud.triton import HTTPSignatureSigner, MantaClient
from ..errors import BackendError
from ..state import State
from .base import CONFIG_FILE, Backend

ROOT = "/stor/triton-kubernetes"
TF_ROOT = "/triton-kubernetes"


class MantaBackend(Backend):
    kind = "manta"

    def __init__(
        self,
        account: str,
        key_path: str,
        key_id: str,
        triton_url: str,
        manta_url: str,
        client: Optional[MantaClient] = None,
        embed_key_material: bool = False,
    ):
        self.account = account
        self.key_path = key_path
        self.key_id = key_id
        self.triton_url = triton_url
        self.manta_url = manta_url
        self.embed_key_material = embed_key_material
        if client is None:
            signer = HTTPSignatureSigner.from_path(account, key_path, key_id or None)
            client = MantaClient(manta_url, signer)
        self.client = client
        self._held = threading.local()  # per-thread {name: depth} of locks held
        self.client.put_directory(ROOT)

    def _p(self, name: str, filename: Optional[str] = None) -> str:
        base = f"{ROOT}/{name}"
        return f"{base}/{filename}" if filename else base

    def states(self) -> List[str]:
        entries = self.client.list_directory(ROOT)
        return [e["name"] for e in entries if e.get("type", "directory") == "directory"]

    def state(self, name: str) -> State:
        raw = self.client.get_object(self._p(name, CONFIG_FILE))
        return State(name, raw if raw is not None else b"{}")

    def _check_held(self, name: str) -> None:
        """Refuse a write under a lock this thread held but lost: the heartbeat found it taken
        over (it had expired, e.g. a suspended laptop), so another writer may have written
        since; writing now would overwrite its work."""
        lost = (getattr(self._held, "lost", None) or {}).get(name)
        if lost is not None and lost.is_set():
            raise BackendError(f"the Manta state lock of '{name}' was taken over by another writer while this "
                               "run held it; not writing, to keep that writer's changes. Re-run the command.")

    def persist_state(self, state: State) -> None:
        self._check_held(state.name)
        self.client.put_directory(self._p(state.name))
        self.client.put_object(self._p(state.name, CONFIG_FILE), state.bytes())

    def delete_state(self, name: str) -> None:
        base = self._p(name)
        try:
            entries = self.client.list_directory(base)
        except HTTPError as exc:
            if exc.status == 404:  # nothing persisted under this name
                return
            raise
        # the main document last: a half-finished delete still lists the manager
        order = sorted(entries, key=lambda e: (e.get("name") == CONFIG_FILE, e.get("name", "")))
        for e in order:
            path = f"{base}/{e['name']}"
            if e.get("type") == "directory":
                self._delete_tree(path)
            else:
                self.client.delete(path)
        self.client.delete(base)

    def _delete_tree(self, path: str) -> None:
        for e in self.client.list_directory(path):
            child = f"{path}/{e['name']}"
            if e.get("type") == "directory":
                self._delete_tree(child)
            else:
                self.client.delete(child)
        self.client.delete(path)

    def state_terraform_config(self, name: str) -> Tuple[str, Any]:
        material = self.key_path
        if self.embed_key_material:
            with open(os.path.expanduser(self.key_path), "r", encoding="utf-8") as fh:
                material = fh.read()
        return "terraform.backend.manta", {
            "account": self.account,
            "key_material": material,
            "key_id": self.key_id,
            "path": f"{TF_ROOT}/{name}",
        }

    def read_blob(self, name: str, filename: str) -> Optional[bytes]:
        return self.client.get_object(self._p(name, filename))

    def write_blob(self, name: str, filename: str, data: bytes) -> None:
        self._check_held(name)
        self.client.put_directory(self._p(name))
        self.client.put_object(self._p(name, filename), data)

    @contextlib.contextmanager
    def lock(self, name: str, timeout: float = 60.0, ttl: float = 900.0, poll: float = 0.25) -> Iterator[None]:
        """Exclusive lock on the manager's documents (``main.tf.json`` and, for Terraform
        >= 1.3, the CLI-carried ``terraform.tfstate``).

        Acquire: create ``.lock`` with ``If-None-Match: *`` (fails if any holder exists);
        a holder past its expiry is replaced with ``If-Match: <its etag>``, so of several
        writers racing for an expired lock exactly one wins.  While held, a heartbeat
        re-PUTs the lock (``If-Match`` our etag) every ``ttl/3`` so a Terraform apply longer
        than the TTL keeps it.  Release: delete with ``If-Match: <our etag>`` (a lock taken
        over after expiring is left alone).  Re-entrant within one thread: the workflow
        holds it around the executor, which takes it again around the tfstate round trip."""
        held = getattr(self._held, "names", None)
        if held is None:
            held = self._held.names = {}
        if name in held:
            held[name] += 1
            try:
                yield
            finally:
                held[name] -= 1
            return
        token = uuid.uuid4().hex
        path = self._p(name, ".lock")
        deadline = time.monotonic() + timeout
        self.client.put_directory(self._p(name))
        etag: Optional[str] = None
        while True:
            body = json.dumps({"token": token, "expires": time.time() + ttl}).encode()
            etag = self.client.put_object(path, body, if_none_match="*")
            if etag is not None:
                break
            raw, held_etag = self.client.get_object_etag(path)
            if raw is not None and held_etag:
                try:
                    holder = json.loads(raw)
                    expires = float(holder.get("expires", 0)) if isinstance(holder, dict) else 0.0
                except (TypeError, ValueError):
                    expires = 0.0  # a lock object that is not ours to read is stale
                if expires < time.time():
                    etag = self.client.put_object(path, body, if_match=held_etag)
                    if etag is not None:
                        break
            if time.monotonic() > deadline:
                raise BackendError(f"timed out waiting for the Manta state lock of '{name}'")
            time.sleep(poll)
        current = [etag]
        stop = threading.Event()
        lost = threading.Event()
        if getattr(self._held, "lost", None) is None:
            self._held.lost = {}
        self._held.lost[name] = lost

        def heartbeat() -> None:
            while not stop.wait(ttl / 3.0):
                refreshed = json.dumps({"token": token, "expires": time.time() + ttl}).encode()
                try:
                    new = self.client.put_object(path, refreshed, if_match=current[0])
                except Exception:  # transient: the next beat retries before the TTL runs out
                    continue
                if new is None:  # taken over: we lost it (an expired lock); every write refuses now
                    lost.set()
                    return
                current[0] = new

        beat = threading.Thread(target=heartbeat, name=f"manta-lock-{name}", daemon=True)
        beat.start()
        held[name] = 1
        try:
            yield
        finally:
            del held[name]
            self._held.lost.pop(name, None)
            stop.set()
            beat.join()
            if not lost.is_set():  # a lock taken over is the new holder's
                self.client.delete(path, if_match=current[0] or None)
