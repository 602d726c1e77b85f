"""Pinned SSH host keys: trust on first use, refuse a changed key afterwards.

The reference connects to every host with host-key checking off (Terraform's
``connection`` blocks without ``host_key``, reference
``terraform/modules/bare-metal-rancher-k8s-host/main.tf:29-41``; its key read-back
``ssh`` in ``triton-rancher/main.tf:128-144``), so the Rancher admin API key is pulled
over a channel an attacker on the path could terminate.  Here every host a cluster
manager's operations reach over SSH has its key recorded the first time it is contacted,
in the manager's state backend next to ``agent-pki.json`` (blob ``known_hosts``, one
``known_hosts(5)`` line per key, so it travels with a shared Manta document), and every
later connection is checked against it:

* :class:`HostKeys` is that store.  ``ssh`` runs with ``UserKnownHostsFile`` = a private
  copy of it and ``StrictHostKeyChecking=accept-new``: an unknown host's key is added (the
  first contact), a known host's key must match -- OpenSSH refuses a mismatch before it
  authenticates, so no key or command is sent to an impostor.  :meth:`HostKeys.save`
  merges what ssh added back into the blob, under the backend lock;
* the DirectExecutor's :class:`~.transport.SSHTransport` uses it for every plan, script
  and file copy (``bind_host_keys``), and the bastion hop too (``ProxyCommand`` with the
  same options: ``-J`` would not pass them on);
* the Terraform executor renders its content into the root variable ``tk_known_hosts``
  for the modules' SSH programs (``read_api_key.sh``, ``read_gpu_labels.sh``), which
  connect the same way and report the keys they learned (module output
  ``ssh_known_hosts``, merged back after the apply), and into each bare-metal module's
  ``host_key`` / ``bastion_host_key``, so Terraform's own provisioner connections to a
  pinned host are checked too.

A changed key raises :class:`HostKeyChanged` naming the host; ``triton-kubernetes forget
host-key`` (``host`` setting) drops a reinstalled machine's entry.
"""

import os
import shutil
import tempfile
import threading
import weakref
from typing import Dict, Iterable, List

from ..errors import ExecutorError

BLOB = "known_hosts"

# Host key algorithms in the order Go's x/crypto/ssh (Terraform's provisioner connections)
# prefers them: ECDSA, then RSA, then Ed25519 last -- OpenSSH's own default puts Ed25519
# first.  Every ssh this framework runs offers this order, so the key it pins on first
# contact is of the type Terraform will be shown later; UpdateHostKeys=yes pins the host's
# other keys too (OpenSSH's hostkeys extension, after the first key was verified), and the
# Terraform render picks the pinned key Go would negotiate (``preferred_key``).
GO_HOSTKEY_ALGORITHMS = ("ecdsa-sha2-nistp256", "ecdsa-sha2-nistp384", "ecdsa-sha2-nistp521",
                         "rsa-sha2-512", "rsa-sha2-256", "ssh-ed25519")
# the key type (known_hosts field 2) each algorithm verifies
_KEY_TYPE = {"rsa-sha2-512": "ssh-rsa", "rsa-sha2-256": "ssh-rsa"}
NEGOTIATION_OPTS = ["-o", "HostKeyAlgorithms=" + ",".join(GO_HOSTKEY_ALGORITHMS), "-o", "UpdateHostKeys=yes"]


def preferred_key(keys: List[str]) -> str:
    """The pinned key (``"<type> <base64>"``) of the type Go's client negotiates first
    among ``keys`` (all keys pinned for one host); ``""`` when none."""
    rank = {}
    for i, alg in enumerate(GO_HOSTKEY_ALGORITHMS):
        rank.setdefault(_KEY_TYPE.get(alg, alg), i)
    ranked = sorted(keys, key=lambda k: rank.get(k.split(" ", 1)[0], len(rank)))
    return ranked[0] if ranked else ""
# what OpenSSH prints when a pinned key does not match
MISMATCH_MARKERS = ("Host key verification failed", "REMOTE HOST IDENTIFICATION HAS CHANGED",
                    "host key mismatch")


class HostKeyChanged(ExecutorError):
    """A host presented a key other than the one pinned for it."""


def parse_lines(text: str) -> List[str]:
    """Non-empty, non-comment known_hosts lines, normalised to single spaces."""
    out = []
    for line in text.splitlines():
        line = line.strip()
        if line and not line.startswith("#"):
            out.append(" ".join(line.split()))
    return out


def merge(old: str, new: str) -> str:
    """``old`` plus the lines of ``new`` it lacks (order kept; nothing is ever replaced:
    a changed key is refused by ssh, never merged)."""
    lines = parse_lines(old)
    have = set(lines)
    for line in parse_lines(new):
        if line not in have:
            lines.append(line)
            have.add(line)
    return "".join(line + "\n" for line in lines)


def _hosts_of(field: str) -> List[str]:
    """The addresses a known_hosts host field names: ``a,b`` and OpenSSH's ``[a]:port`` form
    (written when an ``ssh_config`` Port is not 22)."""
    out = []
    for name in field.split(","):
        if name.startswith("[") and "]:" in name:
            name = name[1:name.index("]:")]
        out.append(name)
    return out


def keys_for(text: str, address: str) -> List[str]:
    """``["<type> <base64>", ...]`` pinned for ``address`` (Terraform's ``host_key`` takes
    one of these)."""
    out = []
    for line in parse_lines(text):
        parts = line.split(" ")
        if len(parts) < 3 or parts[0].startswith("@"):
            continue
        if address in _hosts_of(parts[0]):
            out.append(f"{parts[1]} {parts[2]}")
    return out


def mismatch_error(address: str, detail: str, manager: str = "") -> HostKeyChanged:
    where = f" for cluster manager \"{manager}\"" if manager else ""
    return HostKeyChanged(
        f"the SSH host key of {address} does not match the key pinned{where} when it was first contacted; "
        f"refusing to connect (the Rancher API key and bootstrap scripts would go to whoever answers). If the "
        f"machine was reinstalled, run `triton-kubernetes forget host-key` with host={address} and retry. "
        f"ssh said: {detail.strip()[-300:]}")


def looks_like_mismatch(stderr: str) -> bool:
    return any(m in stderr for m in MISMATCH_MARKERS)


class HostKeys:
    """One cluster manager's pinned host keys (see module docstring)."""

    def __init__(self, backend, manager: str):
        self.backend = backend
        self.manager = manager
        self._dir = tempfile.mkdtemp(prefix="tk-known-hosts-")
        self.path = os.path.join(self._dir, "known_hosts")
        self._mu = threading.Lock()
        self._stored = ""
        weakref.finalize(self, shutil.rmtree, self._dir, True)
        self.reload()

    def _read_blob(self) -> str:
        try:
            raw = self.backend.read_blob(self.manager, BLOB)
        except NotImplementedError:
            raw = None
        return raw.decode() if raw else ""

    def reload(self) -> None:
        with self._mu:
            self._stored = self._read_blob()
            fd = os.open(self.path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
            with os.fdopen(fd, "w") as fh:
                fh.write(self._stored)

    def text(self) -> str:
        """What ssh works with now: the pinned keys plus any it added in this run."""
        with self._mu:
            try:
                with open(self.path, "r", encoding="utf-8") as fh:
                    return fh.read()
            except FileNotFoundError:
                return self._stored

    def keys_for(self, address: str) -> List[str]:
        return keys_for(self.text(), address)

    def add(self, text: str) -> None:
        """Lines learned elsewhere (a Terraform program's ``ssh_known_hosts`` output)."""
        with self._mu:
            with open(self.path, "r+", encoding="utf-8") as fh:
                merged = merge(fh.read(), text)
                fh.seek(0)
                fh.write(merged)
                fh.truncate()

    def save(self) -> bool:
        """Merge the keys ssh pinned in this run into the backend blob (under the manager's
        lock: another CLI may have pinned other hosts meanwhile).  True when it changed."""
        current = self.text()
        if parse_lines(current) == parse_lines(self._stored):
            return False
        try:
            with self.backend.lock(self.manager):
                merged = merge(self._read_blob(), current)
                self.backend.write_blob(self.manager, BLOB, merged.encode())
        except NotImplementedError:
            return False
        with self._mu:
            self._stored = merged
            with open(self.path, "w", encoding="utf-8") as fh:  # and what another CLI pinned meanwhile
                fh.write(merged)
        return True

    def forget(self, address: str) -> int:
        """Drop every pinned key of ``address`` from the backend blob; returns how many."""
        with self.backend.lock(self.manager):
            lines = parse_lines(self._read_blob())
            keep = [ln for ln in lines if address not in _hosts_of(ln.split(" ")[0])]
            self.backend.write_blob(self.manager, BLOB, "".join(ln + "\n" for ln in keep).encode())
        self.reload()
        return len(lines) - len(keep)

    def ssh_options(self) -> List[str]:
        return ["-o", f"UserKnownHostsFile={self.path}", "-o", "StrictHostKeyChecking=accept-new",
                "-o", "HashKnownHosts=no", "-o", "GlobalKnownHostsFile=/dev/null", *NEGOTIATION_OPTS]

    def close(self) -> None:
        shutil.rmtree(self._dir, ignore_errors=True)

    def __enter__(self) -> "HostKeys":
        return self

    def __exit__(self, *exc) -> None:
        self.close()


def pinned_map(text: str, addresses: Iterable[str]) -> Dict[str, str]:
    """``{address: "<type> <base64>"}`` of the addresses with a pinned key (the one Go's
    client negotiates: ``preferred_key``)."""
    out = {}
    for a in addresses:
        k = keys_for(text, a)
        if k:
            out[a] = preferred_key(k)
    return out


__all__ = ["HostKeys", "HostKeyChanged", "BLOB", "merge", "keys_for", "mismatch_error", "looks_like_mismatch",
           "pinned_map", "preferred_key", "GO_HOSTKEY_ALGORITHMS", "NEGOTIATION_OPTS"]
