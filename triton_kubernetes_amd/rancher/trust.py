"""The Rancher server's CA, pinned per cluster manager: every HTTPS call to it is verified.

The reference talks to Rancher with ``curl --insecure`` and hashes ``/v3/settings/cacerts``
as read over that same unverified channel into the nodes' ``--ca-checksum``
(``terraform/modules/bare-metal-rancher-k8s/files/rancher_cluster.sh:19,82-88``).  An
on-path attacker then gets the admin API key, and the nodes pin *its* CA.

Here the CA bundle is read once, over a channel that is already trusted, when the manager
is created, and kept in the manager's state backend next to its pinned SSH host keys
(blob ``rancher-ca.json``):

* a manager this framework installs over SSH: the install script saves the server's
  ``/cacerts`` as read on the host itself (``https://127.0.0.1``, loopback) to
  ``~/rancher_cacerts.pem``; the CLI reads that file over the host-key-pinned SSH session
  (DirectExecutor) or the module's pinned SSH read (Terraform, output ``tk_rancher_ca_certs``);
* an operator-supplied bundle, ``rancher_ca_file`` (an adopted server, a custom CA, or a
  deliberate re-pin after a CA rotation);
* an empty bundle: the server has a publicly trusted certificate (Rancher's ``cacerts`` is
  empty then); the system trust store verifies it.

From then on the DirectExecutor, the readiness waiter, ``get``/``destroy``/``backup`` and the
Terraform modules' Rancher calls (``ensure_cluster.sh``, ``apply_addons.sh``) verify the
server's certificate against the pinned bundle only, and ``rancher_cluster_ca_checksum``
is the sha256 of the pinned bundle -- what ``/cacerts`` must then serve the nodes.  A
server that presents a certificate the pinned CA did not sign is refused before any
credential is sent.

Plain ``http://`` servers (the in-process fake used by tests and the CPU bench) carry no
TLS: their bundle is read from the server and recorded as such (``source`` ``server:``).
"""

import json
import ssl
from dataclasses import asdict, dataclass
from typing import Any, Optional

from ..errors import TKError

BLOB = "rancher-ca.json"
# where a manager install leaves the server's CA bundle as read on the host (loopback)
HOST_CA_FILE = "~/rancher_cacerts.pem"

# Run on the manager host over the pinned SSH session: the saved bundle; a manager installed
# before the bundle was saved there (an older version of this framework) has none, so it is
# read now from the server's own loopback -- what the install does -- and saved.  An empty
# output means the server's cacerts setting is empty (a publicly trusted certificate); a
# server that cannot be read fails (exit 3), never an empty bundle.
HOST_CA_READ = """f=~/rancher_cacerts.pem
if [ ! -e "$f" ]; then
  umask 077
  if ! curl -ksf https://127.0.0.1/cacerts > "$f.tmp"; then
    rm -f "$f.tmp"
    echo "no $f on this host and https://127.0.0.1/cacerts cannot be read: is the Rancher server running? (or give rancher_ca_file)" >&2
    exit 3
  fi
  mv "$f.tmp" "$f"
fi
cat "$f"
"""


@dataclass
class RancherTrust:
    pem: str = ""      # the bundle exactly as /cacerts serves it; "" = publicly trusted certificate
    source: str = ""   # ssh:<host> | file:<path> | server:<url> (plain http) | public

    @property
    def checksum(self) -> str:
        from .client import ca_checksum

        return ca_checksum(self.pem)

    def context(self) -> ssl.SSLContext:
        """Verify the server against the pinned bundle only (the system store when the
        certificate is publicly trusted).

        With a private CA pinned the chain is verified but the hostname is not: the CA is
        this one server's own (Rancher's generated CA, read over the host-key-pinned SSH
        session), so a chain to it already authenticates the server, and the certificate
        Rancher's docker install serves need not name the address the CLI connects to (its
        dynamic listener adds names only as requests arrive; the first bootstrap call
        precedes server-url).  The system store ('public') keeps hostname checks."""
        if self.pem.strip():
            ctx = ssl.create_default_context(cadata=self.pem)
            ctx.check_hostname = False  # verify_mode stays CERT_REQUIRED
            return ctx
        from ..cloud.http import _system_context

        return _system_context()  # built once per process: parsing the system store costs ~70 ms

    def describe(self) -> str:
        if not self.pem.strip():
            return "the system trust store (no private CA pinned: a publicly trusted certificate)"
        return f"the Rancher CA pinned for this cluster manager ({self.source or 'at create manager'})"

    def to_json(self) -> bytes:
        return json.dumps(asdict(self), sort_keys=True).encode()

    @classmethod
    def from_json(cls, raw: bytes) -> "RancherTrust":
        doc = json.loads(raw)
        return cls(str(doc.get("pem", "")), str(doc.get("source", "")))


def normalize(pem: str) -> str:
    """The bundle as Rancher serves it from ``/cacerts``: one trailing newline."""
    pem = pem.strip()
    return pem + "\n" if pem else ""


def load(backend: Any, manager: str) -> Optional[RancherTrust]:
    try:
        raw = backend.read_blob(manager, BLOB)
    except NotImplementedError:
        return None
    if not raw:
        return None
    try:
        return RancherTrust.from_json(raw)
    except ValueError as exc:
        raise TKError(f"the pinned Rancher CA of manager {manager} ({BLOB}) is unreadable: {exc}") from exc


def save(backend: Any, manager: str, trust: RancherTrust) -> None:
    try:
        backend.write_blob(manager, BLOB, trust.to_json())
    except NotImplementedError:
        pass


def from_file(path: str) -> RancherTrust:
    import os

    p = os.path.expanduser(path)
    try:
        with open(p, "r", encoding="utf-8") as fh:
            pem = fh.read()
    except OSError as exc:
        raise TKError(f"rancher_ca_file {path}: {exc}") from exc
    if pem.strip() and "BEGIN CERTIFICATE" not in pem:
        raise TKError(f"rancher_ca_file {path} holds no PEM certificate")
    if pem.strip():
        try:
            ssl.create_default_context(cadata=pem)
        except ssl.SSLError as exc:
            raise TKError(f"rancher_ca_file {path}: not a usable CA bundle: {exc}") from exc
    return RancherTrust(normalize(pem), f"file:{path}")


def client(backend: Any, manager: str, url: str, access_key: str = "", secret_key: str = ""):
    """A :class:`~.client.RancherClient` for manager ``manager``'s server, verified against
    its pinned CA (the system store when none was pinned: a manager created before pinning
    existed; the next apply pins it)."""
    from .client import RancherClient

    return RancherClient(url, access_key, secret_key, trust=load(backend, manager) if backend is not None else None)


__all__ = ["BLOB", "HOST_CA_FILE", "RancherTrust", "client", "from_file", "load", "normalize", "save"]
