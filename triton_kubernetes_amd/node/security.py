"""Node-agent credentials: per-manager CA, per-node tokens, image allow-list.

The node agent runs as root and starts ``docker run --privileged --net=host`` with the
image a plan names, so its API is a root code-execution surface.  The reference had no
agent: it delivered the bootstrap over SSH with the operator's key
(``terraform/modules/bare-metal-rancher-k8s-host/main.tf:24-42``).  The agent keeps an
equivalent bar:

* **TLS** -- every cluster manager has its own CA (:class:`AgentPKI`, stored in the state
  backend next to the manager's documents as ``agent-pki.json``, mode 0600 on the local
  backend).  Each node agent serves a certificate for its address signed by that CA,
  and the CLI verifies it against that CA only.  Plain HTTP is refused unless the agent
  runs with ``--insecure-local``, which binds loopback only;
* **per-node tokens** -- ``HMAC-SHA256(manager secret, "tk-agent-token" | address)``:
  a token read off one node (or its credentials directory) is useless on every other
  node, and tokens are never stored: the CLI derives them from the manager secret;
* **allow-list** -- the agent runs only the Rancher agent images its credentials list
  (:class:`AgentPolicy`, written by the manager at enrollment: the manager's pinned agent
  image, or a digest-pinned one), and joins an RKE2 cluster only through the
  ``system-agent-install.sh`` of a Rancher server the list names (the manager's URL);
  a plan naming any other image or server is refused (403) before any step runs.

``triton-kubernetes credentials node`` (``agent_address: <node>``) writes a node's credential
directory (``agent-token``, ``agent.crt``, ``agent.key``, ``ca.crt``,
``agent-policy.json``) for the node's ``/etc/triton-kubernetes/agent/``.
"""

import hashlib
import hmac
import ipaddress
import json
import os
import secrets
import ssl
import tempfile
import urllib.parse
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

from ..errors import TKError

PKI_BLOB = "agent-pki.json"
CRED_FILES = ("agent-token", "agent.crt", "agent.key", "ca.crt", "agent-policy.json")
DEFAULT_CRED_DIR = "/etc/triton-kubernetes/agent"


def agent_address(url_or_host: str) -> str:
    """The node address a token / certificate is bound to: the host part of an agent URL
    (``agent+https://10.0.0.5:7946`` -> ``10.0.0.5``), or the host given."""
    s = url_or_host[len("agent+"):] if url_or_host.startswith("agent+") else url_or_host
    if "://" in s:
        host = urllib.parse.urlsplit(s).hostname or ""
    else:
        host = s.rsplit(":", 1)[0] if s.count(":") == 1 else s
    return host.strip("[]").lower()


def is_loopback(host: str) -> bool:
    if host in ("localhost", ""):
        return True
    try:
        return ipaddress.ip_address(host.strip("[]")).is_loopback
    except ValueError:
        return False


def server_origin(url: str) -> str:
    """``https://Rancher.example:443/x`` -> ``https://rancher.example:443``: what a
    server allow-list entry and a plan's Rancher URL are compared by."""
    parts = urllib.parse.urlsplit(url.strip())
    if parts.scheme not in ("https", "http") or not parts.hostname:
        return ""
    port = parts.port or (443 if parts.scheme == "https" else 80)
    host = parts.hostname.lower()
    return f"{parts.scheme}://{'[' + host + ']' if ':' in host else host}:{port}"


@dataclass
class AgentPolicy:
    """What a node agent may run: the Rancher agent images it accepts (RKE1: ``docker run``)
    and the Rancher servers whose system-agent installer it may run (RKE2).  An image entry
    with a digest (``repo@sha256:...``) matches only that digest; a tag entry matches that
    tag.  A server entry matches by scheme, host and port.  ``loopback_servers`` (the
    default policy of an agent started without credentials: in-process test agents and
    ``--insecure-local`` development agents, which serve loopback only) also admits any
    Rancher server on a loopback address."""

    images: List[str] = field(default_factory=list)
    servers: List[str] = field(default_factory=list)
    loopback_servers: bool = False
    # the distribution the node was enrolled for (rke2 | rke1); empty: either (credentials
    # issued before the field existed, development agents)
    distributions: List[str] = field(default_factory=list)

    def allows(self, image: str) -> bool:
        return image in self.images

    def allows_distribution(self, dist: str) -> bool:
        return not self.distributions or dist in self.distributions

    def allows_server(self, url: str) -> bool:
        origin = server_origin(url)
        if not origin:
            return False
        if self.loopback_servers and is_loopback(urllib.parse.urlsplit(origin).hostname or ""):
            return True
        return origin in {server_origin(s) for s in self.servers}

    def to_json(self) -> Dict[str, Any]:
        doc: Dict[str, Any] = {"images": list(self.images), "servers": list(self.servers)}
        if self.loopback_servers:
            doc["loopback_servers"] = True
        if self.distributions:
            doc["distributions"] = list(self.distributions)
        return doc

    @classmethod
    def from_json(cls, doc: Dict[str, Any]) -> "AgentPolicy":
        imgs = doc.get("images") or []
        if not isinstance(imgs, list) or not all(isinstance(i, str) and i for i in imgs):
            raise TKError("agent policy: images must be a list of image references")
        servers = doc.get("servers") or []
        if not isinstance(servers, list) or not all(isinstance(u, str) and server_origin(u) for u in servers):
            raise TKError("agent policy: servers must be a list of http(s) Rancher server URLs")
        dists = doc.get("distributions") or []
        if not isinstance(dists, list) or not all(d in ("rke2", "rke1") for d in dists):
            raise TKError("agent policy: distributions must be a list of rke2 / rke1")
        return cls(images=list(imgs), servers=list(servers), loopback_servers=doc.get("loopback_servers") is True,
                   distributions=list(dists))


@dataclass
class NodeCredentials:
    address: str
    token: str
    cert_pem: str
    key_pem: str
    ca_pem: str
    policy: AgentPolicy

    def write(self, directory: str) -> List[str]:
        os.makedirs(directory, mode=0o700, exist_ok=True)
        files = {"agent-token": self.token + "\n", "agent.crt": self.cert_pem, "agent.key": self.key_pem,
                 "ca.crt": self.ca_pem, "agent-policy.json": json.dumps(self.policy.to_json(), indent=1) + "\n"}
        out = []
        for name, text in files.items():
            path = os.path.join(directory, name)
            fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
            with os.fdopen(fd, "w", encoding="utf-8") as fh:
                fh.write(text)
            out.append(path)
        return out


@dataclass
class AgentPKI:
    """One cluster manager's agent trust root: CA + the secret node tokens derive from."""

    ca_cert: str
    ca_key: str
    secret: bytes

    @classmethod
    def create(cls, manager: str) -> "AgentPKI":
        from ..k8s.tls import make_ca

        ca = make_ca(f"triton-kubernetes {manager} node agents")
        return cls(ca.cert_pem, ca.key_pem, secrets.token_bytes(32))

    def node_token(self, address: str) -> str:
        mac = hmac.new(self.secret, b"tk-agent-token\0" + agent_address(address).encode(), hashlib.sha256)
        return "tka1." + mac.hexdigest()

    def issue(self, address: str, images: List[str], extra_names: Optional[List[str]] = None,
              servers: Optional[List[str]] = None, distributions: Optional[List[str]] = None) -> NodeCredentials:
        from ..k8s.tls import CA, issue

        host = agent_address(address)
        names = [host] + [n for n in (extra_names or []) if n != host]
        cert = issue(CA(self.ca_cert, self.ca_key), host, names)
        return NodeCredentials(host, self.node_token(host), cert.cert_pem, cert.key_pem, self.ca_cert,
                               AgentPolicy(list(images), list(servers or []), distributions=list(distributions or [])))

    def client_context(self) -> ssl.SSLContext:
        """Verifies agents against this manager's CA only (not the system trust store)."""
        ctx = ssl.create_default_context(ssl.Purpose.SERVER_AUTH, cadata=self.ca_cert)
        ctx.check_hostname = True
        ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        return ctx

    def to_json(self) -> Dict[str, str]:
        return {"ca_cert": self.ca_cert, "ca_key": self.ca_key, "secret": self.secret.hex()}

    @classmethod
    def from_json(cls, doc: Dict[str, str]) -> "AgentPKI":
        return cls(doc["ca_cert"], doc["ca_key"], bytes.fromhex(doc["secret"]))


def load_pki(backend: Any, manager: str, create: bool = True) -> Optional[AgentPKI]:
    """The manager's agent PKI from the state backend (created on first use)."""
    try:
        raw = backend.read_blob(manager, PKI_BLOB)
    except NotImplementedError:
        raw = None
    if raw:
        return AgentPKI.from_json(json.loads(raw))
    if not create:
        return None
    pki = AgentPKI.create(manager)
    try:
        with backend.lock(manager):
            raw = backend.read_blob(manager, PKI_BLOB)  # another CLI may have won the race
            if raw:
                return AgentPKI.from_json(json.loads(raw))
            backend.write_blob(manager, PKI_BLOB, json.dumps(pki.to_json()).encode())
    except NotImplementedError:
        pass
    return pki


def server_context(cert_pem: str, key_pem: str) -> ssl.SSLContext:
    """TLS context of an agent serving ``cert_pem``."""
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.minimum_version = ssl.TLSVersion.TLSv1_2
    with tempfile.TemporaryDirectory(prefix="tk-agent-tls-") as d:
        cp, kp = os.path.join(d, "c.pem"), os.path.join(d, "k.pem")
        with open(cp, "w", encoding="utf-8") as fh:
            fh.write(cert_pem)
        fd = os.open(kp, os.O_WRONLY | os.O_CREAT, 0o600)
        with os.fdopen(fd, "w", encoding="utf-8") as fh:
            fh.write(key_pem)
        ctx.load_cert_chain(cp, kp)
    return ctx


def metrics_token(node_token: str) -> str:
    """The read-only scrape token of a node: derived from its agent token one way (HMAC), so
    the monitoring stack that holds it can read ``GET /metrics`` and ``GET /v1/health`` and
    nothing else -- it cannot post plans, shut the agent down or run the RCCL endpoints, and
    cannot recover the node's token.  The agent derives it from its own token; the CLI from
    the token it derives for the node (``AgentPKI.node_token``)."""
    return "tkm1." + hmac.new(node_token.encode(), b"tk-agent-metrics", hashlib.sha256).hexdigest()


def read_credentials(directory: str) -> Dict[str, Any]:
    """A node's credential directory -> ``{token, ssl_context, policy}``."""
    def rd(name: str) -> str:
        with open(os.path.join(directory, name), "r", encoding="utf-8") as fh:
            return fh.read()

    return {"token": rd("agent-token").strip(), "ssl_context": server_context(rd("agent.crt"), rd("agent.key")),
            "policy": AgentPolicy.from_json(json.loads(rd("agent-policy.json")))}


__all__ = ["AgentPKI", "AgentPolicy", "NodeCredentials", "load_pki", "server_context", "read_credentials", "metrics_token",
           "agent_address", "is_loopback", "server_origin", "PKI_BLOB", "DEFAULT_CRED_DIR"]
