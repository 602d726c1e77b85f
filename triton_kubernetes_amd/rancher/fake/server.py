"""The fake Rancher server: shared state, HTTP plumbing, routing and the RKE simulation.

Each API the server answers lives in its own module, so each contract can be reviewed
(and is tested, positive and negative) on its own:

=====================  =====================================================================
``v3.py``              Norman ``/v3``: bootstrap, RKE1 clusters, tokens, nodes, registration
``provisioning.py``    Steve ``/v1``: RKE2 custom clusters, Secrets, the node installer
``k8s.py``             ``/k8s/clusters/<id>``: the downstream API servers and kubelets
``admission.py``       mutating webhooks and Pod Security Admission on Pod creates
=====================  =====================================================================

This module holds what they share: :class:`State` (one lock; every index a request
needs, so a request costs the same however many clusters the server holds), the HTTP
handler, the router (unauthenticated endpoints first, then the token check, then each
API in turn) and the simulation of what the real server's controllers do after agents
register:

* a cluster turns ``active`` ``rke_seconds`` after it has at least one etcd, one
  controlplane and one worker node; its nodes turn ``active`` (kubelet ``Ready``)
  ``node_ready_seconds`` after that;
* a Kubernetes release change (:meth:`FakeRancher._upgrade`, from the v3 and the
  provisioning API) must be offered by the server and not lower than the running
  release; the cluster reads ``upgrading`` for ``upgrade_seconds`` and the kubelets then
  report the new release.

Everything is in memory and thread-safe; it serves plain HTTP on 127.0.0.1, or HTTPS with
its own CA (``tls=True``; ``rotate_certificate`` switches CA, for the pinning tests).
"""

import base64
import http.server
import json
import secrets
import socket
import threading
import time
import urllib.parse
from typing import Any, Dict, List, Optional, Sequence, Set, Tuple

from ...utils.httpserver import Server as HTTPServer
from ...versions import (DEFAULT_K8S_VERSION, K8S_VERSIONS, PASSWORD_MIN_LENGTH, RANCHER_VERSION, RKE2_VERSIONS,
                         bootstrap_password, running_version)
from .admission import PSA_LEVELS
from .k8s import K8sCoreApi
from .provisioning import ProvisioningApi
from .v3 import V3Api, version_key

FAKE_CACERTS = "-----BEGIN CERTIFICATE-----\nMIIFAKECERTIFICATEFORTESTS\n-----END CERTIFICATE-----"
Reply = Tuple[int, Any]


class State:
    def __init__(self, rke_seconds: float, node_ready_seconds: float, admin_password: str,
                 k8s_versions: Sequence[str], rke2_versions: Sequence[str] = ()):
        self.mu = threading.RLock()
        self.cond = threading.Condition(self.mu)
        self.admin_password = admin_password
        self.tokens: Dict[str, str] = {}  # name -> secret
        # the settings this server has (GET/PUT of any other -> 404)
        self.settings: Dict[str, str] = {"cacerts": FAKE_CACERTS, "server-url": "",
                                         "server-version": RANCHER_VERSION,
                                         "k8s-versions-current": ",".join(k8s_versions),
                                         "k8s-version": DEFAULT_K8S_VERSION,
                                         "password-min-length": str(PASSWORD_MIN_LENGTH),
                                         "telemetry-opt": "", "first-login": "true"}
        self.clusters: Dict[str, Dict[str, Any]] = {}
        self.rke2_versions: List[str] = list(rke2_versions)
        self.v2_clusters: Dict[str, Dict[str, Any]] = {}  # "<namespace>/<name>" -> provisioning object
        self.secrets: Dict[str, Dict[str, Any]] = {}  # "<namespace>/<name>" -> Secret (management cluster)
        self.reg_tokens: Dict[str, Dict[str, Any]] = {}  # token -> {clusterId, id}
        self.nodes: Dict[str, Dict[str, Any]] = {}
        self.cluster_nodes: Dict[str, Dict[str, Dict[str, Any]]] = {}  # cluster id -> node id -> node
        self.unsettled: Set[str] = set()  # clusters not yet active, or with a node not yet active
        self.objects: Dict[str, Dict[str, Any]] = {}  # "<cluster>|<path>|<name>" -> object
        self.cluster_objects: Dict[str, Dict[str, None]] = {}  # cluster id -> its object keys, in creation order
        self.object_times: Dict[str, float] = {}  # object key -> when it was created
        self.rv_seq = 0  # resourceVersion source of the stored objects
        self.rke_seconds = rke_seconds
        self.node_ready_seconds = node_ready_seconds
        self.device_plugin_seconds = 0.0
        self.upgrade_seconds = 0.0  # a rolling Kubernetes upgrade's duration
        self.upgrades = 0
        self.evictions_refused = 0
        self.requests = 0
        self.log: List[Tuple[str, str]] = []


class FakeRancher(V3Api, ProvisioningApi, K8sCoreApi):
    """In-process fake Rancher 2.x server (the Rancher API fake SURVEY.md §4 calls for)."""

    def __init__(self, rke_seconds: float = 0.0, node_ready_seconds: float = 0.0,
                 bootstrap_password: Optional[str] = None, host: str = "127.0.0.1", port: int = 0,
                 k8s_versions: Optional[Sequence[str]] = None, async_registration_tokens: bool = True,
                 default_pod_security: str = "privileged", rke2_versions: Optional[Sequence[str]] = None,
                 device_plugin_seconds: float = 0.0, tls: bool = False,
                 tls_names: Optional[Sequence[str]] = None):
        if default_pod_security not in PSA_LEVELS:
            raise ValueError(f"default_pod_security must be one of {', '.join(PSA_LEVELS)}")
        # a server started without CATTLE_BOOTSTRAP_PASSWORD has a random one nobody knows
        pw = bootstrap_password if bootstrap_password is not None else secrets.token_hex(16)
        self.state = State(rke_seconds, node_ready_seconds, pw,
                           list(k8s_versions) if k8s_versions is not None else [v for _, v in K8S_VERSIONS],
                           list(rke2_versions) if rke2_versions is not None else [v for _, v in RKE2_VERSIONS])
        self.state.device_plugin_seconds = device_plugin_seconds
        self.bootstrap_password = pw
        # the request bodies the server received, the latest 20000 (the tests check what was
        # sent to it; bounded for long runs such as the bench)
        import collections

        self.request_bodies: "collections.deque[bytes]" = collections.deque(maxlen=20000)
        # "<service>.<namespace>" -> "https://127.0.0.1:<port>" (where an in-cluster
        # webhook service of a test really listens)
        self.service_endpoints: Dict[str, str] = {}
        self.async_registration_tokens = async_registration_tokens
        # Pod Security level of namespaces without an enforce label (the API server's
        # AdmissionConfiguration default; Kubernetes' own default is privileged)
        self.default_pod_security = default_pod_security
        # tls: HTTPS with a certificate for 127.0.0.1 from the server's own CA, which
        # /cacerts and the cacerts setting serve (what a Rancher install with its generated
        # CA does); rotate_certificate() switches to another CA (an impostor, or a rotation)
        self._tls_ctx = None
        # the names the serving certificate carries (default: the loopback address this fake
        # listens on); others model a certificate that does not name the address connected to
        self.tls_names = list(tls_names) if tls_names else ["127.0.0.1", "localhost"]
        if tls:
            self._tls_ctx = self._new_certificate()
        self._server = HTTPServer((host, port), self._handler())
        self._server.daemon_threads = True
        if self._tls_ctx is not None:
            self._server.socket = self._tls_ctx.wrap_socket(self._server.socket, server_side=True,
                                                            do_handshake_on_connect=False)
        self._thread: Optional[threading.Thread] = None

    def _new_certificate(self, ctx: Any = None) -> Any:
        from ...k8s.tls import issue, make_ca

        ca = make_ca(f"fake-rancher-ca-{secrets.token_hex(3)}")
        cert = issue(ca, self.tls_names[0], self.tls_names)
        if ctx is None:
            from ...node.security import server_context

            ctx = server_context(cert.cert_pem, cert.key_pem)
        else:  # later handshakes of the same listening socket present the new certificate
            import os
            import tempfile

            with tempfile.TemporaryDirectory(prefix="tk-fake-rancher-") as d:
                cp, kp = os.path.join(d, "c.pem"), os.path.join(d, "k.pem")
                with open(cp, "w", encoding="utf-8") as fh:
                    fh.write(cert.cert_pem)
                with open(kp, "w", encoding="utf-8") as fh:
                    fh.write(cert.key_pem)
                ctx.load_cert_chain(cp, kp)
        with self.state.mu:
            self.state.settings["cacerts"] = ca.cert_pem
        self.ca_pem = ca.cert_pem
        return ctx

    def rotate_certificate(self) -> str:
        """Serve a certificate from a new CA from now on (and that CA from /cacerts);
        returns the new CA's PEM."""
        if self._tls_ctx is None:
            raise ValueError("this fake serves plain HTTP")
        self._new_certificate(self._tls_ctx)
        return self.ca_pem

    @classmethod
    def for_manager(cls, name: str, admin_password: str, **kw: Any) -> "FakeRancher":
        """A server started the way earlier versions of this framework started one for manager
        ``name`` (the derived first-login password, ``rancher/bootstrap_secret.py``)."""
        return cls(bootstrap_password=bootstrap_password(name, admin_password), **kw)

    @property
    def url(self) -> str:
        host, port = self._server.server_address[:2]
        return f"{'https' if self._tls_ctx is not None else 'http'}://{host}:{port}"

    def start(self) -> "FakeRancher":
        self._thread = threading.Thread(target=self._server.serve_forever, name="fake-rancher", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._server.shutdown()
        self._server.server_close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # --- simulation -----------------------------------------------------------------------
    def _refresh(self) -> None:
        """Advance the simulated RKE provisioning of the clusters still settling."""
        st = self.state
        now = time.time()
        with st.mu:
            for cid in list(st.unsettled):
                c = st.clusters.get(cid)
                if c is None:
                    st.unsettled.discard(cid)
                    continue
                nodes = st.cluster_nodes.get(cid, {}).values()
                if c["state"] != "active":
                    roles = {"etcd": False, "controlplane": False, "worker": False}
                    for n in nodes:
                        for r in roles:
                            roles[r] = roles[r] or n["roles"].get(r, False)
                    if all(roles.values()):
                        if c.get("ready_at") is None:
                            c["ready_at"] = now + st.rke_seconds
                        if now >= c["ready_at"]:
                            c["state"] = "active"
                            c["transitioning"] = "no"
                            st.cond.notify_all()
                if c["state"] == "active":
                    settled = True
                    for n in nodes:
                        if n["state"] != "active":
                            if n.get("ready_at") is None:
                                n["ready_at"] = max(now, c["ready_at"]) + st.node_ready_seconds
                            if now >= n["ready_at"]:
                                n["state"] = "active"
                            else:
                                settled = False
                    if settled:
                        st.unsettled.discard(cid)

    def _upgrade(self, cid: str, body: Any, v2: Optional[Dict[str, Any]] = None) -> Reply:
        """A cluster's new Kubernetes release (caller holds the lock): offered by the server,
        not lower than the running one; the cluster reads ``upgrading`` until the (simulated)
        rolling upgrade is over, and the kubelets report the new release."""
        st = self.state
        c = st.clusters.get(cid)
        if c is None:
            return 404, {"type": "error", "code": "NotFound", "message": f"cluster {cid!r} not found"}
        spec = (body or {}).get("spec") if v2 is not None else (body or {}).get("rancherKubernetesEngineConfig")
        version = (spec or {}).get("kubernetesVersion", "")
        offered = st.rke2_versions if v2 is not None else [v for v in st.settings["k8s-versions-current"].split(",") if v]
        if version not in offered:
            return 422, {"type": "error", "code": "Invalid", "fieldName": "kubernetesVersion",
                         "message": f"{version} is not a supported Kubernetes version"}
        current = (c.get("version") or {}).get("gitVersion", "")
        if version_key(version) < version_key(current):
            return 422, {"type": "error", "code": "Invalid", "message": f"cannot downgrade {current} to {version}"}
        running = version if v2 is not None else running_version(version, "rke1")
        if running != current:
            c["version"] = {"gitVersion": running}
            c["state"], c["transitioning"] = "upgrading", "yes"
            c["ready_at"] = time.time() + st.upgrade_seconds
            st.unsettled.add(cid)
            st.upgrades += 1
        if v2 is not None:
            v2["spec"]["kubernetesVersion"] = version
            return 200, json.loads(json.dumps(v2))
        c.setdefault("rancherKubernetesEngineConfig", {})["kubernetesVersion"] = version
        return 200, dict(c)

    # --- HTTP ------------------------------------------------------------------------------
    def _route(self, method: str, path: str, query: Dict[str, List[str]], body: Any, h) -> Reply:
        if path == "/ping":
            return 200, b"pong"
        for public in (lambda: self._route_v3_public(method, path, query, body, h.headers),
                       lambda: self._route_provisioning_public(method, path)):
            out = public()
            if out is not None:
                return out
        if not h._authed():
            return 401, {"type": "error", "code": "Unauthorized", "message": "must authenticate"}
        for api in (self._route_v3, self._route_provisioning, self._route_k8s):
            out = api(method, path, query, body)
            if out is not None:
                return out
        return 404, {"type": "error", "code": "NotFound", "path": path}

    def _handler(self):
        fake = self

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def setup(self):
                if fake._tls_ctx is not None:  # the handshake on this connection's own thread
                    self.request.settimeout(10.0)
                    self.request.do_handshake()
                    self.request.settimeout(None)
                super().setup()
                # one request/response per segment: no Nagle/delayed-ACK stalls on keep-alive
                self.request.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

            def log_message(self, *args):  # quiet
                pass

            def _send(self, code: int, obj: Any = None, raw: Optional[bytes] = None):
                body = raw if raw is not None else (json.dumps(obj).encode() if obj is not None else b"")
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _body(self) -> Any:
                n = int(self.headers.get("Content-Length") or 0)
                raw = self.rfile.read(n) if n else b""
                fake.request_bodies.append(raw)
                try:
                    return json.loads(raw) if raw else {}
                except ValueError:
                    return {}

            def _authed(self) -> bool:
                auth = self.headers.get("Authorization", "")
                st = fake.state
                if auth.startswith("Basic "):
                    try:
                        user, _, secret = base64.b64decode(auth[6:]).decode().partition(":")
                    except ValueError:
                        return False
                elif auth.startswith("Bearer "):
                    user, _, secret = auth[7:].partition(":")
                else:
                    return False
                with st.mu:
                    return bool(secret) and st.tokens.get(user) == secret

            def do_GET(self):
                self._dispatch("GET")

            def do_POST(self):
                self._dispatch("POST")

            def do_PUT(self):
                self._dispatch("PUT")

            def do_DELETE(self):
                self._dispatch("DELETE")

            def do_PATCH(self):
                self._dispatch("PATCH")

            def do_HEAD(self):
                self._dispatch("HEAD")

            def _dispatch(self, method: str):
                st = fake.state
                parts = urllib.parse.urlsplit(self.path)
                path, query = parts.path.rstrip("/") or "/", urllib.parse.parse_qs(parts.query)
                with st.mu:
                    st.requests += 1
                    st.log.append((method, self.path))
                body = self._body() if method in ("POST", "PUT", "PATCH") else {}
                try:
                    code, obj = fake._route(method, path, query, body, self)
                except Exception as exc:  # pragma: no cover - surfaced to the client
                    code, obj = 500, {"type": "error", "message": str(exc)}
                if isinstance(obj, bytes):
                    self._send(code, raw=obj)
                else:
                    self._send(code, obj)

        return H


__all__ = ["FakeRancher", "State", "FAKE_CACERTS"]
