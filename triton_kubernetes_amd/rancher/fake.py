"""In-process fake Rancher 2.x server (the Rancher API fake SURVEY.md §4 calls for).

Implements the v3 endpoints the framework uses plus a simulation of what the
real server does after agents register:

* S3 bootstrap endpoints (login, token, change password, settings).  Like
  Rancher ≥2.6 the server starts with a *bootstrap* admin password
  (``CATTLE_BOOTSTRAP_PASSWORD``; random when not given — there is no admin/admin)
  and refuses new passwords shorter than ``password-min-length`` (12);
* S4 cluster endpoints (find/create cluster, registration tokens, cacerts).  A
  cluster whose ``kubernetesVersion`` is not in the server's KDM list (setting
  ``k8s-versions-current``: the pinned Rancher's RKE1 releases, versions.py) is
  rejected with 422, as the real server does;
* RKE2 custom clusters (provisioning v2): ``POST /v1/provisioning.cattle.io.clusters``
  (``fleet-default``; a release outside ``/v1-rke2-release/releases`` or an unknown CNI
  is rejected with 422), ``GET …/fleet-default/<name>`` whose ``status.clusterName``
  (the ``c-m-…`` management cluster) the controllers fill in after the create returns;
  the management cluster then behaves like an RKE1 one (tokens, nodes, proxy, state);
  ``GET /system-agent-install.sh`` serves the node installer;  A new registration token's value is
  filled in by the server's controller after the create returns
  (``async_registration_tokens``, default on): the POST answers with an empty
  ``token`` and the first read of the object after that sees it, so clients must poll;
* ``POST /v3/connect/register`` — agent registration (``X-API-Tunnel-Token`` +
  base64 JSON ``X-API-Tunnel-Params`` with hostname, roles, labels, capacity),
  standing in for the rancher-agent websocket tunnel; ``X-Cattle-Agent-Kind:
  system-agent`` marks an RKE2 node's ``rancher-system-agent``.  A node of the wrong
  kind for its cluster's distribution is refused (400);
* RKE simulation: a cluster turns ``active`` ``rke_seconds`` after it has at
  least one etcd, one controlplane and one worker node; nodes then report the
  Kubernetes ``Ready`` condition;
* ``/k8s/clusters/<id>/...`` proxy: ``api/v1/nodes`` (labels, conditions,
  allocatable) and a generic object store for applied manifests;
* device plugins, as the kubelet sees them: ``amd.com/gpu`` appears in a node's
  capacity/allocatable only when a device-plugin pod runs on it and registers.  A
  DaemonSet counts as the AMD GPU plugin when a container runs a
  ``rocm/k8s-device-plugin`` image (not the labeller tag) and mounts the host's
  ``/var/lib/kubelet/device-plugins`` (the registration socket) and ``/sys`` (where it
  enumerates the KFD devices).  Its pod lands on a node only if the node is Ready, its
  labels satisfy the ``nodeSelector`` and required node affinity, and the pod
  tolerates the node's taints; it registers ``device_plugin_seconds`` after both the
  DaemonSet and the node exist.  The count it registers is the number of GPU devices
  the node has (what its agent reported at registration: the KFD GPU nodes, i.e.
  logical GPUs under a partition mode).  DaemonSet reads carry ``status``
  (``desiredNumberScheduled``, ``numberReady``);
* mutating admission: a Pod created through the proxy goes through every applied
  ``MutatingWebhookConfiguration`` whose rules and namespace selector match — the
  webhook is called over HTTPS, its certificate verified against the ``caBundle``
  for ``<service>.<namespace>.svc`` (``service_endpoints`` maps a service to the
  address it really listens on), and the returned JSONPatch is applied;
  ``failurePolicy: Fail`` turns a webhook error into a rejected create.  Namespace
  selectors see the labels of the Namespace objects created through the proxy;
* Pod Security Admission, after mutation as in a real API server: the namespace's
  ``pod-security.kubernetes.io/enforce`` label (else ``default_pod_security``) at
  ``baseline`` rejects host namespaces, privileged containers, added capabilities
  beyond the default set, hostPath volumes and host ports; ``restricted`` also
  requires ``runAsNonRoot``, ``allowPrivilegeEscalation: false``, dropping ``ALL``
  capabilities, a RuntimeDefault/Localhost seccomp profile and only the restricted
  volume types (403 ``violates PodSecurity``).

Everything is in memory and thread-safe; it serves plain HTTP on 127.0.0.1.
"""

import base64
import http.client
import http.server
import json
import re
import secrets
import socket
import ssl
import threading
import time
import urllib.parse
import uuid
from typing import Any, Dict, List, Optional, Sequence, Set, Tuple

from ..versions import (DEFAULT_K8S_VERSION, FLEET_NAMESPACE, K8S_VERSIONS, PASSWORD_MIN_LENGTH, RANCHER_VERSION,
                        RKE2_CNIS, RKE2_VERSIONS, SYSTEM_AGENT_INSTALL_PATH, bootstrap_password, running_version)
from ..utils.httpserver import Server as HTTPServer

FAKE_CACERTS = "-----BEGIN CERTIFICATE-----\nMIIFAKECERTIFICATEFORTESTS\n-----END CERTIFICATE-----"
# what GET /system-agent-install.sh serves here: records its arguments (tests run it)
SYSTEM_AGENT_INSTALL_SCRIPT = r"""#!/bin/sh
# fake rancher-system-agent installer: takes the flags the real system-agent-install.sh
# takes, checks --ca-checksum the way it does (sha256 of GET <server>/cacerts), then
# registers the node with this server -- what the installed rancher-system-agent does
echo "system-agent-install $*" >> "${TK_FAKE_SYSTEM_AGENT_LOG:-/dev/null}"
server=""; token=""; checksum=""; name=""; etcd=false; cp=false; worker=false; labels=""; taints=""
while [ $# -gt 0 ]; do
  case "$1" in
    --server) server=$2; shift 2 ;;
    --token) token=$2; shift 2 ;;
    --ca-checksum) checksum=$2; shift 2 ;;
    --node-name) name=$2; shift 2 ;;
    --label) labels="$labels${labels:+,}\"${2%%=*}\":\"${2#*=}\""; shift 2 ;;
    --taints) _r=${2#*=}; taints="$taints${taints:+,}{\"key\":\"${2%%=*}\",\"value\":\"${_r%%:*}\",\"effect\":\"${_r#*:}\"}"; shift 2 ;;
    --etcd) etcd=true; shift ;;
    --controlplane) cp=true; shift ;;
    --worker) worker=true; shift ;;
    *) echo "system-agent-install: unknown option $1" >&2; exit 1 ;;
  esac
done
[ -n "$server" ] && [ -n "$token" ] || { echo "system-agent-install: --server and --token are required" >&2; exit 1; }
if [ -n "$checksum" ]; then
  got=$(curl -fsSk "$server/cacerts" | sha256sum | cut -d' ' -f1)
  [ "$got" = "$checksum" ] || { echo "system-agent-install: configured cacerts checksum ($got) does not match --ca-checksum ($checksum)" >&2; exit 1; }
fi
[ -n "$name" ] || name=$(hostname)
params=$(printf '{"node":{"requestedHostname":"%s","etcd":%s,"controlPlane":%s,"worker":%s,"labels":{%s},"taints":[%s]}}' \
  "$name" $etcd $cp $worker "$labels" "$taints" | base64 | tr -d '\n')
curl -fsSk -o /dev/null -X POST -H "X-API-Tunnel-Token: $token" -H "X-API-Tunnel-Params: $params" \
  -H "X-Cattle-Agent-Kind: system-agent" -d '{}' "$server/v3/connect/register" \
  || { echo "system-agent-install: registration with $server failed" >&2; exit 1; }
"""


class _State:
    def __init__(self, rke_seconds: float, node_ready_seconds: float, admin_password: str,
                 k8s_versions: Sequence[str], rke2_versions: Sequence[str] = ()):
        self.mu = threading.RLock()
        self.cond = threading.Condition(self.mu)
        self.admin_password = admin_password
        self.tokens: Dict[str, str] = {}  # name -> secret
        self.settings: Dict[str, str] = {"cacerts": FAKE_CACERTS, "server-url": "",
                                         "server-version": RANCHER_VERSION,
                                         "k8s-versions-current": ",".join(k8s_versions),
                                         "k8s-version": DEFAULT_K8S_VERSION,
                                         "password-min-length": str(PASSWORD_MIN_LENGTH)}
        self.clusters: Dict[str, Dict[str, Any]] = {}
        self.rke2_versions: List[str] = list(rke2_versions)
        self.v2_clusters: Dict[str, Dict[str, Any]] = {}  # "<namespace>/<name>" -> provisioning object
        self.secrets: Dict[str, Dict[str, Any]] = {}  # "<namespace>/<name>" -> Secret (management cluster)
        self.reg_tokens: Dict[str, Dict[str, Any]] = {}  # token -> {clusterId, id}
        self.nodes: Dict[str, Dict[str, Any]] = {}
        # indexes, so a request costs the same however many clusters the server holds
        self.cluster_nodes: Dict[str, Dict[str, Dict[str, Any]]] = {}  # cluster id -> node id -> node
        self.unsettled: Set[str] = set()  # clusters not yet active, or with a node not yet active
        self.objects: Dict[str, Dict[str, Any]] = {}  # "<cluster>|<path>|<name>" -> object
        self.cluster_objects: Dict[str, Dict[str, None]] = {}  # cluster id -> its object keys, in creation order
        self.object_times: Dict[str, float] = {}  # object key -> when it was created
        self.rke_seconds = rke_seconds
        self.node_ready_seconds = node_ready_seconds
        self.device_plugin_seconds = 0.0
        self.upgrade_seconds = 0.0  # a rolling Kubernetes upgrade's duration
        self.requests = 0
        self.log: List[Tuple[str, str]] = []


class FakeRancher:
    def __init__(self, rke_seconds: float = 0.0, node_ready_seconds: float = 0.0,
                 bootstrap_password: Optional[str] = None, host: str = "127.0.0.1", port: int = 0,
                 k8s_versions: Optional[Sequence[str]] = None, async_registration_tokens: bool = True,
                 default_pod_security: str = "privileged", rke2_versions: Optional[Sequence[str]] = None,
                 device_plugin_seconds: float = 0.0):
        # a server started without CATTLE_BOOTSTRAP_PASSWORD has a random one nobody knows
        pw = bootstrap_password if bootstrap_password is not None else secrets.token_hex(16)
        self.state = _State(rke_seconds, node_ready_seconds, pw,
                            list(k8s_versions) if k8s_versions is not None else [v for _, v in K8S_VERSIONS],
                            list(rke2_versions) if rke2_versions is not None else [v for _, v in RKE2_VERSIONS])
        self.state.device_plugin_seconds = device_plugin_seconds
        # "<service>.<namespace>" -> "https://127.0.0.1:<port>" (where an in-cluster
        # webhook service of a test really listens)
        self.service_endpoints: Dict[str, str] = {}
        self.async_registration_tokens = async_registration_tokens
        # Pod Security level of namespaces without an enforce label (the API server's
        # AdmissionConfiguration default; Kubernetes' own default is privileged)
        self.default_pod_security = default_pod_security
        self._server = HTTPServer((host, port), self._handler())
        self._server.daemon_threads = True
        self._thread: Optional[threading.Thread] = None

    def _token_view(self, tok: str, fill: bool = True) -> Dict[str, Any]:
        """A registration token as the API shows it: its value only once the (simulated)
        controller has filled it in — which happens on the first read after the create."""
        t = self.state.reg_tokens[tok]
        shown = tok if t["ready"] else ""
        if fill:
            t["ready"] = True
        return {"id": t["id"], "clusterId": t["clusterId"], "token": shown}

    @classmethod
    def for_manager(cls, name: str, admin_password: str, **kw: Any) -> "FakeRancher":
        """A server started the way this framework starts one for manager ``name``."""
        return cls(bootstrap_password=bootstrap_password(name, admin_password), **kw)

    @property
    def url(self) -> str:
        host, port = self._server.server_address[:2]
        return f"http://{host}:{port}"

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

    # --- kubelet / DaemonSet model ------------------------------------------------------------
    def _daemonsets(self, cid: str) -> List[Tuple[str, Dict[str, Any]]]:
        """(key, object) of the cluster's DaemonSets (caller holds the lock)."""
        st = self.state
        return [(k, st.objects[k]) for k in st.cluster_objects.get(cid, ())
                if k.split("|")[1].endswith("/daemonsets") and k in st.objects]

    @staticmethod
    def _node_labels(n: Dict[str, Any]) -> Dict[str, str]:
        labels = dict(n["labels"])
        labels.setdefault("kubernetes.io/hostname", n["hostname"])
        for r, on in n["roles"].items():
            if on:
                labels[f"node-role.kubernetes.io/{r}"] = "true"
        return labels

    def _runs_on(self, ds: Dict[str, Any], n: Dict[str, Any], ds_key: str = "") -> bool:
        """Does a pod of ``ds`` run on node ``n`` (Ready, selector, affinity, taints)?  As in
        Kubernetes, a ``NoSchedule`` taint added after the pod was scheduled does not evict
        it (only ``NoExecute`` does); one present at scheduling time keeps it off."""
        if n["state"] != "active":
            return False
        pod = ((ds.get("spec") or {}).get("template") or {}).get("spec") or {}
        labels = self._node_labels(n)
        if any(labels.get(k) != v for k, v in (pod.get("nodeSelector") or {}).items()):
            return False
        terms = (((pod.get("affinity") or {}).get("nodeAffinity") or {})
                 .get("requiredDuringSchedulingIgnoredDuringExecution") or {}).get("nodeSelectorTerms")
        if terms and not any(_match_expressions(t.get("matchExpressions") or [], labels) for t in terms):
            return False
        tolerations = pod.get("tolerations") or []
        scheduled = max(self.state.object_times.get(ds_key, 0.0), n.get("ready_at") or 0.0)
        added = n.get("taint_added") or {}
        return all(_tolerated(t, tolerations) for t in n.get("taints") or []
                   if t.get("effect") == "NoExecute"
                   or (t.get("effect") == "NoSchedule" and added.get(t.get("key"), 0.0) <= scheduled))

    @staticmethod
    def _is_gpu_plugin(ds: Dict[str, Any]) -> bool:
        """A DaemonSet whose pod can register ``amd.com/gpu`` with the kubelet."""
        pod = ((ds.get("spec") or {}).get("template") or {}).get("spec") or {}
        host = {v.get("name"): (v.get("hostPath") or {}).get("path") for v in pod.get("volumes") or []
                if "hostPath" in v}
        for c in pod.get("containers") or []:
            repo, _, tag = str(c.get("image", "")).rpartition(":")
            if repo not in DEVICE_PLUGIN_REPOS or tag.startswith("labeller"):
                continue
            mounted = {m.get("mountPath"): host.get(m.get("name")) for m in c.get("volumeMounts") or []}
            if (mounted.get(DEVICE_PLUGIN_SOCKET_DIR) == DEVICE_PLUGIN_SOCKET_DIR
                    and mounted.get("/sys") == "/sys"):
                return True
        return False

    def _plugin_ready_at(self, cid: str, ds_key: str, n: Dict[str, Any]) -> float:
        created = self.state.object_times.get(ds_key, 0.0)
        return max(created, n.get("ready_at") or 0.0) + self.state.device_plugin_seconds

    def _gpu_allocatable(self, cid: str, n: Dict[str, Any], now: float) -> Optional[int]:
        """GPUs a running, registered device-plugin pod advertises on ``n`` (None: none):
        the devices the node agent reported, else what its labeller counted (a node joined
        through the installer reports only labels)."""
        devices = int(n["capacity"].get("amd.com/gpu", 0) or n["labels"].get("amd.com/gpu.logical-count", 0) or 0)
        for key, ds in self._daemonsets(cid):
            if self._is_gpu_plugin(ds) and self._runs_on(ds, n, key) and now >= self._plugin_ready_at(cid, key, n):
                return devices
        return None

    def _daemonset_status(self, cid: str, key: str, ds: Dict[str, Any]) -> Dict[str, Any]:
        now = time.time()
        nodes = [n for n in self.state.cluster_nodes.get(cid, {}).values() if self._runs_on(ds, n, key)]
        ready = [n for n in nodes if now >= self._plugin_ready_at(cid, key, n)]
        return {"desiredNumberScheduled": len(nodes), "currentNumberScheduled": len(nodes),
                "numberReady": len(ready), "numberAvailable": len(ready)}

    def device_plugin_applied(self, cluster_id: str) -> bool:
        with self.state.mu:
            return any(self._is_gpu_plugin(ds) for _, ds in self._daemonsets(cluster_id))

    def k8s_nodes(self, cluster_id: str) -> List[Dict[str, Any]]:
        self._refresh()
        st = self.state
        items = []
        now = time.time()
        with st.mu:
            for n in st.cluster_nodes.get(cluster_id, {}).values():
                ready = n["state"] == "active"
                alloc = {"cpu": "64", "memory": "1Ti", "pods": "110"}
                gpus = self._gpu_allocatable(cluster_id, n, now)
                if gpus is not None:
                    alloc["amd.com/gpu"] = str(gpus)
                items.append({
                    "metadata": {"name": n["hostname"], "labels": self._node_labels(n),
                                 "resourceVersion": str(n.get("rv", 1))},
                    "spec": dict({"taints": list(n.get("taints") or [])},
                                 **({"unschedulable": True} if n.get("unschedulable") else {})),
                    "status": {"conditions": [{"type": "Ready", "status": "True" if ready else "False"}],
                               "nodeInfo": {"kubeletVersion": str(((st.clusters.get(cluster_id) or {})
                                                                   .get("version") or {}).get("gitVersion", ""))},
                               "allocatable": alloc, "capacity": dict(alloc)},
                })
        return items

    # --- HTTP ------------------------------------------------------------------------------
    def _handler(self):
        fake = self

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def setup(self):
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
                    with st.mu:
                        return st.tokens.get(user) == secret
                if auth.startswith("Bearer "):
                    user, _, secret = auth[7:].partition(":")
                    with st.mu:
                        return st.tokens.get(user) == secret
                return False

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

    def _route(self, method: str, path: str, query: Dict[str, List[str]], body: Any, h) -> Tuple[int, Any]:
        st = self.state
        if path == "/ping":
            return 200, b"pong"
        if path == "/v3-public/localProviders/local" and query.get("action") == ["login"]:
            if body.get("username") == "admin" and body.get("password") == st.admin_password:
                name, secret = f"token-{uuid.uuid4().hex[:5]}", uuid.uuid4().hex
                with st.mu:
                    st.tokens[name] = secret
                return 201, {"token": f"{name}:{secret}", "type": "token"}
            return 401, {"type": "error", "code": "Unauthorized"}
        if path == "/v3/connect/register" and method == "POST":
            return self._register(h)
        if path == SYSTEM_AGENT_INSTALL_PATH and method == "GET":
            return 200, SYSTEM_AGENT_INSTALL_SCRIPT.encode()
        if path == "/cacerts" and method == "GET":  # unauthenticated, what the installers pin
            with st.mu:
                ca = st.settings.get("cacerts", "")
                return 200, (ca if not ca or ca.endswith("\n") else ca + "\n").encode()
        if not h._authed():
            return 401, {"type": "error", "code": "Unauthorized"}
        if path == "/v1-rke2-release/releases" and method == "GET":
            return 200, {"data": [{"id": v, "version": v, "type": "release"} for v in st.rke2_versions]}
        if path == "/v1/provisioning.cattle.io.clusters" and method == "POST":
            return self._create_v2(body)
        if path == "/v1/secrets" and method == "POST":
            meta = dict((body or {}).get("metadata") or {})
            ns = meta.get("namespace") or "default"
            name = meta.get("name") or (meta.get("generateName", "secret-") + uuid.uuid4().hex[:5])
            with st.mu:
                if f"{ns}/{name}" in st.secrets:
                    return 409, {"type": "error", "code": "AlreadyExists"}
                st.secrets[f"{ns}/{name}"] = dict(body, metadata=dict(meta, name=name, namespace=ns))
                return 201, json.loads(json.dumps(st.secrets[f"{ns}/{name}"]))
        if path.startswith("/v1/provisioning.cattle.io.clusters/"):
            key = path[len("/v1/provisioning.cattle.io.clusters/"):]
            return self._v2_cluster(method, key, body)
        if path == "/v3/token" and method == "POST":
            name, secret = f"token-{uuid.uuid4().hex[:5]}", uuid.uuid4().hex
            with st.mu:
                st.tokens[name] = secret
            return 201, {"name": name, "token": f"{name}:{secret}", "type": "token"}
        if path == "/v3/users" and query.get("action") == ["changepassword"]:
            if body.get("currentPassword") != st.admin_password:
                return 400, {"type": "error", "message": "invalid current password"}
            if len(body.get("newPassword", "")) < int(st.settings["password-min-length"]):
                return 422, {"type": "error", "code": "InvalidFormat",
                             "message": f"Password must be at least {st.settings['password-min-length']} characters"}
            st.admin_password = body.get("newPassword", "")
            return 200, {}
        if path.startswith("/v3/settings/"):
            key = path.rsplit("/", 1)[1]
            if method == "PUT":
                st.settings[key] = body.get("value", "")
            return 200, {"id": key, "name": key, "value": st.settings.get(key, "")}
        if path == "/v3/clusters" and method == "GET":
            self._refresh()
            names = query.get("name")
            with st.mu:
                data = [c for c in st.clusters.values() if not names or c["name"] in names]
            return 200, {"data": data}
        if path == "/v3/cluster" and method == "POST":
            version = (body.get("rancherKubernetesEngineConfig") or {}).get("kubernetesVersion", "")
            offered = [v for v in st.settings["k8s-versions-current"].split(",") if v]
            if version not in offered:
                return 422, {"type": "error", "code": "InvalidBodyContent", "fieldName": "kubernetesVersion",
                             "message": f"{version} is not a supported Kubernetes version"}
            cid = f"c-{uuid.uuid4().hex[:5]}"
            with st.mu:
                st.clusters[cid] = {"id": cid, "name": body.get("name", ""), "state": "provisioning",
                                    "transitioning": "yes", "rancherKubernetesEngineConfig":
                                        body.get("rancherKubernetesEngineConfig", {}), "created": time.time(),
                                    "driver": "rancherKubernetesEngine",
                                    # Rancher reports an RKE1 cluster's upstream version
                                    "version": {"gitVersion": running_version(version, "rke1")}}
                st.cluster_nodes[cid] = {}
                st.unsettled.add(cid)
                return 201, dict(st.clusters[cid])
        if path.startswith("/v3/clusters/"):
            rest = path[len("/v3/clusters/"):].split("/")
            cid = rest[0]
            with st.mu:
                if cid not in st.clusters:
                    return 404, {"type": "error", "code": "NotFound"}
            if len(rest) == 2 and rest[1] == "clusterregistrationtokens":
                with st.mu:
                    data = [self._token_view(tok) for tok, t in st.reg_tokens.items() if t["clusterId"] == cid]
                return 200, {"data": data}
            if method == "DELETE":
                with st.mu:
                    st.clusters.pop(cid, None)
                    st.unsettled.discard(cid)
                    for nid in st.cluster_nodes.pop(cid, {}):
                        st.nodes.pop(nid, None)
                return 200, {}
            if method == "POST" and query.get("action") == ["generateKubeconfig"]:
                return 200, {"config": f"apiVersion: v1\nkind: Config\nclusters:\n- name: {cid}\n"}
            if method == "PUT":
                with st.mu:
                    if st.clusters[cid].get("driver") == "rke2":  # the provisioning object owns it
                        return 422, {"type": "error", "code": "Invalid",
                                     "message": "an RKE2 cluster is changed through provisioning.cattle.io"}
                    return self._upgrade(cid, body)
            self._refresh()
            with st.mu:
                return 200, dict(st.clusters[cid])
        if path == "/v3/clusterregistrationtoken" and method == "POST":
            tok = uuid.uuid4().hex + uuid.uuid4().hex[:8]
            cid = body.get("clusterId")
            with st.mu:
                if cid not in st.clusters:
                    return 422, {"type": "error", "code": "InvalidReference", "fieldName": "clusterId"}
                n = sum(1 for t in st.reg_tokens.values() if t["clusterId"] == cid)
                st.reg_tokens[tok] = {"id": f"{cid}:crt-{n}", "clusterId": cid,
                                      "ready": not self.async_registration_tokens}
                return 201, dict(self._token_view(tok, fill=False), type="clusterRegistrationToken")
        if path.startswith("/v3/clusterregistrationtokens/") and method == "GET":
            tid = urllib.parse.unquote(path[len("/v3/clusterregistrationtokens/"):])
            with st.mu:
                tok = next((k for k, t in st.reg_tokens.items() if t["id"] == tid), None)
                if tok is None:
                    return 404, {"type": "error", "code": "NotFound"}
                return 200, self._token_view(tok)
        if path == "/v3/nodes" and method == "GET":
            self._refresh()
            cids = query.get("clusterId")
            with st.mu:
                if cids:
                    data = [dict(n) for c in cids for n in st.cluster_nodes.get(c, {}).values()]
                else:
                    data = [dict(n) for n in st.nodes.values()]
            return 200, {"data": data}
        if path.startswith("/v3/nodes/") and method == "DELETE":
            with st.mu:
                n = st.nodes.pop(path.rsplit("/", 1)[1], None)
                if n is not None:
                    st.cluster_nodes.get(n["clusterId"], {}).pop(n["id"], None)
            return 200, {}
        if path.startswith("/k8s/clusters/"):
            return self._k8s(method, path, body, query)
        return 404, {"type": "error", "code": "NotFound", "path": path}

    def _admit(self, cid: str, namespace: str, pod: Dict[str, Any]) -> Dict[str, Any]:
        return _admit_pod(self, cid, namespace, pod)

    # --- RKE2 custom clusters (provisioning.cattle.io/v1) ------------------------------------------
    def _upgrade(self, cid: str, body: Any, v2: Optional[Dict[str, Any]] = None) -> Tuple[int, Any]:
        """A cluster's new Kubernetes release (caller holds the lock): offered by the server,
        not lower than the running one; the cluster reads ``upgrading`` until the (simulated)
        rolling upgrade is over, and the kubelets report the new release."""
        st = self.state
        c = st.clusters.get(cid)
        if c is None:
            return 404, {"type": "error", "code": "NotFound"}
        spec = (body or {}).get("spec") if v2 is not None else (body or {}).get("rancherKubernetesEngineConfig")
        version = (spec or {}).get("kubernetesVersion", "")
        offered = st.rke2_versions if v2 is not None else [v for v in st.settings["k8s-versions-current"].split(",") if v]
        if version not in offered:
            return 422, {"type": "error", "code": "Invalid", "fieldName": "kubernetesVersion",
                         "message": f"{version} is not a supported Kubernetes version"}

        def key(v: str) -> Tuple[int, ...]:
            return tuple(int(x) for x in re.findall(r"\d+", v.split("+")[0].split("-")[0]))

        current = (c.get("version") or {}).get("gitVersion", "")
        if key(version) < key(current):
            return 422, {"type": "error", "code": "Invalid", "message": f"cannot downgrade {current} to {version}"}
        running = version if v2 is not None else running_version(version, "rke1")
        if running != current:
            c["version"] = {"gitVersion": running}
            c["state"], c["transitioning"] = "upgrading", "yes"
            c["ready_at"] = time.time() + st.upgrade_seconds
            st.unsettled.add(cid)
            st.upgrades = getattr(st, "upgrades", 0) + 1
        if v2 is not None:
            v2["spec"]["kubernetesVersion"] = version
            return 200, json.loads(json.dumps(v2))
        c.setdefault("rancherKubernetesEngineConfig", {})["kubernetesVersion"] = version
        return 200, dict(c)

    def _create_v2(self, body: Dict[str, Any]) -> Tuple[int, Any]:
        st = self.state
        meta, spec = body.get("metadata") or {}, body.get("spec") or {}
        ns, name = meta.get("namespace") or FLEET_NAMESPACE, meta.get("name", "")
        version = spec.get("kubernetesVersion", "")
        if version not in st.rke2_versions:
            return 422, {"type": "error", "code": "Invalid", "fieldName": "spec.kubernetesVersion",
                         "message": f"{version} is not a supported RKE2 version"}
        cni = ((spec.get("rkeConfig") or {}).get("machineGlobalConfig") or {}).get("cni", "canal")
        if cni not in RKE2_CNIS:
            return 422, {"type": "error", "code": "Invalid", "message": f"unsupported cni {cni!r}"}
        for host, conf in (((spec.get("rkeConfig") or {}).get("registries") or {}).get("configs") or {}).items():
            unknown = set(conf) - {"authConfigSecretName", "caBundle", "insecureSkipVerify", "tlsSecretName"}
            ref = conf.get("authConfigSecretName")
            if unknown or (ref and f"{ns}/{ref}" not in st.secrets):
                # the schema has no inline credentials: they live in a Secret of the namespace
                return 422, {"type": "error", "code": "Invalid",
                             "message": f"registries.configs[{host}]: unknown fields {sorted(unknown)} or "
                                        f"missing secret {ref!r}"}
        with st.mu:
            if f"{ns}/{name}" in st.v2_clusters:
                return 409, {"type": "error", "code": "AlreadyExists"}
            obj = json.loads(json.dumps(body))
            obj["metadata"].update(namespace=ns, uid=str(uuid.uuid4()))
            obj["status"] = {"ready": False}  # clusterName: filled in by the controllers
            st.v2_clusters[f"{ns}/{name}"] = obj
            return 201, json.loads(json.dumps(obj))

    def _v2_cluster(self, method: str, key: str, body: Any = None) -> Tuple[int, Any]:
        st = self.state
        with st.mu:
            obj = st.v2_clusters.get(key)
            if obj is None:
                return 404, {"type": "error", "code": "NotFound"}
            if method == "PUT":
                return self._upgrade(obj["status"].get("clusterName", ""), body, v2=obj)
            if method == "DELETE":
                st.v2_clusters.pop(key)
                cid = obj["status"].get("clusterName")
                if cid:
                    st.clusters.pop(cid, None)
                    for nid in st.cluster_nodes.pop(cid, {}):
                        st.nodes.pop(nid, None)
                return 200, {}
            if not obj["status"].get("clusterName"):
                # the provisioning controller creates the management cluster after the create
                cid = f"c-m-{uuid.uuid4().hex[:8]}"
                version = obj["spec"].get("kubernetesVersion", "")
                st.clusters[cid] = {"id": cid, "name": obj["metadata"]["name"], "state": "provisioning",
                                    "transitioning": "yes", "driver": "rke2", "created": time.time(),
                                    "version": {"gitVersion": version}}
                st.cluster_nodes[cid] = {}
                st.unsettled.add(cid)
                obj["status"]["clusterName"] = cid
                return 200, json.loads(json.dumps(obj))
            cid = obj["status"]["clusterName"]
        self._refresh()
        with st.mu:
            obj["status"]["ready"] = (st.clusters.get(cid) or {}).get("state") == "active"
            return 200, json.loads(json.dumps(obj))

    def registration(self, name: str = "test", distribution: str = "rke2") -> Tuple[str, str, str]:
        """``(cluster id, registration token, ca checksum)`` of a new cluster: what an admin
        copies out of the UI's registration command (tests of the node-side join)."""
        from .client import ca_checksum

        st = self.state
        with st.mu:
            cid = f"c-m-{uuid.uuid4().hex[:8]}" if distribution == "rke2" else f"c-{uuid.uuid4().hex[:5]}"
            st.clusters[cid] = {"id": cid, "name": name, "state": "provisioning", "transitioning": "yes",
                                "driver": "rke2" if distribution == "rke2" else "rancherKubernetesEngine",
                                "created": time.time(), "version": {"gitVersion": ""}}
            st.cluster_nodes[cid] = {}
            st.unsettled.add(cid)
            tok = secrets.token_hex(16)
            st.reg_tokens[tok] = {"id": f"{cid}:default-token", "clusterId": cid, "ready": True}
            return cid, tok, ca_checksum(st.settings.get("cacerts", ""))

    def registry_auth(self, secret: str, namespace: str = FLEET_NAMESPACE) -> Dict[str, str]:
        """Decoded ``username``/``password`` of a registry basic-auth Secret."""
        with self.state.mu:
            data = (self.state.secrets.get(f"{namespace}/{secret}") or {}).get("data") or {}
        return {k: base64.b64decode(v).decode() for k, v in data.items()}

    def namespace_labels(self, cid: str, namespace: str) -> Dict[str, str]:
        """Labels of a Namespace created through the proxy (+ the automatic name label)."""
        with self.state.mu:
            ns = self.state.objects.get(f"{cid}|/api/v1/namespaces|{namespace}") or {}
        labels = dict((ns.get("metadata") or {}).get("labels") or {})
        labels["kubernetes.io/metadata.name"] = namespace
        return labels

    def _register(self, h) -> Tuple[int, Any]:
        st = self.state
        token = h.headers.get("X-API-Tunnel-Token", "")
        with st.mu:
            reg = st.reg_tokens.get(token)
        if reg is None:
            return 401, {"type": "error", "code": "InvalidRegistrationToken"}
        try:
            params = json.loads(base64.b64decode(h.headers.get("X-API-Tunnel-Params", "")) or b"{}")
        except ValueError:
            return 400, {"type": "error", "message": "bad tunnel params"}
        kind = h.headers.get("X-Cattle-Agent-Kind", "rancher-agent")
        with st.mu:
            prov = "rke2" if (st.clusters.get(reg["clusterId"]) or {}).get("driver") == "rke2" else "rke1"
        if (prov == "rke2") != (kind == "system-agent"):
            want = "rancher-system-agent (system-agent-install.sh)" if prov == "rke2" else "rancher-agent"
            return 400, {"type": "error", "code": "InvalidAgent",
                         "message": f"{reg['clusterId']} is an {prov.upper()} cluster: nodes join with {want}"}
        node = params.get("node", {})
        hostname = node.get("requestedHostname", "")
        roles = {"etcd": bool(node.get("etcd")), "controlplane": bool(node.get("controlPlane")),
                 "worker": bool(node.get("worker"))}
        with st.mu:
            members = st.cluster_nodes.setdefault(reg["clusterId"], {})
            existing = [nid for nid, n in members.items() if n["hostname"] == hostname]
            nid = existing[0] if existing else f"m-{uuid.uuid4().hex[:6]}"
            st.nodes[nid] = members[nid] = {
                "id": nid, "clusterId": reg["clusterId"], "hostname": hostname, "nodeName": hostname, "agentKind": kind,
                "roles": roles, "labels": dict(node.get("labels", {})), "capacity": dict(node.get("capacity", {})),
                "taints": [dict(t) for t in node.get("taints") or [] if isinstance(t, dict)],
                "state": "registering", "registered": time.time(), "ready_at": None}
            st.unsettled.add(reg["clusterId"])
            st.cond.notify_all()
        self._refresh()
        return 201, {"id": nid, "clusterId": reg["clusterId"]}

    def _k8s(self, method: str, path: str, body: Any, query: Optional[Dict[str, List[str]]] = None) -> Tuple[int, Any]:
        st = self.state
        rest = path[len("/k8s/clusters/"):]
        cid, _, kpath = rest.partition("/")
        with st.mu:
            if cid not in st.clusters:
                return 404, {"kind": "Status", "code": 404}
        kpath = "/" + kpath
        if kpath == "/api/v1/nodes" and method == "GET":
            return 200, {"kind": "NodeList", "items": self.k8s_nodes(cid)}
        if kpath.startswith("/api/v1/nodes/") and method == "PATCH":
            return self._patch_node(cid, kpath[len("/api/v1/nodes/"):], body)
        if kpath == "/api/v1/pods" and method == "GET":
            # every namespace's pods; the one field selector drain uses (spec.nodeName=...)
            sel = dict(s.split("=", 1) for s in ((query or {}).get("fieldSelector") or [""])[0].split(",") if "=" in s)
            with st.mu:
                pods = [st.objects[k] for k in st.cluster_objects.get(cid, ())
                        if k.split("|")[1].startswith("/api/v1/namespaces/") and k.split("|")[1].endswith("/pods")]
            if "spec.nodeName" in sel:
                pods = [p for p in pods if (p.get("spec") or {}).get("nodeName") == sel["spec.nodeName"]]
            return 200, {"kind": "PodList", "items": pods}
        parts = kpath.strip("/").split("/")
        if (method == "POST" and len(parts) == 7 and parts[:3] == ["api", "v1", "namespaces"] and parts[4] == "pods"
                and parts[6] == "eviction"):
            return self._evict(cid, parts[3], parts[5])
        if kpath == "/version":
            with st.mu:
                v = (st.clusters[cid].get("version") or {}).get("gitVersion") or DEFAULT_K8S_VERSION
            major, minor = v.lstrip("v").split(".")[:2]
            return 200, {"major": major, "minor": minor, "gitVersion": v.split("-")[0].split("+")[0]}
        if method == "POST":
            parts = kpath.strip("/").split("/")
            if len(parts) == 5 and parts[:3] == ["api", "v1", "namespaces"] and parts[4] == "pods":
                try:
                    body = self._admit(cid, parts[3], body)
                except _Rejected as exc:
                    return 400, {"kind": "Status", "reason": "BadRequest", "code": 400, "message": str(exc)}
                level = self.namespace_labels(cid, parts[3]).get(PSA_ENFORCE, self.default_pod_security)
                problems = pod_security_violations(body, level)
                if problems:
                    name = (body.get("metadata") or {}).get("name", "")
                    return 403, {"kind": "Status", "reason": "Forbidden", "code": 403,
                                 "message": f'pods "{name}" is forbidden: violates PodSecurity "{level}:latest": '
                                            + "; ".join(problems)}
            name = (body.get("metadata") or {}).get("name", uuid.uuid4().hex[:6])
            key = f"{cid}|{kpath}|{name}"
            with st.mu:
                if key in st.objects:
                    return 409, {"kind": "Status", "reason": "AlreadyExists", "code": 409}
                # server-populated fields, as a real API server adds them
                obj = json.loads(json.dumps(body))
                meta = obj.setdefault("metadata", {})
                meta.update({"uid": str(uuid.uuid4()), "resourceVersion": str(len(st.objects) + 1),
                             "creationTimestamp": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())})
                obj.setdefault("status", {})
                st.objects[key] = obj
                st.object_times[key] = time.time()
                st.cluster_objects.setdefault(cid, {})[key] = None
            return 201, obj
        if method in ("PUT", "GET", "DELETE"):
            base, _, name = kpath.rpartition("/")
            key = f"{cid}|{base}|{name}"
            with st.mu:
                if method == "PUT":
                    st.objects[key] = body
                    st.object_times.setdefault(key, time.time())
                    st.cluster_objects.setdefault(cid, {})[key] = None
                    return 200, body
                if method == "DELETE":
                    if key not in st.objects:
                        return 404, {"code": 404}
                    st.cluster_objects.get(cid, {}).pop(key, None)
                    st.object_times.pop(key, None)
                    return 200, st.objects.pop(key)
                if key in st.objects:
                    if base.endswith("/daemonsets"):
                        return 200, dict(st.objects[key], status=self._daemonset_status(cid, key, st.objects[key]))
                    return 200, st.objects[key]
                prefix = f"{cid}|{kpath}|"
                items = [st.objects[k] for k in st.cluster_objects.get(cid, ()) if k.startswith(prefix)]
                return 200, {"items": items}
        return 404, {"kind": "Status", "code": 404}


    def _patch_node(self, cid: str, name: str, patch: Any) -> Tuple[int, Any]:
        """JSON merge patch of a Node: labels merge (null deletes), ``spec.taints`` replaced."""
        st = self.state
        if not isinstance(patch, dict):
            return 400, {"kind": "Status", "code": 400, "message": "merge patch must be an object"}
        now = time.time()
        with st.mu:
            node = next((n for n in st.cluster_nodes.get(cid, {}).values() if n["hostname"] == name), None)
            if node is None:
                return 404, {"kind": "Status", "reason": "NotFound", "code": 404}
            # optimistic concurrency: a patch naming a resourceVersion applies to that one only
            want = (patch.get("metadata") or {}).get("resourceVersion")
            if want is not None and str(want) != str(node.get("rv", 1)):
                return 409, {"kind": "Status", "reason": "Conflict", "code": 409,
                             "message": f'Operation cannot be fulfilled on nodes "{name}": the object has been '
                                        "modified; please apply your changes to the latest version and try again"}
            node["rv"] = int(node.get("rv", 1)) + 1
            for k, v in ((patch.get("metadata") or {}).get("labels") or {}).items():
                if v is None:
                    node["labels"].pop(k, None)
                else:
                    node["labels"][k] = str(v)
            spec = patch.get("spec") or {}
            if "unschedulable" in spec:  # cordon / uncordon
                node["unschedulable"] = bool(spec["unschedulable"])
            if "taints" in spec:
                taints = [dict(t) for t in spec["taints"] or [] if isinstance(t, dict)]
                added = node.setdefault("taint_added", {})
                for t in taints:
                    added.setdefault(t.get("key"), now)
                for k in [k for k in added if k not in {t.get("key") for t in taints}]:
                    del added[k]
                node["taints"] = taints
        items = {i["metadata"]["name"]: i for i in self.k8s_nodes(cid)}
        return 200, items[name]


    # a pod annotated with this many refusals answers 429 (a PodDisruptionBudget at its
    # minimum) that many times before the eviction goes through; "always" never does
    PDB_ANNOTATION = "fake.triton-kubernetes.io/pdb-refusals"

    def _evict(self, cid: str, namespace: str, name: str) -> Tuple[int, Any]:
        """The Eviction subresource: the pod is deleted unless its budget refuses (429)."""
        st = self.state
        key = f"{cid}|/api/v1/namespaces/{namespace}/pods|{name}"
        with st.mu:
            pod = st.objects.get(key)
            if pod is None:
                return 404, {"kind": "Status", "reason": "NotFound", "code": 404}
            ann = (pod.get("metadata") or {}).setdefault("annotations", {})
            left = ann.get(self.PDB_ANNOTATION)
            if left == "always" or (left and int(left) > 0):
                if left != "always":
                    ann[self.PDB_ANNOTATION] = str(int(left) - 1)
                st.evictions_refused = getattr(st, "evictions_refused", 0) + 1
                return 429, {"kind": "Status", "reason": "TooManyRequests", "code": 429,
                             "message": "Cannot evict pod as it would violate the pod's disruption budget."}
            st.objects.pop(key)
            st.object_times.pop(key, None)
            st.cluster_objects.get(cid, {}).pop(key, None)
        return 201, {"kind": "Status", "status": "Success", "code": 201}


class _Rejected(Exception):
    pass


DEVICE_PLUGIN_REPOS = ("rocm/k8s-device-plugin", "docker.io/rocm/k8s-device-plugin")
DEVICE_PLUGIN_SOCKET_DIR = "/var/lib/kubelet/device-plugins"


def _match_expressions(exprs: List[Dict[str, Any]], labels: Dict[str, str]) -> bool:
    """A nodeSelectorTerm's ``matchExpressions`` (all must hold)."""
    for e in exprs:
        key, op, values = e.get("key", ""), e.get("operator", ""), list(e.get("values") or [])
        have = key in labels
        if op == "In" and not (have and labels[key] in values):
            return False
        if op == "NotIn" and have and labels[key] in values:
            return False
        if op == "Exists" and not have:
            return False
        if op == "DoesNotExist" and have:
            return False
        if op in ("Gt", "Lt"):
            try:
                v, ref = int(labels.get(key, "")), int(values[0])
            except (ValueError, IndexError):
                return False
            if (op == "Gt" and not v > ref) or (op == "Lt" and not v < ref):
                return False
    return True


def _tolerated(taint: Dict[str, Any], tolerations: List[Dict[str, Any]]) -> bool:
    for t in tolerations:
        if t.get("effect") and t.get("effect") != taint.get("effect"):
            continue
        if t.get("operator") == "Exists" and (not t.get("key") or t.get("key") == taint.get("key")):
            return True
        if t.get("key") == taint.get("key") and t.get("value", "") == taint.get("value", ""):
            return True
    return False


PSA_ENFORCE = "pod-security.kubernetes.io/enforce"
_BASELINE_CAPS = {"AUDIT_WRITE", "CHOWN", "DAC_OVERRIDE", "FOWNER", "FSETID", "KILL", "MKNOD", "NET_BIND_SERVICE",
                  "SETFCAP", "SETGID", "SETPCAP", "SETUID", "SYS_CHROOT"}
_RESTRICTED_VOLUMES = {"configMap", "csi", "downwardAPI", "emptyDir", "ephemeral", "persistentVolumeClaim",
                       "projected", "secret"}


def pod_security_violations(pod: Dict[str, Any], level: str) -> List[str]:
    """Pod Security Standards checks (the subset a GPU workload meets) for ``level``:
    ``privileged`` allows everything, ``baseline`` and ``restricted`` as documented."""
    if level not in ("baseline", "restricted"):
        return []
    spec = pod.get("spec") or {}
    containers = list(spec.get("initContainers") or []) + list(spec.get("containers") or [])
    out: List[str] = []
    for f in ("hostNetwork", "hostPID", "hostIPC"):
        if spec.get(f):
            out.append(f"host namespaces ({f}=true)")
    host_path = [v.get("name") for v in spec.get("volumes") or [] if "hostPath" in v]
    if host_path:
        out.append("hostPath volumes (" + ", ".join(f'volume "{n}"' for n in host_path) + ")")
    for c in containers:
        sc = c.get("securityContext") or {}
        if sc.get("privileged"):
            out.append(f'privileged (container "{c.get("name")}")')
        added = set(((sc.get("capabilities") or {}).get("add")) or [])
        if added - _BASELINE_CAPS:
            out.append(f'non-default capabilities (container "{c.get("name")}")')
        if any(p.get("hostPort") for p in c.get("ports") or []):
            out.append(f'hostPort (container "{c.get("name")}")')
    if level == "restricted":
        psc = spec.get("securityContext") or {}
        bad_vol = [v.get("name") for v in spec.get("volumes") or []
                   if not (set(v) - {"name"}) & _RESTRICTED_VOLUMES]
        if bad_vol:
            out.append("restricted volume types (" + ", ".join(f'volume "{n}"' for n in bad_vol) + ")")
        for c in containers:
            sc = c.get("securityContext") or {}
            name = c.get("name")
            if sc.get("allowPrivilegeEscalation") is not False:
                out.append(f'allowPrivilegeEscalation != false (container "{name}")')
            if "ALL" not in (((sc.get("capabilities") or {}).get("drop")) or []):
                out.append(f'unrestricted capabilities (container "{name}" must drop ALL)')
            if not (sc.get("runAsNonRoot", psc.get("runAsNonRoot"))):
                out.append(f'runAsNonRoot != true (container "{name}")')
            prof = (sc.get("seccompProfile") or psc.get("seccompProfile") or {}).get("type")
            if prof not in ("RuntimeDefault", "Localhost"):
                out.append(f'seccompProfile (container "{name}" must be RuntimeDefault or Localhost)')
    return out


def _ns_selected(selector: Dict[str, Any], labels: Dict[str, str]) -> bool:
    """A namespaceSelector against the namespace's labels."""
    for k, v in (selector.get("matchLabels") or {}).items():
        if labels.get(k) != v:
            return False
    for e in selector.get("matchExpressions") or []:
        have = labels.get(e.get("key"))
        op, vals = e.get("operator"), e.get("values") or []
        if (op == "In" and have not in vals) or (op == "NotIn" and have in vals) \
                or (op == "Exists" and have is None) or (op == "DoesNotExist" and have is not None):
            return False
    return True


def _rule_matches(rule: Dict[str, Any]) -> bool:
    def has(key: str, want: str) -> bool:
        vals = rule.get(key) or []
        return "*" in vals or want in vals

    return has("operations", "CREATE") and has("apiGroups", "") and has("apiVersions", "v1") \
        and has("resources", "pods")


def _call_webhook(fake: "FakeRancher", hook: Dict[str, Any], review: Dict[str, Any]) -> Dict[str, Any]:
    cc = hook.get("clientConfig") or {}
    svc = cc.get("service") or {}
    base = fake.service_endpoints.get(f"{svc.get('name')}.{svc.get('namespace')}")
    if base is None:
        raise ConnectionError(f"service {svc.get('name')}.{svc.get('namespace')} has no endpoints")
    u = urllib.parse.urlsplit(base)
    ctx = ssl.create_default_context(cadata=base64.b64decode(cc.get("caBundle", "")).decode())
    raw = socket.create_connection((u.hostname, u.port), timeout=float(hook.get("timeoutSeconds", 10)))
    conn = http.client.HTTPConnection(u.hostname, u.port)
    conn.sock = ctx.wrap_socket(raw, server_hostname=f"{svc['name']}.{svc['namespace']}.svc")
    try:
        data = json.dumps(review).encode()
        conn.request("POST", svc.get("path", "/"), body=data, headers={"Content-Type": "application/json"})
        resp = conn.getresponse()
        out = resp.read()
        if resp.status != 200:
            raise ConnectionError(f"webhook HTTP {resp.status}")
        return json.loads(out)
    finally:
        conn.close()


def _admit_pod(fake: "FakeRancher", cid: str, namespace: str, pod: Dict[str, Any]) -> Dict[str, Any]:
    from ..k8s.webhook import apply_patch

    st = fake.state
    prefix = f"{cid}|/apis/admissionregistration.k8s.io/v1/mutatingwebhookconfigurations|"
    with st.mu:
        configs = [st.objects[k] for k in st.cluster_objects.get(cid, ()) if k.startswith(prefix)]
    for cfg in configs:
        for hook in cfg.get("webhooks") or []:
            if not any(_rule_matches(r) for r in hook.get("rules") or []):
                continue
            if not _ns_selected(hook.get("namespaceSelector") or {}, fake.namespace_labels(cid, namespace)):
                continue
            review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                      "request": {"uid": str(uuid.uuid4()), "kind": {"group": "", "version": "v1", "kind": "Pod"},
                                  "operation": "CREATE", "namespace": namespace, "object": pod}}
            try:
                resp = _call_webhook(fake, hook, review).get("response") or {}
            except (OSError, ValueError, ssl.SSLError) as exc:
                if hook.get("failurePolicy", "Fail") == "Fail":
                    raise _Rejected(f"failed calling webhook {hook.get('name')}: {exc}") from exc
                continue
            if not resp.get("allowed", False):
                raise _Rejected(f"admission webhook {hook.get('name')} denied the request")
            if resp.get("patch"):
                pod = apply_patch(pod, json.loads(base64.b64decode(resp["patch"])))
    return pod


def tunnel_params(hostname: str, roles: Dict[str, bool], labels: Dict[str, str],
                  capacity: Dict[str, Any], taints: Optional[List[Dict[str, str]]] = None) -> str:
    """The ``X-API-Tunnel-Params`` header a node agent sends (base64 JSON).  ``capacity``
    carries the node's GPU devices (``amd.com/gpu``: what a device plugin on it would
    enumerate), not what the kubelet advertises."""
    node = {"requestedHostname": hostname, "etcd": roles.get("etcd", False),
            "controlPlane": roles.get("controlplane", False), "worker": roles.get("worker", False),
            "labels": labels, "capacity": capacity, "taints": list(taints or [])}
    return base64.b64encode(json.dumps({"node": node}).encode()).decode()
