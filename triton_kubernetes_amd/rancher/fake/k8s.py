"""Kubernetes core API of the fake Rancher's downstream clusters (``/k8s/clusters/<id>/...``).

Rancher proxies each downstream cluster's API server under ``/k8s/clusters/<cluster id>``;
this module is that API server, as far as the framework talks to it:

* ``GET api/v1/nodes`` -- the registered nodes as the kubelets report them: labels (the
  agent's plus ``kubernetes.io/hostname`` and ``node-role.kubernetes.io/<role>``), taints,
  the ``Ready`` condition once the RKE simulation made the node active, ``kubeletVersion``
  (the cluster's running version: upstream ``vX.Y.Z`` for RKE1) and allocatable resources;
* ``PATCH api/v1/nodes/<name>`` -- JSON merge patch: labels merge (``null`` deletes),
  ``spec.taints`` replaced, ``spec.unschedulable``; a ``metadata.resourceVersion`` in the
  patch is a precondition (409 ``Conflict`` when the node changed meanwhile);
* ``GET api/v1/pods?fieldSelector=spec.nodeName=<n>`` and the ``eviction`` subresource (a pod
  annotated :attr:`K8sCoreApi.PDB_ANNOTATION` answers 429 as a PodDisruptionBudget would);
* ``GET version``;
* a generic object store for everything else (create, get, list, replace, delete) with the
  server-populated metadata a real API server adds (``uid``, ``resourceVersion``,
  ``creationTimestamp``).  Pod creates go through admission (``admission.py``);
* the kubelet's device-plugin model: ``amd.com/gpu`` appears in a node's capacity and
  allocatable only when a device-plugin DaemonSet pod runs on it and has registered.  A
  DaemonSet counts as the AMD GPU plugin when a container runs a ``rocm/k8s-device-plugin``
  image (not the labeller tag) and mounts the host's ``/var/lib/kubelet/device-plugins``
  and ``/sys``.  Its pod lands on a node only if the node is Ready, its labels satisfy the
  ``nodeSelector`` and required node affinity, and the pod tolerates the node's taints;
  it registers ``device_plugin_seconds`` after both exist.  DaemonSet reads carry
  ``status`` (``desiredNumberScheduled``, ``numberReady``).

Refusals, as a real API server words them (negative tests in
``tests/test_fake_rancher_contract.py``, ``test_k8s_*``):

* unknown cluster -> 404; unknown object on get/replace/delete/evict/patch -> 404;
* create without ``metadata.name`` or ``generateName`` -> 422 ``Invalid``; a name already
  taken -> 409 ``AlreadyExists``;
* a namespaced create into a namespace that does not exist -> 404 ``NotFound``
  (``default``, ``kube-system``, ``kube-public``, ``kube-node-lease`` and
  ``cattle-system`` exist from the start, as on a Rancher-managed cluster);
* a body whose ``metadata.namespace`` or (on replace) ``metadata.name`` differs from the
  URL -> 400 ``BadRequest``;
* replace or merge-patch carrying a stale ``metadata.resourceVersion`` -> 409 ``Conflict``;
* a Namespace whose ``pod-security.kubernetes.io/enforce`` label is not a Pod Security
  level -> 403 ``Forbidden`` (the PodSecurity admission plugin checks namespace labels);
* a MutatingWebhookConfiguration that admissionregistration/v1 validation refuses (a webhook
  name that is not fully qualified or repeats, ``sideEffects`` other than None /
  NoneOnDryRun, no v1/v1beta1 ``admissionReviewVersions``, a ``clientConfig`` without
  exactly one of url / service, an unknown ``failurePolicy``) -> 422 ``Invalid``;
* a DaemonSet / Deployment without a ``spec.selector`` matching its template's labels, a
  Job whose template's ``restartPolicy`` is not Never / OnFailure, or a pod template
  without named containers with images -> 422 ``Invalid``;
* Secret data that is not base64, a TLS Secret without ``tls.crt`` / ``tls.key``, a
  service-account token Secret without ``kubernetes.io/service-account.name``, ConfigMap /
  Secret keys outside ``[-._a-zA-Z0-9]``, Service ports outside 1-65535, a (Cluster)RoleBinding
  without a complete ``roleRef`` -> 422 ``Invalid``;
* a merge patch that is not a JSON object -> 400.
"""

import base64
import binascii
import json
import re
import time
import uuid
from typing import Any, Dict, List, Optional, Tuple

from ...versions import DEFAULT_K8S_VERSION
from .admission import PSA_ENFORCE, PSA_LEVELS, WEBHOOK_CONFIGS, admit_pod

DEVICE_PLUGIN_REPOS = ("rocm/k8s-device-plugin", "docker.io/rocm/k8s-device-plugin")
DEVICE_PLUGIN_SOCKET_DIR = "/var/lib/kubelet/device-plugins"
# namespaces a Rancher-managed cluster has before anything is applied
INITIAL_NAMESPACES = ("default", "kube-system", "kube-public", "kube-node-lease", "cattle-system")
NAMESPACES = "/api/v1/namespaces"

Reply = Tuple[int, Any]


def _status(code: int, reason: str, message: str = "") -> Reply:
    return code, {"kind": "Status", "apiVersion": "v1", "status": "Failure", "reason": reason, "code": code,
                  "message": message}


def match_expressions(exprs: List[Dict[str, Any]], labels: Dict[str, str]) -> bool:
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


def tolerated(taint: Dict[str, Any], tolerations: List[Dict[str, Any]]) -> bool:
    for t in tolerations:
        if t.get("effect") and t.get("effect") != taint.get("effect"):
            continue
        if t.get("operator") == "Exists" and (not t.get("key") or t.get("key") == taint.get("key")):
            return True
        if t.get("key") == taint.get("key") and t.get("value", "") == taint.get("value", ""):
            return True
    return False


def _webhook_config_problem(cfg: Dict[str, Any]) -> str:
    """What admissionregistration.k8s.io/v1 validation refuses in a
    MutatingWebhookConfiguration ("" when valid): per webhook a fully qualified name,
    ``sideEffects`` None/NoneOnDryRun, ``admissionReviewVersions`` naming v1 or v1beta1, and
    a ``clientConfig`` with exactly one of ``url`` / ``service``."""
    names = set()
    for i, hook in enumerate(cfg.get("webhooks") or []):
        at = f"webhooks[{i}]"
        name = str(hook.get("name", ""))
        if name.count(".") < 2:
            return f'{at}.name: Invalid value: "{name}": should be a domain with at least three segments'
        if name in names:
            return f'{at}.name: Duplicate value: "{name}"'
        names.add(name)
        if hook.get("sideEffects") not in ("None", "NoneOnDryRun"):
            return f"{at}.sideEffects: Required value: must be one of None, NoneOnDryRun"
        versions = hook.get("admissionReviewVersions") or []
        if not any(v in ("v1", "v1beta1") for v in versions):
            return f"{at}.admissionReviewVersions: Required value: must include at least one of v1, v1beta1"
        cc = hook.get("clientConfig") or {}
        if ("url" in cc) == ("service" in cc):
            return f"{at}.clientConfig: Required value: exactly one of url or service is required"
        if hook.get("failurePolicy", "Fail") not in ("Fail", "Ignore"):
            return f"{at}.failurePolicy: Unsupported value: \"{hook.get('failurePolicy')}\""
    return ""


def _workload_problem(kind: str, obj: Dict[str, Any]) -> str:
    """What apps/v1 and batch/v1 validation refuses in a DaemonSet / Deployment / Job ("" when
    valid): a pod template with containers that each have a name and an image; for
    DaemonSets and Deployments a ``spec.selector`` whose ``matchLabels`` the template's labels
    carry; for Jobs a ``restartPolicy`` of Never or OnFailure."""
    spec = obj.get("spec") or {}
    tmpl = spec.get("template") or {}
    pod = tmpl.get("spec") or {}
    containers = pod.get("containers") or []
    if not containers:
        return "spec.template.spec.containers: Required value"
    for i, c in enumerate(containers):
        if not c.get("name") or not c.get("image"):
            return f"spec.template.spec.containers[{i}]: Required value: name and image"
    if kind in ("daemonsets", "deployments"):
        sel = (spec.get("selector") or {}).get("matchLabels") or {}
        if not sel and not (spec.get("selector") or {}).get("matchExpressions"):
            return "spec.selector: Required value"
        labels = (tmpl.get("metadata") or {}).get("labels") or {}
        if any(labels.get(k) != v for k, v in sel.items()):
            return "spec.template.metadata.labels: Invalid value: `selector` does not match template `labels`"
    if kind == "jobs" and pod.get("restartPolicy") not in ("Never", "OnFailure"):
        return (f'spec.template.spec.restartPolicy: Required value: valid values: "OnFailure", "Never" '
                f'(got {pod.get("restartPolicy")!r})')
    return ""


_DATA_KEY_RE = re.compile(r"^[-._a-zA-Z0-9]+$")


def _core_problem(kind: str, obj: Dict[str, Any]) -> str:
    """What core/v1 and rbac/v1 validation refuses in the other objects the add-ons apply
    ("" when valid): Secret ``data`` that is not base64, a ``kubernetes.io/tls`` Secret
    without ``tls.crt`` / ``tls.key``, a service-account token Secret without its
    service-account annotation, ConfigMap / Secret keys outside ``[-._a-zA-Z0-9]``, Service
    ports outside 1-65535, and (Cluster)RoleBindings without a complete ``roleRef``."""
    if kind in ("secrets", "configmaps"):
        for field in ("data", "binaryData") if kind == "configmaps" else ("data", "stringData"):
            for key in (obj.get(field) or {}):
                if not _DATA_KEY_RE.fullmatch(str(key)):
                    return f"{field}[{key}]: Invalid value: a valid config key must consist of alphanumeric characters, '-', '_' or '.'"
    if kind == "secrets":
        data = obj.get("data") or {}
        for key, val in data.items():
            try:
                base64.b64decode(str(val), validate=True)
            except (ValueError, binascii.Error):
                return f"data[{key}]: Invalid value: illegal base64 data"
        have = set(data) | set(obj.get("stringData") or {})
        if obj.get("type") == "kubernetes.io/tls":
            for key in ("tls.crt", "tls.key"):
                if key not in have:
                    return f"data[{key}]: Required value"
        if obj.get("type") == "kubernetes.io/service-account-token" and not (
                (obj.get("metadata") or {}).get("annotations") or {}).get("kubernetes.io/service-account.name"):
            return "metadata.annotations[kubernetes.io/service-account.name]: Required value"
    if kind == "services":
        for i, port in enumerate((obj.get("spec") or {}).get("ports") or []):
            if not 1 <= int(port.get("port", 0) or 0) <= 65535:
                return f"spec.ports[{i}].port: Invalid value: must be between 1 and 65535, inclusive"
    if kind in ("rolebindings", "clusterrolebindings"):
        ref = obj.get("roleRef") or {}
        for key in ("apiGroup", "kind", "name"):
            if not ref.get(key):
                return f"roleRef.{key}: Required value"
    return ""


def _namespace_of(kpath: str) -> Optional[str]:
    """``ns`` of ``/api/v1/namespaces/<ns>/...`` or ``/apis/<g>/<v>/namespaces/<ns>/...``."""
    parts = kpath.strip("/").split("/")
    for i in (2, 3):
        if len(parts) > i + 1 and parts[i] == "namespaces":
            return parts[i + 1]
    return None


def _is_collection(kpath: str) -> bool:
    """``/api/v1/<res>``, ``/api/v1/namespaces/<ns>/<res>`` and their ``/apis/<group>/<v>``
    forms name a collection; one more segment names an object."""
    parts = kpath.strip("/").split("/")
    rest = parts[2:] if parts[:1] == ["api"] else parts[3:]
    return len(rest) == 1 or (len(rest) == 3 and rest[0] == "namespaces")


class K8sCoreApi:
    """Mixin of :class:`~.server.FakeRancher`: the downstream clusters' API servers."""

    # a pod annotated with this many refusals answers 429 (a PodDisruptionBudget at its
    # minimum) that many times before the eviction goes through; "always" never does
    PDB_ANNOTATION = "fake.triton-kubernetes.io/pdb-refusals"

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
        if terms and not any(match_expressions(t.get("matchExpressions") or [], labels) for t in terms):
            return False
        tolerations = pod.get("tolerations") or []
        scheduled = max(self.state.object_times.get(ds_key, 0.0), n.get("ready_at") or 0.0)
        added = n.get("taint_added") or {}
        return all(tolerated(t, tolerations) for t in n.get("taints") or []
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

    def namespace_labels(self, cid: str, namespace: str) -> Dict[str, str]:
        """Labels of a Namespace created through the proxy (+ the automatic name label)."""
        with self.state.mu:
            ns = self.state.objects.get(f"{cid}|{NAMESPACES}|{namespace}") or {}
        labels = dict((ns.get("metadata") or {}).get("labels") or {})
        labels["kubernetes.io/metadata.name"] = namespace
        return labels

    def _namespace_exists(self, cid: str, namespace: str) -> bool:
        return namespace in INITIAL_NAMESPACES or f"{cid}|{NAMESPACES}|{namespace}" in self.state.objects

    # --- HTTP ---------------------------------------------------------------------------------
    def _route_k8s(self, method: str, path: str, query: Dict[str, List[str]], body: Any) -> Optional[Reply]:
        if not path.startswith("/k8s/clusters/"):
            return None
        return self._k8s(method, path, body, query)

    def _k8s(self, method: str, path: str, body: Any, query: Optional[Dict[str, List[str]]] = None) -> Reply:
        st = self.state
        rest = path[len("/k8s/clusters/"):]
        cid, _, kpath = rest.partition("/")
        with st.mu:
            if cid not in st.clusters:
                return _status(404, "NotFound", f'cluster "{cid}" not found')
        kpath = "/" + kpath
        parts = kpath.strip("/").split("/")
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
        if (method == "POST" and len(parts) == 7 and parts[:3] == ["api", "v1", "namespaces"] and parts[4] == "pods"
                and parts[6] == "eviction"):
            return self._evict(cid, parts[3], parts[5])
        if kpath == "/version":
            with st.mu:
                v = (st.clusters[cid].get("version") or {}).get("gitVersion") or DEFAULT_K8S_VERSION
            major, minor = v.lstrip("v").split(".")[:2]
            return 200, {"major": major, "minor": minor, "gitVersion": v.split("-")[0].split("+")[0]}
        if method == "POST":
            return self._create(cid, kpath, body)
        if method == "PUT":
            return self._replace(cid, kpath, body)
        if method in ("GET", "DELETE"):
            base, _, name = kpath.rpartition("/")
            key = f"{cid}|{base}|{name}"
            with st.mu:
                if method == "DELETE":
                    if key not in st.objects:
                        return _status(404, "NotFound", f'"{name}" not found')
                    st.cluster_objects.get(cid, {}).pop(key, None)
                    st.object_times.pop(key, None)
                    return 200, st.objects.pop(key)
                if key in st.objects:
                    if base.endswith("/daemonsets"):
                        return 200, dict(st.objects[key], status=self._daemonset_status(cid, key, st.objects[key]))
                    return 200, st.objects[key]
                if not _is_collection(kpath):
                    return _status(404, "NotFound", f'"{name}" not found')
                prefix = f"{cid}|{kpath}|"
                items = [st.objects[k] for k in st.cluster_objects.get(cid, ()) if k.startswith(prefix)]
                return 200, {"items": items}
        return _status(405, "MethodNotAllowed", f"{method} {kpath}")

    def _check_object(self, cid: str, kpath: str, body: Any) -> Optional[Reply]:
        """Refusals common to create and replace (see the module docstring); ``kpath`` is
        the collection.  Placement (request body, namespace) first, then content."""
        return self._check_placement(cid, kpath, body) or self._check_content(kpath, body)

    def _check_placement(self, cid: str, kpath: str, body: Any) -> Optional[Reply]:
        if not isinstance(body, dict):
            return _status(400, "BadRequest", "the request body must be an object")
        meta = body.get("metadata") or {}
        ns = _namespace_of(kpath)
        if ns is not None:
            if meta.get("namespace") not in (None, "", ns):
                return _status(400, "BadRequest", "the namespace of the provided object does not match the "
                                                  "namespace sent on the request")
            with self.state.mu:
                if not self._namespace_exists(cid, ns):
                    return _status(404, "NotFound", f'namespaces "{ns}" not found')
        return None

    @staticmethod
    def _check_content(kpath: str, body: Dict[str, Any]) -> Optional[Reply]:
        """What validation and admission refuse in the object itself (after the API server
        found where it goes and, on replace, that it exists and is current)."""
        meta = body.get("metadata") or {}
        kind = kpath.rstrip("/").rsplit("/", 1)[-1]
        problem = _core_problem(kind, body)
        if problem:
            return _status(422, "Invalid", f'{kind[:-1]} "{meta.get("name", "")}" is invalid: {problem}')
        if kind in ("daemonsets", "deployments", "jobs"):
            problem = _workload_problem(kind, body)
            if problem:
                return _status(422, "Invalid", f'{kind[:-1]} "{meta.get("name", "")}" is invalid: {problem}')
        if kpath.rstrip("/") == WEBHOOK_CONFIGS:
            problem = _webhook_config_problem(body)
            if problem:
                return _status(422, "Invalid", f'MutatingWebhookConfiguration.admissionregistration.k8s.io '
                                               f'"{meta.get("name", "")}" is invalid: {problem}')
        if kpath.rstrip("/") == NAMESPACES:
            level = (meta.get("labels") or {}).get(PSA_ENFORCE)
            if level is not None and level not in PSA_LEVELS:
                return _status(403, "Forbidden", f'namespaces "{meta.get("name", "")}" is forbidden: invalid '
                                                 f'{PSA_ENFORCE} label value "{level}": must be one of '
                                                 + ", ".join(PSA_LEVELS))
        return None

    def _create(self, cid: str, kpath: str, body: Any) -> Reply:
        st = self.state
        bad = self._check_object(cid, kpath, body)
        if bad is not None:
            return bad
        meta = body.get("metadata") or {}
        name = meta.get("name") or (meta.get("generateName", "") + uuid.uuid4().hex[:5] if meta.get("generateName")
                                    else "")
        if not name:
            return _status(422, "Invalid", "metadata.name: Required value: name or generateName is required")
        parts = kpath.strip("/").split("/")
        if len(parts) == 5 and parts[:3] == ["api", "v1", "namespaces"] and parts[4] == "pods":
            body, refused = admit_pod(self, cid, parts[3], body)
            if refused is not None:
                return refused
        key = f"{cid}|{kpath}|{name}"
        with st.mu:
            if key in st.objects:
                return _status(409, "AlreadyExists", f'"{name}" already exists')
            # server-populated fields, as a real API server adds them
            obj = json.loads(json.dumps(body))
            m = obj.setdefault("metadata", {})
            m["name"] = name
            ns = _namespace_of(kpath)
            if ns is not None:
                m["namespace"] = ns
            m.update({"uid": str(uuid.uuid4()), "resourceVersion": self._next_rv(),
                      "creationTimestamp": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())})
            obj.setdefault("status", {})
            st.objects[key] = obj
            st.object_times[key] = time.time()
            st.cluster_objects.setdefault(cid, {})[key] = None
        return 201, obj

    def _replace(self, cid: str, kpath: str, body: Any) -> Reply:
        st = self.state
        base, _, name = kpath.rpartition("/")
        # as the API server orders them: request (400), existence (404), precondition (409),
        # then validation and admission of the new content (422 / 403)
        bad = self._check_placement(cid, base, body)
        if bad is not None:
            return bad
        meta = body.get("metadata") or {}
        if meta.get("name") not in (None, "", name):
            return _status(400, "BadRequest", f'the name of the object ({meta.get("name")}) does not match the '
                                              f"name on the URL ({name})")
        key = f"{cid}|{base}|{name}"
        with st.mu:
            cur = st.objects.get(key)
            if cur is None:
                return _status(404, "NotFound", f'"{name}" not found')
            cur_meta = cur.get("metadata") or {}
            want = meta.get("resourceVersion")
            if want not in (None, "") and str(want) != str(cur_meta.get("resourceVersion")):
                return _status(409, "Conflict", f'Operation cannot be fulfilled on "{name}": the object has been '
                                                "modified; please apply your changes to the latest version and "
                                                "try again")
            bad = self._check_content(base, body)
            if bad is not None:
                return bad
            obj = json.loads(json.dumps(body))
            m = obj.setdefault("metadata", {})
            m.update(name=name, uid=cur_meta.get("uid"), creationTimestamp=cur_meta.get("creationTimestamp"),
                     resourceVersion=self._next_rv())
            if "namespace" in cur_meta:
                m["namespace"] = cur_meta["namespace"]
            st.objects[key] = obj
        return 200, obj

    def _next_rv(self) -> str:
        st = self.state
        with st.mu:
            st.rv_seq += 1
            return str(st.rv_seq)

    def _patch_node(self, cid: str, name: str, patch: Any) -> Reply:
        """JSON merge patch of a Node: labels merge (null deletes), ``spec.taints`` replaced."""
        st = self.state
        if not isinstance(patch, dict):
            return _status(400, "BadRequest", "merge patch must be an object")
        now = time.time()
        with st.mu:
            node = next((n for n in st.cluster_nodes.get(cid, {}).values() if n["hostname"] == name), None)
            if node is None:
                return _status(404, "NotFound", f'nodes "{name}" not found')
            # optimistic concurrency: a patch naming a resourceVersion applies to that one only
            want = (patch.get("metadata") or {}).get("resourceVersion")
            if want is not None and str(want) != str(node.get("rv", 1)):
                return _status(409, "Conflict", f'Operation cannot be fulfilled on nodes "{name}": the object has '
                                                "been modified; please apply your changes to the latest version "
                                                "and try again")
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

    def _evict(self, cid: str, namespace: str, name: str) -> Reply:
        """The Eviction subresource: the pod is deleted unless its budget refuses (429)."""
        st = self.state
        key = f"{cid}|/api/v1/namespaces/{namespace}/pods|{name}"
        with st.mu:
            pod = st.objects.get(key)
            if pod is None:
                return _status(404, "NotFound", f'pods "{name}" not found')
            ann = (pod.get("metadata") or {}).setdefault("annotations", {})
            left = ann.get(self.PDB_ANNOTATION)
            if left == "always" or (left and int(left) > 0):
                if left != "always":
                    ann[self.PDB_ANNOTATION] = str(int(left) - 1)
                st.evictions_refused += 1
                return _status(429, "TooManyRequests", "Cannot evict pod as it would violate the pod's "
                                                       "disruption budget.")
            st.objects.pop(key)
            st.object_times.pop(key, None)
            st.cluster_objects.get(cid, {}).pop(key, None)
        return 201, {"kind": "Status", "status": "Success", "code": 201}


__all__ = ["K8sCoreApi", "DEVICE_PLUGIN_REPOS", "DEVICE_PLUGIN_SOCKET_DIR", "INITIAL_NAMESPACES",
           "match_expressions", "tolerated"]
