"""RCCL-env injector: a mutating admission webhook for GPU pods.

Every pod that requests ``amd.com/gpu`` (limits or requests, any container or init
container) gets, at admission time:

* the cluster's RCCL/HSA environment (the ``rccl-env`` ConfigMap, mounted into the
  webhook's pod as files and re-read on every request) as literal ``env`` entries on each
  GPU container -- a variable the container already sets wins, so a workload can
  override any value;
* the node's own ``/etc/rccl`` (written by the node bootstrap: discovered RDMA ports,
  per-node overrides) mounted read-only at ``/etc/rccl`` plus ``TK_RCCL_ENV_FILE``
  pointing at ``/etc/rccl/rccl.env``, so launchers can source the node values on top;
* the annotation ``amd.com/rccl-env: injected``;
* xGMI-aware placement (the BASELINE north star's "xGMI-topology-aware pod affinity"):
  a pod asking for 2+ GPUs must land on a node whose GPUs form one fully connected xGMI
  hive (``amd.com/xgmi.fully-connected=true``, added to every required node-selector term,
  so a pod's own terms still apply), and pods sharing an ``amd.com/xgmi-group`` label
  prefer the same hive (pod affinity on ``amd.com/xgmi.hive-id``).

Pod Security Admission runs *after* mutating webhooks, and its ``baseline`` and
``restricted`` levels forbid ``hostPath`` volumes: mounting ``/etc/rccl`` into a pod in
such a namespace would get the pod rejected for a change it never asked for.  A
namespace's label does not say which level applies to it: clusters that enforce Pod
Security by default (an API-server ``AdmissionConfiguration`` default -- Rancher's
``rancher-restricted`` PSA template, RKE2's CIS profile) apply it to every *unlabelled*
namespace.  So the ``hostPath`` is opt-in, and the add-ons register the injector three
times (``k8s/addons.py``), split by namespace label:

* ``amd.com/rccl-node-env=true`` or ``pod-security.kubernetes.io/enforce=privileged``:
  served on ``/mutate`` -- the cluster env plus the node's ``/etc/rccl``;
* every other namespace: served on ``/mutate?node-env=omit`` -- the cluster env, the
  placement, no ``hostPath``, no ``TK_RCCL_ENV_FILE``, and the annotation
  ``amd.com/rccl-env-node: omitted (...)`` saying how to opt in.

A pod opts out of the env with the annotation ``amd.com/rccl-env-inject: "false"`` and of
the placement with ``amd.com/xgmi-placement: "false"``.  The
ConfigMap lives in ``kube-system``; ``envFrom`` cannot reach across namespaces, which
is why the values are injected literally.

This replaces round 1's opt-in ``envFrom`` + wrapper in the example Job
(``manifests.gpu_job_manifest``): the BASELINE north star asks for the RCCL env on
every GPU workload, not only on Jobs that know about it.

The module is deliberately stdlib-only and self-contained: the add-on manifests ship
its source text in a ConfigMap and run it with a pinned Python image
(``versions.WEBHOOK_IMAGE``); ``python webhook.py --cert ... --key ... --env-dir ...``.
"""

import base64
import json
import os
import ssl
import sys
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional

GPU_RESOURCE = "amd.com/gpu"


class _Server(ThreadingHTTPServer):
    """Listen backlog of the system's somaxconn, not socketserver's 5 (utils/httpserver.py;
    this file stays standalone: the injector pod runs it by itself)."""
    request_queue_size = 4096
OPT_OUT = "amd.com/rccl-env-inject"
MARK = "amd.com/rccl-env"
VOLUME = "tk-node-rccl-env"
NODE_DIR = "/etc/rccl"
ENV_FILE_VAR = "TK_RCCL_ENV_FILE"
NODE_ENV_MARK = "amd.com/rccl-env-node"
PSA_LABEL = "pod-security.kubernetes.io/enforce"
NODE_ENV_OPT_IN = "amd.com/rccl-node-env"  # namespace label: "true" = mount the node's /etc/rccl
PLACEMENT_OPT_OUT = "amd.com/xgmi-placement"
GROUP_LABEL = "amd.com/xgmi-group"
HIVE_KEY = "amd.com/xgmi.hive-id"
FULLY_CONNECTED = {"key": "amd.com/xgmi.fully-connected", "operator": "In", "values": ["true"]}


def _esc(key: str) -> str:
    """JSON-pointer escaping of one path segment (RFC 6901)."""
    return key.replace("~", "~0").replace("/", "~1")


def _wants_gpu(container: Dict[str, Any]) -> bool:
    res = container.get("resources") or {}
    for part in ("limits", "requests"):
        v = (res.get(part) or {}).get(GPU_RESOURCE)
        if v is not None:
            try:
                if int(str(v)) > 0:
                    return True
            except ValueError:
                return True  # a quantity we cannot parse still asks for GPUs
    return False


def _gpu_count(container: Dict[str, Any]) -> int:
    res = container.get("resources") or {}
    for part in ("limits", "requests"):
        v = (res.get(part) or {}).get(GPU_RESOURCE)
        if v is not None:
            try:
                return int(str(v))
            except ValueError:
                return 0
    return 0


def placement_affinity(pod: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    """The pod's ``spec.affinity`` with the xGMI placement added; None when nothing changes."""
    meta = pod.get("metadata") or {}
    if str((meta.get("annotations") or {}).get(PLACEMENT_OPT_OUT, "")).lower() == "false":
        return None
    spec = pod.get("spec") or {}
    # GPUs the pod holds at once: its app containers together, or its largest init container
    gpus = max(sum(_gpu_count(c) for c in spec.get("containers") or []),
               max([_gpu_count(c) for c in spec.get("initContainers") or []], default=0))
    group = (meta.get("labels") or {}).get(GROUP_LABEL)
    if gpus < 2 and not group:
        return None
    aff = json.loads(json.dumps(spec.get("affinity") or {}))
    changed = False
    if gpus >= 2:
        na = aff.setdefault("nodeAffinity", {})
        req = na.setdefault("requiredDuringSchedulingIgnoredDuringExecution", {})
        terms = req.setdefault("nodeSelectorTerms", [])
        if not terms:
            terms.append({})
        for term in terms:  # terms are ORed: the hive constraint goes into each
            exprs = term.setdefault("matchExpressions", [])
            if not any(e.get("key") == FULLY_CONNECTED["key"] for e in exprs):
                exprs.append(dict(FULLY_CONNECTED, values=list(FULLY_CONNECTED["values"])))
                changed = True
    if group:
        pa = aff.setdefault("podAffinity", {})
        pref = pa.setdefault("preferredDuringSchedulingIgnoredDuringExecution", [])
        if not any((t.get("podAffinityTerm") or {}).get("topologyKey") == HIVE_KEY for t in pref):
            pref.append({"weight": 100, "podAffinityTerm": {
                "labelSelector": {"matchLabels": {GROUP_LABEL: group}}, "topologyKey": HIVE_KEY}})
            changed = True
    return aff if changed else None


def load_env(env_dir: str) -> Dict[str, str]:
    """A ConfigMap mounted as a directory: one file per key (``..data`` links skipped)."""
    out: Dict[str, str] = {}
    if not env_dir or not os.path.isdir(env_dir):
        return out
    for name in sorted(os.listdir(env_dir)):
        path = os.path.join(env_dir, name)
        if name.startswith(".") or not os.path.isfile(path):
            continue
        with open(path, "r", encoding="utf-8") as fh:
            out[name] = fh.read()
    return out


def patch_for_pod(pod: Dict[str, Any], env: Dict[str, str], node_env: bool = True) -> List[Dict[str, Any]]:
    """RFC 6902 operations for a pod: the RCCL env on its GPU containers and the xGMI
    placement ([] = nothing to change).  ``node_env`` False: no ``/etc/rccl`` hostPath
    (namespaces whose Pod Security level forbids it)."""
    ops = _env_ops(pod, env, node_env)
    spec = pod.get("spec") or {}
    if any(_wants_gpu(c) for kind in ("initContainers", "containers") for c in spec.get(kind) or []):
        aff = placement_affinity(pod)
        if aff is not None:
            ops.append({"op": "add", "path": "/spec/affinity", "value": aff})
    return ops


def _env_ops(pod: Dict[str, Any], env: Dict[str, str], node_env: bool = True) -> List[Dict[str, Any]]:
    meta = pod.get("metadata") or {}
    annotations = meta.get("annotations") or {}
    if str(annotations.get(OPT_OUT, "")).lower() == "false" or annotations.get(MARK) == "injected":
        return []
    spec = pod.get("spec") or {}
    ops: List[Dict[str, Any]] = []
    touched = False
    for kind in ("initContainers", "containers"):
        for i, c in enumerate(spec.get(kind) or []):
            if not _wants_gpu(c):
                continue
            touched = True
            have = {e.get("name") for e in (c.get("env") or [])}
            add = [{"name": k, "value": v} for k, v in sorted(env.items()) if k not in have]
            if node_env and ENV_FILE_VAR not in have:
                add.append({"name": ENV_FILE_VAR, "value": f"{NODE_DIR}/rccl.env"})
            base = f"/spec/{kind}/{i}"
            if add:
                if c.get("env"):
                    ops += [{"op": "add", "path": f"{base}/env/-", "value": e} for e in add]
                else:
                    ops.append({"op": "add", "path": f"{base}/env", "value": add})
            mounts = c.get("volumeMounts") or []
            if node_env and not any(m.get("mountPath") == NODE_DIR for m in mounts):
                m = {"name": VOLUME, "mountPath": NODE_DIR, "readOnly": True}
                if mounts:
                    ops.append({"op": "add", "path": f"{base}/volumeMounts/-", "value": m})
                else:
                    ops.append({"op": "add", "path": f"{base}/volumeMounts", "value": [m]})
    if not touched:
        return []
    marks = {MARK: "injected"}
    if node_env:
        vol = {"name": VOLUME, "hostPath": {"path": NODE_DIR, "type": "DirectoryOrCreate"}}
        if not any(v.get("name") == VOLUME for v in spec.get("volumes") or []):
            if spec.get("volumes"):
                ops.append({"op": "add", "path": "/spec/volumes/-", "value": vol})
            else:
                ops.append({"op": "add", "path": "/spec/volumes", "value": [vol]})
    else:
        marks[NODE_ENV_MARK] = (f"omitted (the /etc/rccl hostPath is opt-in: label the namespace {NODE_ENV_OPT_IN}=true "
                                f"or {PSA_LABEL}=privileged)")
    if meta.get("annotations"):
        ops += [{"op": "add", "path": f"/metadata/annotations/{_esc(k)}", "value": v} for k, v in marks.items()]
    else:
        ops.append({"op": "add", "path": "/metadata/annotations", "value": marks})
    return ops


def review(doc: Dict[str, Any], env: Dict[str, str], node_env: bool = True) -> Dict[str, Any]:
    """admission.k8s.io/v1 AdmissionReview in -> AdmissionReview response out.  Never
    denies: a pod the injector cannot parse is admitted unchanged."""
    req = doc.get("request") or {}
    resp: Dict[str, Any] = {"uid": req.get("uid", ""), "allowed": True}
    obj = req.get("object")
    if isinstance(obj, dict) and (req.get("kind") or {}).get("kind", "Pod") == "Pod":
        ops = patch_for_pod(obj, env, node_env)
        if ops:
            resp["patchType"] = "JSONPatch"
            resp["patch"] = base64.b64encode(json.dumps(ops).encode()).decode()
    return {"apiVersion": doc.get("apiVersion", "admission.k8s.io/v1"), "kind": "AdmissionReview",
            "response": resp}


def apply_patch(obj: Dict[str, Any], ops: List[Dict[str, Any]]) -> Dict[str, Any]:
    """Apply ``add`` operations (the only kind :func:`patch_for_pod` emits) -- the API
    server's side, for tests and the fake Rancher's admission chain."""
    out = json.loads(json.dumps(obj))
    for op in ops:
        if op["op"] != "add":
            raise ValueError(f"unsupported op {op['op']}")
        parts = [p.replace("~1", "/").replace("~0", "~") for p in op["path"].lstrip("/").split("/")]
        cur: Any = out
        for p in parts[:-1]:
            cur = cur[int(p)] if isinstance(cur, list) else cur.setdefault(p, {})
        last = parts[-1]
        if isinstance(cur, list):
            if last == "-":
                cur.append(op["value"])
            else:
                cur.insert(int(last), op["value"])
        else:
            cur[last] = op["value"]
    return out


def make_server(port: int, env_dir: str, certfile: str = "", keyfile: str = "",
                host: str = "0.0.0.0") -> ThreadingHTTPServer:
    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *args):
            pass

        def _reply(self, code: int, body: bytes, ctype: str = "application/json"):
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def do_GET(self):
            if self.path in ("/healthz", "/readyz"):
                return self._reply(200, b"ok", "text/plain")
            return self._reply(404, b"{}")

        def setup(self):
            # TLS handshake on this connection's thread, with a deadline: one client that
            # connects and stalls cannot block the accept loop (and every other admission)
            if certfile:
                self.request.settimeout(5.0)
                self.request.do_handshake()
                self.request.settimeout(None)
            super().setup()

        def do_POST(self):
            path, _, query = self.path.partition("?")
            if path != "/mutate":
                return self._reply(404, b"{}")
            n = int(self.headers.get("Content-Length") or 0)
            try:
                doc = json.loads(self.rfile.read(n) or b"{}")
                out = review(doc, load_env(env_dir), node_env="node-env=omit" not in query.split("&"))
            except ValueError as exc:
                return self._reply(400, json.dumps({"error": str(exc)}).encode())
            return self._reply(200, json.dumps(out).encode())

    srv = _Server((host, port), H)
    srv.daemon_threads = True
    if certfile:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        ctx.load_cert_chain(certfile, keyfile)
        srv.socket = ctx.wrap_socket(srv.socket, server_side=True, do_handshake_on_connect=False)
    return srv


def main(argv: Optional[List[str]] = None) -> int:
    import argparse

    ap = argparse.ArgumentParser(prog="rccl-env-injector")
    ap.add_argument("--port", type=int, default=8443)
    ap.add_argument("--cert", default="/tls/tls.crt")
    ap.add_argument("--key", default="/tls/tls.key")
    ap.add_argument("--env-dir", default="/etc/rccl-env")
    args = ap.parse_args(argv)
    srv = make_server(args.port, args.env_dir, args.cert, args.key)
    print(json.dumps({"listening": args.port, "env_keys": sorted(load_env(args.env_dir))}), flush=True)
    srv.serve_forever()
    return 0


if __name__ == "__main__":
    sys.exit(main())
