"""Provisioning v1 (Steve) API of the fake Rancher server: RKE2 custom clusters.

* ``GET /v1-rke2-release/releases`` -- the RKE2 releases the server's KDM data offers;
* ``POST /v1/provisioning.cattle.io.clusters`` -- a custom cluster in ``fleet-default``.
  The provisioning controller creates its management cluster (``c-m-…``, reported as
  ``status.clusterName``) after the create returns: the first read after the create sees
  it, so clients poll.  From then on the management cluster behaves like an RKE1 one
  (registration tokens, nodes, the ``/k8s/clusters`` proxy, state);
* ``GET / PUT / DELETE /v1/provisioning.cattle.io.clusters/<namespace>/<name>`` -- read
  (``status.ready`` follows the management cluster), change the Kubernetes release
  (``spec.kubernetesVersion``: the simulated rolling upgrade of ``server._upgrade``),
  delete (with the management cluster and its nodes);
* ``POST /v1/secrets`` -- Secrets of the management cluster (registry credentials, which
  ``rkeConfig.registries.configs.<host>.authConfigSecretName`` refers to);
* ``GET /system-agent-install.sh`` (unauthenticated) -- the node installer: a shell script
  that takes the real installer's flags, checks ``--ca-checksum`` against ``/cacerts`` and
  registers the node (as ``rancher-system-agent``) through ``/v3/connect/register``.  Under
  a ``TK_HOST_ROOT`` it also models the host (``hostsim.py``): it refuses a host still
  holding another cluster's agent or RKE2, and leaves the installation and its uninstallers.

Refusals (negative tests in ``tests/test_fake_rancher_contract.py``, ``test_v1_*``):

* a release outside ``/v1-rke2-release/releases`` or an unknown CNI -> 422;
* registry config with inline credentials (fields the schema lacks) or naming a Secret
  that does not exist in the cluster's namespace -> 422;
* a cluster or Secret without ``metadata.name`` (Secrets: or ``generateName``) -> 422; a
  name already taken -> 409;
* a PUT whose ``metadata.name`` differs from the URL -> 400, whose
  ``metadata.resourceVersion`` is stale -> 409 (objects carry a ``resourceVersion`` that
  every change bumps, the controller's included); a downgrade or a release the server
  does not offer -> 422;
* unknown cluster -> 404.
"""

import base64
import json
import time
import uuid
from typing import Any, Dict, List, Optional, Tuple

from ...versions import FLEET_NAMESPACE, RKE2_CNIS, SYSTEM_AGENT_INSTALL_PATH
from . import hostsim

Reply = Tuple[int, Any]
CLUSTERS = "/v1/provisioning.cattle.io.clusters"
REGISTRY_CONFIG_FIELDS = {"authConfigSecretName", "caBundle", "insecureSkipVerify", "tlsSecretName"}

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
if [ -n "${TK_HOST_ROOT:-}" ]; then  # the host model (rancher/fake/hostsim.py)
@@HOSTSIM@@
fi
params=$(printf '{"node":{"requestedHostname":"%s","etcd":%s,"controlPlane":%s,"worker":%s,"labels":{%s},"taints":[%s]}}' \
  "$name" $etcd $cp $worker "$labels" "$taints" | base64 | tr -d '\n')
curl -fsSk -o /dev/null -X POST -H "X-API-Tunnel-Token: $token" -H "X-API-Tunnel-Params: $params" \
  -H "X-Cattle-Agent-Kind: system-agent" -d '{}' "$server/v3/connect/register" \
  || { echo "system-agent-install: registration with $server failed" >&2; exit 1; }
if [ -n "${TK_HOST_ROOT:-}" ]; then _tk_install_files; fi
""".replace("@@HOSTSIM@@", hostsim.installer_shell().rstrip("\n"))


def _err(code: int, kind: str, message: str = "", **extra: Any) -> Reply:
    return code, dict({"type": "error", "code": kind, "message": message}, **extra)


def _copy(obj: Dict[str, Any]) -> Dict[str, Any]:
    return json.loads(json.dumps(obj))


class ProvisioningApi:
    """Mixin of :class:`~.server.FakeRancher`: ``provisioning.cattle.io/v1`` and friends."""

    def _route_provisioning_public(self, method: str, path: str) -> Optional[Reply]:
        if path == SYSTEM_AGENT_INSTALL_PATH and method == "GET":
            return 200, SYSTEM_AGENT_INSTALL_SCRIPT.encode()
        return None

    def _route_provisioning(self, method: str, path: str, query: Dict[str, List[str]], body: Any) -> Optional[Reply]:
        st = self.state
        if path == "/v1-rke2-release/releases" and method == "GET":
            return 200, {"data": [{"id": v, "version": v, "type": "release"} for v in st.rke2_versions]}
        if path == CLUSTERS and method == "POST":
            return self._create_v2(body)
        if path == "/v1/secrets" and method == "POST":
            return self._create_secret(body)
        if path.startswith(CLUSTERS + "/"):
            return self._v2_cluster(method, path[len(CLUSTERS) + 1:], body)
        return None

    def _create_secret(self, body: Any) -> Reply:
        st = self.state
        meta = dict((body or {}).get("metadata") or {})
        ns = meta.get("namespace") or "default"
        name = meta.get("name") or (meta["generateName"] + uuid.uuid4().hex[:5] if meta.get("generateName") else "")
        if not name:
            return _err(422, "MissingRequired", "metadata.name or metadata.generateName is required",
                        fieldName="metadata.name")
        with st.mu:
            if f"{ns}/{name}" in st.secrets:
                return _err(409, "AlreadyExists", f'secrets "{name}" already exists')
            st.secrets[f"{ns}/{name}"] = dict(body, metadata=dict(meta, name=name, namespace=ns))
            return 201, _copy(st.secrets[f"{ns}/{name}"])

    def _create_v2(self, body: Dict[str, Any]) -> Reply:
        st = self.state
        meta, spec = body.get("metadata") or {}, body.get("spec") or {}
        ns, name = meta.get("namespace") or FLEET_NAMESPACE, meta.get("name", "")
        if not name:
            return _err(422, "MissingRequired", "metadata.name is required", fieldName="metadata.name")
        version = spec.get("kubernetesVersion", "")
        if version not in st.rke2_versions:
            return _err(422, "Invalid", f"{version} is not a supported RKE2 version",
                        fieldName="spec.kubernetesVersion")
        cni = ((spec.get("rkeConfig") or {}).get("machineGlobalConfig") or {}).get("cni", "canal")
        if cni not in RKE2_CNIS:
            return _err(422, "Invalid", f"unsupported cni {cni!r}")
        for host, conf in (((spec.get("rkeConfig") or {}).get("registries") or {}).get("configs") or {}).items():
            unknown = set(conf) - REGISTRY_CONFIG_FIELDS
            ref = conf.get("authConfigSecretName")
            if unknown or (ref and f"{ns}/{ref}" not in st.secrets):
                # the schema has no inline credentials: they live in a Secret of the namespace
                return _err(422, "Invalid", f"registries.configs[{host}]: unknown fields {sorted(unknown)} or "
                                            f"missing secret {ref!r}")
        with st.mu:
            if f"{ns}/{name}" in st.v2_clusters:
                return _err(409, "AlreadyExists", f'clusters.provisioning.cattle.io "{name}" already exists')
            obj = _copy(body)
            obj["metadata"].update(namespace=ns, uid=str(uuid.uuid4()), resourceVersion=self._next_rv())
            obj["status"] = {"ready": False}  # clusterName: filled in by the controllers
            st.v2_clusters[f"{ns}/{name}"] = obj
            return 201, _copy(obj)

    def _v2_cluster(self, method: str, key: str, body: Any = None) -> Reply:
        st = self.state
        with st.mu:
            obj = st.v2_clusters.get(key)
            if obj is None:
                return _err(404, "NotFound", f'clusters.provisioning.cattle.io "{key}" not found')
            if method == "PUT":
                meta = (body or {}).get("metadata") or {}
                name = key.rpartition("/")[2]
                if meta.get("name") not in (None, "", name):
                    return _err(400, "BadRequest", f"the name of the object ({meta.get('name')}) does not match "
                                                   f"the name on the URL ({name})")
                want = meta.get("resourceVersion")
                if want not in (None, "") and str(want) != str(obj["metadata"].get("resourceVersion")):
                    return _err(409, "Conflict", f'Operation cannot be fulfilled on clusters.provisioning.cattle.io '
                                                 f'"{name}": the object has been modified; please apply your '
                                                 "changes to the latest version and try again")
                code, out = self._upgrade(obj["status"].get("clusterName", ""), body, v2=obj)
                if code == 200:
                    obj["metadata"]["resourceVersion"] = out["metadata"]["resourceVersion"] = self._next_rv()
                return code, out
            if method == "DELETE":
                st.v2_clusters.pop(key)
                cid = obj["status"].get("clusterName")
                if cid:
                    st.clusters.pop(cid, None)
                    for nid in st.cluster_nodes.pop(cid, {}):
                        st.nodes.pop(nid, None)
                return 200, {}
            if method != "GET":
                return _err(405, "MethodNotAllowed", method)
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
                obj["metadata"]["resourceVersion"] = self._next_rv()
                return 200, _copy(obj)
            cid = obj["status"]["clusterName"]
        self._refresh()
        with st.mu:
            ready = (st.clusters.get(cid) or {}).get("state") == "active"
            if ready != obj["status"].get("ready"):
                obj["status"]["ready"] = ready
                obj["metadata"]["resourceVersion"] = self._next_rv()
            return 200, _copy(obj)

    def registry_auth(self, secret: str, namespace: str = FLEET_NAMESPACE) -> Dict[str, str]:
        """Decoded ``username``/``password`` of a registry basic-auth Secret."""
        with self.state.mu:
            data = (self.state.secrets.get(f"{namespace}/{secret}") or {}).get("data") or {}
        return {k: base64.b64decode(v).decode() for k, v in data.items()}


__all__ = ["ProvisioningApi", "SYSTEM_AGENT_INSTALL_SCRIPT"]
