"""Rancher v3 (Norman) API of the fake server: bootstrap, RKE1 clusters, tokens, nodes.

* bootstrap: ``POST /v3-public/localProviders/local?action=login``,
  ``POST /v3/token``, ``POST /v3/users?action=changepassword``, ``GET/PUT
  /v3/settings/<name>``, unauthenticated ``GET /cacerts``.  Like Rancher >=2.6 the server
  starts with a *bootstrap* admin password (``CATTLE_BOOTSTRAP_PASSWORD``; random when not
  given -- there is no admin/admin);
* clusters (S4): ``GET /v3/clusters?name=``, ``POST /v3/cluster`` (an RKE1 custom cluster),
  ``GET / PUT / DELETE /v3/clusters/<id>``, ``?action=generateKubeconfig``.  Rancher
  reports an RKE1 cluster's upstream version (``version.gitVersion`` ``v1.30.10`` for
  ``v1.30.10-rancher1-1``);
* registration tokens: ``POST /v3/clusterregistrationtoken``,
  ``GET /v3/clusters/<id>/clusterregistrationtokens``,
  ``GET /v3/clusterregistrationtokens/<id>``.  A new token's value is filled in by the
  server's controller after the create returns (``async_registration_tokens``, default
  on): the POST answers with an empty ``token`` and the first read after that sees it;
* ``GET /v3/nodes?clusterId=``, ``DELETE /v3/nodes/<id>``;
* ``POST /v3/connect/register`` -- agent registration (``X-API-Tunnel-Token`` + base64 JSON
  ``X-API-Tunnel-Params`` with hostname, roles, labels, capacity, taints), standing in for
  the rancher-agent websocket tunnel; ``X-Cattle-Agent-Kind: system-agent`` marks an RKE2
  node's ``rancher-system-agent``.

Refusals (negative tests in ``tests/test_fake_rancher_contract.py``, ``test_v3_*``):

* no or a wrong token -> 401; a wrong login -> 401; a wrong current password -> 400; a
  new password shorter than ``password-min-length`` (12) -> 422;
* a setting the server does not have -> 404;
* a cluster without a name -> 422; a name already taken -> 422 ``NotUnique``; a
  ``kubernetesVersion`` outside ``k8s-versions-current`` or a network plugin RKE1 does not
  deploy -> 422; a downgrade -> 422; a
  ``PUT`` on an RKE2 (provisioning-owned) cluster -> 422;
* a registration token for an unknown cluster -> 422; unknown cluster, token or node
  -> 404;
* registration with an unknown token -> 401, with unreadable params -> 400, with the
  wrong agent kind for the cluster's distribution -> 400.
"""

import base64
import json
import re
import secrets
import time
import urllib.parse
import uuid
from typing import Any, Dict, List, Optional, Tuple

from ...versions import running_version
from ..connect import tunnel_params

Reply = Tuple[int, Any]
# the network plugins RKE1 deploys (rancherKubernetesEngineConfig.network.plugin)
RKE1_NETWORK_PLUGINS = ("canal", "flannel", "calico", "weave", "none")


def _err(code: int, kind: str, message: str = "", **extra: Any) -> Reply:
    return code, dict({"type": "error", "code": kind, "message": message}, **extra)


def version_key(v: str) -> Tuple[int, ...]:
    """``v1.30.10-rancher1-1`` / ``v1.31.6+rke2r1`` -> ``(1, 30, 10)``."""
    return tuple(int(x) for x in re.findall(r"\d+", v.split("+")[0].split("-")[0]))


class V3Api:
    """Mixin of :class:`~.server.FakeRancher`: the ``/v3`` API and agent registration."""

    def _route_v3_public(self, method: str, path: str, query: Dict[str, List[str]], body: Any,
                         headers: Any) -> Optional[Reply]:
        st = self.state
        if path == "/v3-public/localProviders/local" and query.get("action") == ["login"]:
            if body.get("username") == "admin" and body.get("password") == st.admin_password:
                name, secret = f"token-{uuid.uuid4().hex[:5]}", uuid.uuid4().hex
                with st.mu:
                    st.tokens[name] = secret
                return 201, {"token": f"{name}:{secret}", "type": "token"}
            return _err(401, "Unauthorized", "authentication failed")
        if path == "/v3/connect/register" and method == "POST":
            return self._register(headers)
        if path == "/cacerts" and method == "GET":  # unauthenticated, what the installers pin
            with st.mu:
                ca = st.settings.get("cacerts", "")
                return 200, (ca if not ca or ca.endswith("\n") else ca + "\n").encode()
        return None

    def _route_v3(self, method: str, path: str, query: Dict[str, List[str]], body: Any) -> Optional[Reply]:
        st = self.state
        if path == "/v3/token" and method == "POST":
            name, secret = f"token-{uuid.uuid4().hex[:5]}", uuid.uuid4().hex
            with st.mu:
                st.tokens[name] = secret
            return 201, {"name": name, "token": f"{name}:{secret}", "type": "token"}
        if path == "/v3/users" and query.get("action") == ["changepassword"]:
            if body.get("currentPassword") != st.admin_password:
                return _err(400, "InvalidBodyContent", "invalid current password")
            if len(body.get("newPassword", "")) < int(st.settings["password-min-length"]):
                return _err(422, "InvalidFormat",
                            f"Password must be at least {st.settings['password-min-length']} characters")
            st.admin_password = body.get("newPassword", "")
            return 200, {}
        if path.startswith("/v3/settings/"):
            key = path.rsplit("/", 1)[1]
            with st.mu:
                if key not in st.settings:
                    return _err(404, "NotFound", f"setting {key} not found")
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
            return self._create_cluster(body)
        if path.startswith("/v3/clusters/"):
            return self._cluster(method, path[len("/v3/clusters/"):].split("/"), query, body)
        if path == "/v3/clusterregistrationtoken" and method == "POST":
            tok = uuid.uuid4().hex + uuid.uuid4().hex[:8]
            cid = body.get("clusterId")
            with st.mu:
                if cid not in st.clusters:
                    return _err(422, "InvalidReference", f"cluster {cid} not found", fieldName="clusterId")
                n = sum(1 for t in st.reg_tokens.values() if t["clusterId"] == cid)
                st.reg_tokens[tok] = {"id": f"{cid}:crt-{n}", "clusterId": cid,
                                      "ready": not self.async_registration_tokens}
                return 201, dict(self._token_view(tok, fill=False), type="clusterRegistrationToken")
        if path.startswith("/v3/clusterregistrationtokens/") and method == "GET":
            tid = urllib.parse.unquote(path[len("/v3/clusterregistrationtokens/"):])
            with st.mu:
                tok = next((k for k, t in st.reg_tokens.items() if t["id"] == tid), None)
                if tok is None:
                    return _err(404, "NotFound", f"clusterregistrationtoken {tid} not found")
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
            nid = path.rsplit("/", 1)[1]
            with st.mu:
                n = st.nodes.pop(nid, None)
                if n is None:
                    return _err(404, "NotFound", f"node {nid} not found")
                st.cluster_nodes.get(n["clusterId"], {}).pop(n["id"], None)
            return 200, {}
        return None

    def _create_cluster(self, body: Any) -> Reply:
        st = self.state
        name = str(body.get("name", "") or "")
        if not name:
            return _err(422, "MissingRequired", "name is required", fieldName="name")
        version = (body.get("rancherKubernetesEngineConfig") or {}).get("kubernetesVersion", "")
        offered = [v for v in st.settings["k8s-versions-current"].split(",") if v]
        if version not in offered:
            return _err(422, "InvalidBodyContent", f"{version} is not a supported Kubernetes version",
                        fieldName="kubernetesVersion")
        plugin = ((body.get("rancherKubernetesEngineConfig") or {}).get("network") or {}).get("plugin", "canal")
        if plugin not in RKE1_NETWORK_PLUGINS:
            return _err(422, "InvalidOption", f"{plugin} is not a supported network plugin",
                        fieldName="rancherKubernetesEngineConfig.network.plugin")
        cid = f"c-{uuid.uuid4().hex[:5]}"
        with st.mu:
            if any(c["name"] == name for c in st.clusters.values()):
                return _err(422, "NotUnique", "Cluster name must be unique", fieldName="name")
            st.clusters[cid] = {"id": cid, "name": name, "state": "provisioning", "transitioning": "yes",
                                "rancherKubernetesEngineConfig": body.get("rancherKubernetesEngineConfig", {}),
                                "created": time.time(), "driver": "rancherKubernetesEngine",
                                # Rancher reports an RKE1 cluster's upstream version
                                "version": {"gitVersion": running_version(version, "rke1")}}
            st.cluster_nodes[cid] = {}
            st.unsettled.add(cid)
            return 201, dict(st.clusters[cid])

    def _cluster(self, method: str, rest: List[str], query: Dict[str, List[str]], body: Any) -> Reply:
        st = self.state
        cid = rest[0]
        with st.mu:
            if cid not in st.clusters:
                return _err(404, "NotFound", f"cluster {cid} not found")
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
                    return _err(422, "Invalid", "an RKE2 cluster is changed through provisioning.cattle.io")
                return self._upgrade(cid, body)
        self._refresh()
        with st.mu:
            return 200, dict(st.clusters[cid])

    def _token_view(self, tok: str, fill: bool = True) -> Dict[str, Any]:
        """A registration token as the API shows it: its value only once the (simulated)
        controller has filled it in -- which happens on the first read after the create."""
        t = self.state.reg_tokens[tok]
        shown = tok if t["ready"] else ""
        if fill:
            t["ready"] = True
        return {"id": t["id"], "clusterId": t["clusterId"], "token": shown}

    def registration(self, name: str = "test", distribution: str = "rke2") -> Tuple[str, str, str]:
        """``(cluster id, registration token, ca checksum)`` of a new cluster: what an admin
        copies out of the UI's registration command (tests of the node-side join)."""
        from ..client import ca_checksum

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

    def _register(self, headers: Any) -> Reply:
        st = self.state
        token = headers.get("X-API-Tunnel-Token", "")
        with st.mu:
            reg = st.reg_tokens.get(token)
        if reg is None:
            return _err(401, "InvalidRegistrationToken", "unknown registration token")
        try:
            params = json.loads(base64.b64decode(headers.get("X-API-Tunnel-Params", "")) or b"{}")
        except ValueError:
            return _err(400, "InvalidBodyContent", "bad tunnel params")
        kind = headers.get("X-Cattle-Agent-Kind", "rancher-agent")
        with st.mu:
            prov = "rke2" if (st.clusters.get(reg["clusterId"]) or {}).get("driver") == "rke2" else "rke1"
        if (prov == "rke2") != (kind == "system-agent"):
            want = "rancher-system-agent (system-agent-install.sh)" if prov == "rke2" else "rancher-agent"
            return _err(400, "InvalidAgent", f"{reg['clusterId']} is an {prov.upper()} cluster: nodes join with {want}")
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


__all__ = ["V3Api", "tunnel_params", "version_key"]
