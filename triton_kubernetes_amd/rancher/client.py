"""Rancher v3 REST client.

In-process replacements for the reference's shell + curl + jq scripts:

* :meth:`RancherClient.bootstrap` — ``setup_rancher.sh.tpl`` (S3): wait for the
  server, log in as admin with the bootstrap password the server was started with
  (``CATTLE_BOOTSTRAP_PASSWORD``; Rancher ≥2.6 has no admin/admin), create the
  non-expiring ``triton-kubernetes`` API token, change the admin password, set
  ``server-url``;
* :meth:`RancherClient.ensure_cluster` — ``rancher_cluster.sh`` (S4): find or
  create the cluster by name, get or create its registration token, and the
  CA checksum (sha256 of ``cacerts`` + newline, exactly what the script hashes).
  RKE2 (default, ``versions.py``): a ``provisioning.cattle.io/v1`` ``Cluster`` in
  ``fleet-default`` with an ``rkeConfig``, whose management cluster (``status.clusterName``,
  ``c-m-…``) carries the registration token nodes hand to ``system-agent-install.sh``;
  RKE1: the reference's v3 ``cluster`` with ``rancherKubernetesEngineConfig``;
* new: cluster / node status, Kubernetes API through Rancher's ``/k8s/clusters``
  proxy (used by the readiness waiter and the MI355X add-on step), cleanup.

Waits poll adaptively (20 ms doubling to ``max_interval``) instead of the
reference's fixed ``sleep 5``.
"""

import base64
import hashlib
import json
import time
import urllib.parse
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional

from ..cloud.http import HTTPClient, HTTPError, TLSVerificationError
from ..errors import TKError
from ..versions import FLEET_NAMESPACE, default_version, resolve_against, resolve_distribution

TOKEN_NAME = "triton-kubernetes"


@dataclass
class ClusterInfo:
    cluster_id: str
    registration_token: str
    ca_checksum: str
    existed: bool = False

    def outputs(self) -> Dict[str, str]:
        return {"rancher_cluster_id": self.cluster_id,
                "rancher_cluster_registration_token": self.registration_token,
                "rancher_cluster_ca_checksum": self.ca_checksum}


def ca_checksum(cacerts: str) -> str:
    """Rancher's own rule (what ``/cacerts`` serves and the agents hash): the bundle with
    one trailing newline; an empty CA (a publicly trusted certificate) has no checksum."""
    if not cacerts:
        return ""
    return hashlib.sha256((cacerts if cacerts.endswith("\n") else cacerts + "\n").encode()).hexdigest()


def wait_until(fn: Callable[[], Any], timeout: float, what: str, first: float = 0.02,
               max_interval: float = 1.0) -> Any:
    """Call ``fn`` until it returns a truthy value (adaptive backoff)."""
    deadline = time.monotonic() + timeout
    delay = first
    last_exc: Optional[BaseException] = None
    while True:
        try:
            value = fn()
            if value:
                return value
        except TLSVerificationError:
            raise  # not a server that is still starting: another certificate (never retried)
        except (TKError, OSError) as exc:
            last_exc = exc
        if time.monotonic() >= deadline:
            detail = f": {last_exc}" if last_exc else ""
            raise TKError(f"timed out after {timeout:.0f}s waiting for {what}{detail}")
        time.sleep(delay)
        delay = min(max_interval, delay * 2)


class RancherClient:
    """``trust``: the server's pinned CA (``rancher/trust.py``): HTTPS is verified against
    it alone, and cluster CA checksums are computed from it.  Without one the system trust
    store verifies (a publicly trusted certificate, or a manager not pinned yet)."""

    def __init__(self, url: str, access_key: str = "", secret_key: str = "", verify_tls: bool = True,
                 timeout: float = 30.0, trust: Any = None):
        self.url = url.rstrip("/")
        self.token_timeout = 120.0  # registration token value, filled in asynchronously
        self.access_key = access_key
        self.secret_key = secret_key
        self.last_version_note = ""  # set when resolve_k8s_version substituted a release
        self.trust = trust
        tls = self.url.startswith("https://")
        self.http = HTTPClient(base_url=self.url, verify_tls=verify_tls, timeout=timeout,
                               ssl_context=trust.context() if trust is not None and tls and verify_tls else None,
                               tls_hint=(trust.describe() if trust is not None else "the system trust store")
                               + ". If the server's CA was rotated on purpose, pin the new one with "
                                 "rancher_ca_file=<PEM bundle>")
        self._apply_auth()

    def _apply_auth(self) -> None:
        if self.access_key or self.secret_key:
            cred = base64.b64encode(f"{self.access_key}:{self.secret_key}".encode()).decode()
            self.http.default_headers["Authorization"] = f"Basic {cred}"
        else:
            self.http.default_headers.pop("Authorization", None)

    # --- server bootstrap (S3) -------------------------------------------------------
    def ping(self) -> bool:
        try:
            self.http.request("GET", "/ping", ok=(200,))
            return True
        except TLSVerificationError:
            raise
        except TKError:
            return False

    def wait_for_server(self, timeout: float = 600.0) -> None:
        wait_until(self.ping, timeout, f"Rancher at {self.url}")

    def login(self, username: str, password: str) -> str:
        data = self.http.post_json("/v3-public/localProviders/local?action=login",
                                   {"username": username, "password": password, "ttl": 60000,
                                    "description": "Initial Token"})
        token = data.get("token", "")
        if not token:
            raise TKError("Rancher login returned no token")
        return token

    def bootstrap(self, admin_password: str, server_url: str, initial_password: str,
                  timeout: float = 600.0) -> Dict[str, str]:
        """Run S3 from the operator side; returns the manager module outputs.

        ``initial_password`` is the server's bootstrap password.  A server whose
        bootstrap already changed it (a re-run after a later step failed) accepts the
        admin password instead; the password change is then skipped."""
        self.wait_for_server(timeout)
        try:
            initial = self.login("admin", initial_password)
        except HTTPError as exc:
            if exc.status != 401 or not admin_password or admin_password == initial_password:
                raise
            initial = self.login("admin", admin_password)
            initial_password = admin_password
        user, _, secret = initial.partition(":")
        self.access_key, self.secret_key = user, secret
        self._apply_auth()
        tok = self.http.post_json("/v3/token", {"type": "token", "description": "Managed by triton-kubernetes",
                                                "name": TOKEN_NAME, "ttl": 0, "expired": False,
                                                "isDerived": False})
        name = tok.get("name", "")
        secret_key = tok.get("token", "").split(":", 1)[-1]
        self.access_key, self.secret_key = name, secret_key
        self._apply_auth()
        if admin_password and admin_password != initial_password:
            self.http.post_json("/v3/users?action=changepassword",
                                {"currentPassword": initial_password, "newPassword": admin_password})
        self.http.put_json("/v3/settings/server-url", {"baseType": "setting", "id": "server-url",
                                                       "name": "server-url", "type": "setting",
                                                       "value": server_url})
        return {"rancher_url": server_url, "rancher_access_key": name, "rancher_secret_key": secret_key}

    # --- clusters (S4) -------------------------------------------------------------------
    def find_cluster(self, name: str) -> Optional[Dict[str, Any]]:
        data = self.http.get_json("/v3/clusters", params={"name": name}).get("data", [])
        return data[0] if data else None

    def create_cluster(self, name: str, k8s_version: str, network_provider: str, k8s_registry: str = "",
                       k8s_registry_username: str = "", k8s_registry_password: str = "") -> Dict[str, Any]:
        rke: Dict[str, Any] = {
            "ignoreDockerVersion": False,
            "sshAgentAuth": False,
            "type": "rancherKubernetesEngineConfig",
            "kubernetesVersion": k8s_version,
            "authentication": {"type": "authnConfig", "strategy": "x509"},
            "network": {"type": "networkConfig", "plugin": network_provider},
            "services": {"type": "rkeConfigServices", "kubeApi": {"podSecurityPolicy": False,
                                                                 "type": "kubeAPIService"}},
        }
        if k8s_registry:
            rke["privateRegistries"] = [{"url": k8s_registry, "user": k8s_registry_username,
                                         "password": k8s_registry_password}]
        body = {"type": "cluster", "googleKubernetesEngineConfig": None, "name": name,
                "rancherKubernetesEngineConfig": rke, "id": ""}
        return self.http.post_json("/v3/cluster", body)

    def registration_token(self, cluster_id: str, create: bool) -> str:
        if not create:
            data = self.http.get_json(f"/v3/clusters/{cluster_id}/clusterregistrationtokens").get("data", [])
            if data and data[0].get("token"):
                return data[0]["token"]
        resp = self.http.post_json("/v3/clusterregistrationtoken",
                                   {"clusterId": cluster_id, "type": "clusterRegistrationToken"})
        token = resp.get("token", "")
        if token or not resp.get("id"):
            return token
        # the server's controller fills the value in after the create returns
        return wait_until(lambda: self.http.get_json(f"/v3/clusterregistrationtokens/{resp['id']}").get("token"),
                          self.token_timeout, f"cluster registration token {resp['id']}")

    def cacerts(self) -> str:
        return self.http.get_json("/v3/settings/cacerts").get("value", "") or ""

    def setting(self, name: str) -> str:
        try:
            return str(self.http.get_json(f"/v3/settings/{name}").get("value", "") or "")
        except HTTPError as exc:
            if exc.status in (403, 404):
                return ""
            raise

    def k8s_versions(self) -> List[str]:
        """RKE1 releases this server offers (its KDM list, setting ``k8s-versions-current``)."""
        return [v.strip() for v in self.setting("k8s-versions-current").split(",") if v.strip()]

    def rke2_versions(self) -> List[str]:
        """RKE2 releases this server offers (``/v1-rke2-release/releases``, from its KDM data)."""
        try:
            data = self.http.get_json("/v1-rke2-release/releases").get("data", [])
        except HTTPError as exc:
            if exc.status in (403, 404):
                return []
            raise
        return [str(r.get("version") or r.get("id") or "") for r in data if r.get("version") or r.get("id")]

    def resolve_k8s_version(self, requested: str, distribution: str = "rke1") -> str:
        """``requested`` if offered, else the server's release of the same minor; a minor
        the server does not offer is an error here rather than a failed provision."""
        offered = self.rke2_versions() if distribution == "rke2" else self.k8s_versions()
        try:
            version, note = resolve_against(requested, offered)
        except ValueError as exc:
            raise TKError(str(exc)) from None
        self.last_version_note = note
        return version

    # --- RKE2 (provisioning v2) ------------------------------------------------------------------
    def find_v2_cluster(self, name: str) -> Optional[Dict[str, Any]]:
        try:
            return self.http.get_json(f"/v1/provisioning.cattle.io.clusters/{FLEET_NAMESPACE}/{name}")
        except HTTPError as exc:
            if exc.status == 404:
                return None
            raise

    def create_v2_cluster(self, name: str, k8s_version: str, cni: str, k8s_registry: str = "",
                          k8s_registry_username: str = "", k8s_registry_password: str = "") -> Dict[str, Any]:
        """A custom RKE2 cluster: nodes are added by running the registration command."""
        rke: Dict[str, Any] = {"machineGlobalConfig": {"cni": cni, "disable-kube-proxy": False},
                               "machinePools": [], "upgradeStrategy": {"controlPlaneConcurrency": "1",
                                                                       "workerConcurrency": "1"}}
        if k8s_registry:
            config: Dict[str, Any] = {}
            if k8s_registry_username:
                # registry credentials: a basic-auth Secret in fleet-default the config names
                config["authConfigSecretName"] = self.create_registry_secret(k8s_registry_username,
                                                                             k8s_registry_password)
            rke["registries"] = {"mirrors": {"docker.io": {"endpoint": [f"https://{k8s_registry}"]}},
                                 "configs": {k8s_registry: config}}
        body = {"apiVersion": "provisioning.cattle.io/v1", "kind": "Cluster",
                "metadata": {"name": name, "namespace": FLEET_NAMESPACE},
                "spec": {"kubernetesVersion": k8s_version, "rkeConfig": rke}}
        return self.http.post_json("/v1/provisioning.cattle.io.clusters", body)

    def create_registry_secret(self, username: str, password: str) -> str:
        """A ``kubernetes.io/basic-auth`` Secret in fleet-default -> its name."""
        b64 = lambda v: base64.b64encode(v.encode()).decode()  # noqa: E731
        body = {"type": "kubernetes.io/basic-auth",
                "metadata": {"generateName": "registryconfig-auth-", "namespace": FLEET_NAMESPACE},
                "data": {"username": b64(username), "password": b64(password)}}
        return str(self.http.post_json("/v1/secrets", body)["metadata"]["name"])

    def v2_management_id(self, name: str, timeout: float = 120.0) -> str:
        """The management cluster (``c-m-…``) Rancher's controllers create for a
        provisioning cluster, once ``status.clusterName`` is set."""
        return wait_until(lambda: ((self.find_v2_cluster(name) or {}).get("status") or {}).get("clusterName"),
                          timeout, f"the management cluster of {name}")

    def ensure_cluster(self, name: str, k8s_version: str = "", network_provider: str = "flannel",
                       k8s_registry: str = "", k8s_registry_username: str = "",
                       k8s_registry_password: str = "", distribution: str = "") -> ClusterInfo:
        """Find or create cluster ``name`` of ``distribution`` (default: the one ``k8s_version``
        names, else RKE2) -> id, registration token, CA checksum.  ``k8s_version`` defaults
        to the pinned release of the distribution."""
        try:
            dist = resolve_distribution(k8s_version, distribution)
        except ValueError as exc:
            raise TKError(str(exc)) from None
        k8s_version = k8s_version or default_version(dist)
        other = self.find_cluster(name)  # v3: every cluster, RKE1 or the management side of RKE2
        other_dist = None if other is None else ("rke2" if other.get("driver") == "rke2" else "rke1")
        if other_dist is not None and other_dist != dist:
            raise TKError(f"cluster '{name}' already exists as an {other_dist.upper()} cluster; "
                          f"it cannot be reused as {dist.upper()}")
        if dist == "rke2":
            existing = self.find_v2_cluster(name)
            existed = existing is not None
            if not existed:
                version = self.resolve_k8s_version(k8s_version, "rke2")
                self.create_v2_cluster(name, version, network_provider, k8s_registry, k8s_registry_username,
                                       k8s_registry_password)
            cluster_id = self.v2_management_id(name)
        else:
            if other is not None:
                cluster_id, existed = other.get("id", ""), True
            else:
                k8s_version = self.resolve_k8s_version(k8s_version, "rke1")
                cluster_id = self.create_cluster(name, k8s_version, network_provider, k8s_registry,
                                                 k8s_registry_username, k8s_registry_password).get("id", "")
                existed = False
        if not cluster_id:
            raise TKError("Unable to create cluster!")
        token = self.registration_token(cluster_id, create=not existed)
        if not token:
            raise TKError("Unable to create cluster registration token!")
        # the checksum nodes pin: of the bundle pinned at create manager, not of what the
        # server says now (over a channel that bundle verified, when there is one)
        checksum = self.trust.checksum if self.trust is not None else ca_checksum(self.cacerts())
        return ClusterInfo(cluster_id, token, checksum, existed)

    # --- status -------------------------------------------------------------------------------
    def cluster(self, cluster_id: str) -> Dict[str, Any]:
        return self.http.get_json(f"/v3/clusters/{cluster_id}")

    def cluster_version(self, cluster_id: str) -> str:
        """The Kubernetes release the cluster runs (``version.gitVersion``)."""
        return str((self.cluster(cluster_id).get("version") or {}).get("gitVersion", ""))

    def upgrade_cluster(self, cluster_id: str, version: str) -> None:
        """Set the cluster's Kubernetes release: an RKE2 cluster's provisioning object
        (``spec.kubernetesVersion``), an RKE1 cluster's ``rancherKubernetesEngineConfig``.
        Rancher's controllers then upgrade the nodes (control plane first)."""
        if cluster_id.startswith("c-m-"):
            name = str(self.cluster(cluster_id).get("name", ""))
            for attempt in range(5):
                obj = self.find_v2_cluster(name)
                if obj is None:
                    raise TKError(f"no provisioning cluster '{name}' for {cluster_id}")
                obj.setdefault("spec", {})["kubernetesVersion"] = version
                try:
                    # the object carries the resourceVersion it was read at: the controllers
                    # update it too, so a conflict means re-read and re-apply
                    self.http.request("PUT", f"/v1/provisioning.cattle.io.clusters/{FLEET_NAMESPACE}/{name}",
                                      json_body=obj, ok=(200,))
                    return
                except HTTPError as exc:
                    if exc.status != 409 or attempt == 4:
                        raise
        else:
            c = self.cluster(cluster_id)
            c.setdefault("rancherKubernetesEngineConfig", {})["kubernetesVersion"] = version
            self.http.request("PUT", f"/v3/clusters/{cluster_id}", json_body=c, ok=(200,))

    def cluster_state(self, cluster_id: str) -> str:
        return str(self.cluster(cluster_id).get("state", ""))

    def nodes(self, cluster_id: str) -> List[Dict[str, Any]]:
        return self.http.get_json("/v3/nodes", params={"clusterId": cluster_id}).get("data", [])

    def delete_cluster(self, cluster_id: str) -> None:
        """Delete a cluster.  An RKE2 cluster's management object (``c-m-…``) is owned by
        its provisioning cluster, which is what gets deleted (the controllers would
        otherwise recreate the management cluster)."""
        try:
            if cluster_id.startswith("c-m-"):
                name = str(self.cluster(cluster_id).get("name", ""))
                self.http.request("DELETE", f"/v1/provisioning.cattle.io.clusters/{FLEET_NAMESPACE}/{name}")
            else:
                self.http.request("DELETE", f"/v3/clusters/{cluster_id}")
        except HTTPError as exc:
            if exc.status != 404:
                raise

    def delete_node(self, node_id: str) -> None:
        try:
            self.http.request("DELETE", f"/v3/nodes/{node_id}")
        except HTTPError as exc:
            if exc.status != 404:
                raise

    # --- Kubernetes API via the Rancher proxy ------------------------------------------------
    def k8s(self, cluster_id: str, method: str, path: str, body: Any = None, ok=(200, 201, 202, 204)) -> Any:
        resp = self.http.request(method, f"/k8s/clusters/{cluster_id}/{path.lstrip('/')}", json_body=body, ok=ok)
        return resp.json() if resp.body else None

    def k8s_nodes(self, cluster_id: str) -> List[Dict[str, Any]]:
        return (self.k8s(cluster_id, "GET", "/api/v1/nodes") or {}).get("items", [])

    def patch_node(self, cluster_id: str, name: str, patch: Dict[str, Any]) -> Dict[str, Any]:
        """JSON merge patch (RFC 7386) of a Kubernetes Node: ``metadata.labels`` merge (null
        removes a key), ``spec.taints`` is replaced whole."""
        resp = self.http.request("PATCH", f"/k8s/clusters/{cluster_id}/api/v1/nodes/{name}",
                                 data=json.dumps(patch).encode(),
                                 headers={"Content-Type": "application/merge-patch+json"}, ok=(200,))
        return resp.json()

    def cordon(self, cluster_id: str, name: str, unschedulable: bool = True) -> Dict[str, Any]:
        """``kubectl cordon`` / ``uncordon``: ``spec.unschedulable`` of the Node."""
        return self.patch_node(cluster_id, name, {"spec": {"unschedulable": unschedulable}})

    def node_pods(self, cluster_id: str, name: str) -> List[Dict[str, Any]]:
        """Every pod bound to node ``name`` (all namespaces; a field selector)."""
        q = urllib.parse.urlencode({"fieldSelector": f"spec.nodeName={name}"})
        return (self.k8s(cluster_id, "GET", f"/api/v1/pods?{q}") or {}).get("items", [])

    def evict_pod(self, cluster_id: str, namespace: str, name: str) -> int:
        """POST an Eviction (policy/v1): 201 evicted, 429 refused by a PodDisruptionBudget
        (retry later), 404 already gone."""
        body = {"apiVersion": "policy/v1", "kind": "Eviction", "metadata": {"name": name, "namespace": namespace}}
        resp = self.http.request("POST", f"/k8s/clusters/{cluster_id}/api/v1/namespaces/{namespace}/pods/{name}/eviction",
                                 json_body=body, ok=(200, 201, 404, 429))
        return resp.status
