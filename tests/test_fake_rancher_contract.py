"""The fake Rancher server's contract, API by API: it refuses what a real server refuses.

Each fake behaviour the workflows rely on has a positive test elsewhere (the workflow
tests); this file pins the refusals listed in each module of ``rancher/fake/`` -- the
status code and reason a real Rancher / kube-apiserver answers -- so a client bug that a
real server would reject cannot pass against the fake.
"""

import base64
import http.client
import json
import urllib.parse

import pytest

from triton_kubernetes_amd.rancher.fake import FakeRancher, tunnel_params
from triton_kubernetes_amd.versions import FLEET_NAMESPACE, K8S_VERSIONS, RKE2_VERSIONS

RKE1 = K8S_VERSIONS[1][1]
RKE2_OLD, RKE2_NEW = RKE2_VERSIONS[1][1], RKE2_VERSIONS[0][1]


class Api:
    """A bare HTTP client for the fake (no retries, no client-side checks)."""

    def __init__(self, fake: FakeRancher, token: str = ""):
        u = urllib.parse.urlsplit(fake.url)
        self.host, self.port, self.token = u.hostname, u.port, token

    def __call__(self, method, path, body=None, headers=None):
        conn = http.client.HTTPConnection(self.host, self.port, timeout=10)
        hdrs = {"Content-Type": "application/json"}
        if self.token:
            hdrs["Authorization"] = "Bearer " + self.token
        hdrs.update(headers or {})
        data = json.dumps(body).encode() if body is not None else None
        try:
            conn.request(method, path, body=data, headers=hdrs)
            resp = conn.getresponse()
            raw = resp.read()
        finally:
            conn.close()
        try:
            return resp.status, json.loads(raw) if raw else {}
        except ValueError:
            return resp.status, raw


@pytest.fixture
def fake():
    with FakeRancher(bootstrap_password="bootstrap-pw-0123") as f:
        yield f


@pytest.fixture
def api(fake):
    code, out = Api(fake)("POST", "/v3-public/localProviders/local?action=login",
                          {"username": "admin", "password": "bootstrap-pw-0123"})
    assert code == 201
    return Api(fake, out["token"])


def _rke1(api, name="c1", version=RKE1):
    code, out = api("POST", "/v3/cluster", {"name": name, "rancherKubernetesEngineConfig":
                                            {"kubernetesVersion": version}})
    assert code == 201, out
    return out["id"]


def _rke2(api, name="r1", version=RKE2_OLD):
    code, out = api("POST", "/v1/provisioning.cattle.io.clusters",
                    {"metadata": {"name": name, "namespace": FLEET_NAMESPACE},
                     "spec": {"kubernetesVersion": version, "rkeConfig": {}}})
    assert code == 201, out
    code, obj = api("GET", f"/v1/provisioning.cattle.io.clusters/{FLEET_NAMESPACE}/{name}")
    assert code == 200 and obj["status"]["clusterName"].startswith("c-m-")
    return obj


# --- v3 -------------------------------------------------------------------------------------------
def test_v3_authentication(fake):
    anon = Api(fake)
    assert anon("GET", "/v3/clusters")[0] == 401
    assert Api(fake, "token-x:nope")("GET", "/v3/clusters")[0] == 401
    assert Api(fake, "token-x:")("GET", "/v3/clusters")[0] == 401  # an empty secret is no secret
    assert anon("POST", "/v3-public/localProviders/local?action=login",
                {"username": "admin", "password": "admin"})[0] == 401  # no admin/admin
    assert anon("POST", "/v3-public/localProviders/local?action=login",
                {"username": "root", "password": "bootstrap-pw-0123"})[0] == 401
    # the unauthenticated endpoints stay open
    assert anon("GET", "/ping")[0] == 200 and anon("GET", "/cacerts")[0] == 200
    assert anon("GET", "/system-agent-install.sh")[0] == 200


def test_v3_password_change_refusals(api):
    code, out = api("POST", "/v3/users?action=changepassword",
                    {"currentPassword": "wrong", "newPassword": "a-long-enough-pw"})
    assert code == 400
    code, out = api("POST", "/v3/users?action=changepassword",
                    {"currentPassword": "bootstrap-pw-0123", "newPassword": "short"})
    assert code == 422 and out["code"] == "InvalidFormat" and "12" in out["message"]
    assert api("POST", "/v3/users?action=changepassword",
               {"currentPassword": "bootstrap-pw-0123", "newPassword": "a-long-enough-pw"})[0] == 200


def test_v3_unknown_setting_is_not_found(api):
    assert api("GET", "/v3/settings/no-such-setting")[0] == 404
    assert api("PUT", "/v3/settings/no-such-setting", {"value": "x"})[0] == 404
    assert api("PUT", "/v3/settings/server-url", {"value": "https://r.example"})[0] == 200
    assert api("GET", "/v3/settings/server-url")[1]["value"] == "https://r.example"


def test_v3_cluster_create_refusals(api):
    code, out = api("POST", "/v3/cluster", {"name": "c1", "rancherKubernetesEngineConfig":
                                            {"kubernetesVersion": "v1.9.7-rancher2-2"}})
    assert code == 422 and out["fieldName"] == "kubernetesVersion"
    code, out = api("POST", "/v3/cluster", {"rancherKubernetesEngineConfig": {"kubernetesVersion": RKE1}})
    assert code == 422 and out["code"] == "MissingRequired"
    code, out = api("POST", "/v3/cluster", {"name": "c1", "rancherKubernetesEngineConfig":
                                            {"kubernetesVersion": RKE1, "network": {"plugin": "cilium"}}})
    assert code == 422 and out["fieldName"] == "rancherKubernetesEngineConfig.network.plugin"  # RKE2 only
    _rke1(api)
    code, out = api("POST", "/v3/cluster", {"name": "c1", "rancherKubernetesEngineConfig":
                                            {"kubernetesVersion": RKE1}})
    assert code == 422 and out["code"] == "NotUnique"


def test_v3_cluster_update_refusals(api):
    cid = _rke1(api)
    cluster = api("GET", f"/v3/clusters/{cid}")[1]
    assert cluster["version"]["gitVersion"] == RKE1.split("-")[0]  # upstream version for RKE1
    older = dict(cluster, rancherKubernetesEngineConfig={"kubernetesVersion": K8S_VERSIONS[2][1]})
    code, out = api("PUT", f"/v3/clusters/{cid}", older)
    assert code == 422 and "downgrade" in out["message"]
    code, out = api("PUT", f"/v3/clusters/{cid}", dict(cluster, rancherKubernetesEngineConfig=
                                                      {"kubernetesVersion": "v1.31.99-rancher1-1"}))
    assert code == 422
    # an RKE2 cluster's management object is owned by its provisioning object
    mgmt = _rke2(api)["status"]["clusterName"]
    code, out = api("PUT", f"/v3/clusters/{mgmt}", {"rancherKubernetesEngineConfig": {"kubernetesVersion": RKE1}})
    assert code == 422 and "provisioning.cattle.io" in out["message"]
    assert api("GET", "/v3/clusters/c-nope")[0] == 404
    assert api("DELETE", "/v3/clusters/c-nope")[0] == 404


def test_v3_registration_token_and_node_refusals(api):
    code, out = api("POST", "/v3/clusterregistrationtoken", {"clusterId": "c-nope"})
    assert code == 422 and out["code"] == "InvalidReference"
    assert api("GET", "/v3/clusterregistrationtokens/c-nope:crt-0")[0] == 404
    assert api("DELETE", "/v3/nodes/m-nope")[0] == 404


def test_v3_registration_refusals(fake, api):
    anon = Api(fake)
    params = tunnel_params("n1", {"etcd": True, "controlplane": True, "worker": True}, {}, {})
    code, out = anon("POST", "/v3/connect/register", {},
                     {"X-API-Tunnel-Token": "not-a-token", "X-API-Tunnel-Params": params})
    assert code == 401 and out["code"] == "InvalidRegistrationToken"
    cid, tok, _ = fake.registration("r", "rke1")
    code, out = anon("POST", "/v3/connect/register", {},
                     {"X-API-Tunnel-Token": tok, "X-API-Tunnel-Params": "!!not base64 json"})
    assert code == 400
    # an RKE1 cluster refuses the RKE2 system agent, an RKE2 cluster the rancher-agent
    code, out = anon("POST", "/v3/connect/register", {},
                     {"X-API-Tunnel-Token": tok, "X-API-Tunnel-Params": params, "X-Cattle-Agent-Kind": "system-agent"})
    assert code == 400 and out["code"] == "InvalidAgent"
    _, tok2, _ = fake.registration("r2", "rke2")
    code, out = anon("POST", "/v3/connect/register", {}, {"X-API-Tunnel-Token": tok2, "X-API-Tunnel-Params": params})
    assert code == 400 and "rancher-system-agent" in out["message"]
    assert api("GET", f"/v3/nodes?clusterId={cid}")[1]["data"] == []  # nothing joined


# --- provisioning v1 ----------------------------------------------------------------------------
def test_v1_create_refusals(api):
    path = "/v1/provisioning.cattle.io.clusters"
    meta = {"name": "r1", "namespace": FLEET_NAMESPACE}
    code, out = api("POST", path, {"metadata": meta, "spec": {"kubernetesVersion": RKE1}})  # an RKE1 release
    assert code == 422 and out["fieldName"] == "spec.kubernetesVersion"
    code, out = api("POST", path, {"metadata": meta, "spec": {"kubernetesVersion": RKE2_NEW, "rkeConfig":
                                                              {"machineGlobalConfig": {"cni": "weave"}}}})
    assert code == 422 and "cni" in out["message"]
    code, out = api("POST", path, {"metadata": {"namespace": FLEET_NAMESPACE},
                                   "spec": {"kubernetesVersion": RKE2_NEW}})
    assert code == 422 and out["code"] == "MissingRequired"
    inline = {"registries": {"configs": {"reg.example": {"username": "u", "password": "p"}}}}
    code, out = api("POST", path, {"metadata": meta, "spec": {"kubernetesVersion": RKE2_NEW, "rkeConfig": inline}})
    assert code == 422 and "unknown fields" in out["message"]
    missing = {"registries": {"configs": {"reg.example": {"authConfigSecretName": "nope"}}}}
    code, out = api("POST", path, {"metadata": meta, "spec": {"kubernetesVersion": RKE2_NEW, "rkeConfig": missing}})
    assert code == 422 and "missing secret" in out["message"]
    _rke2(api)
    code, out = api("POST", path, {"metadata": meta, "spec": {"kubernetesVersion": RKE2_NEW}})
    assert code == 409 and out["code"] == "AlreadyExists"
    assert api("GET", f"{path}/{FLEET_NAMESPACE}/nope")[0] == 404


def test_v1_secret_refusals(api):
    code, out = api("POST", "/v1/secrets", {"metadata": {"namespace": FLEET_NAMESPACE}, "type": "Opaque"})
    assert code == 422
    body = {"metadata": {"name": "s", "namespace": FLEET_NAMESPACE}, "type": "Opaque"}
    assert api("POST", "/v1/secrets", body)[0] == 201
    assert api("POST", "/v1/secrets", body)[0] == 409
    code, out = api("POST", "/v1/secrets", {"metadata": {"generateName": "reg-", "namespace": FLEET_NAMESPACE}})
    assert code == 201 and out["metadata"]["name"].startswith("reg-")


def test_v1_update_preconditions(fake, api):
    obj = _rke2(api)
    path = f"/v1/provisioning.cattle.io.clusters/{FLEET_NAMESPACE}/r1"
    rv = obj["metadata"]["resourceVersion"]
    renamed = json.loads(json.dumps(obj))
    renamed["metadata"]["name"] = "other"
    assert api("PUT", path, renamed)[0] == 400
    older = json.loads(json.dumps(obj))
    older["spec"]["kubernetesVersion"] = RKE2_VERSIONS[2][1]
    code, out = api("PUT", path, older)
    assert code == 422 and "downgrade" in out["message"]
    newer = json.loads(json.dumps(obj))
    newer["spec"]["kubernetesVersion"] = RKE2_NEW
    code, out = api("PUT", path, newer)
    assert code == 200 and out["metadata"]["resourceVersion"] != rv
    # the same (now stale) object again: someone else changed it meanwhile
    code, out = api("PUT", path, newer)
    assert code == 409 and out["code"] == "Conflict"
    # without a resourceVersion the write is unconditional, as in Kubernetes
    del newer["metadata"]["resourceVersion"]
    assert api("PUT", path, newer)[0] == 200
    assert api("PATCH", path, {})[0] == 405


# --- k8s core -------------------------------------------------------------------------------------
def _cluster_with_node(fake, api):
    cid, tok, _ = fake.registration("k", "rke1")
    params = tunnel_params("n1", {"etcd": True, "controlplane": True, "worker": True}, {}, {})
    code, _ = Api(fake)("POST", "/v3/connect/register", {}, {"X-API-Tunnel-Token": tok, "X-API-Tunnel-Params": params})
    assert code == 201
    return cid


def test_k8s_create_refusals(fake, api):
    cid = _cluster_with_node(fake, api)
    k = f"/k8s/clusters/{cid}"
    assert api("POST", "/k8s/clusters/c-nope/api/v1/namespaces", {"metadata": {"name": "x"}})[0] == 404
    code, out = api("POST", f"{k}/api/v1/namespaces/default/configmaps", {"kind": "ConfigMap", "metadata": {}})
    assert code == 422 and out["reason"] == "Invalid"
    code, out = api("POST", f"{k}/api/v1/namespaces/nowhere/configmaps", {"metadata": {"name": "a"}})
    assert code == 404 and 'namespaces "nowhere" not found' in out["message"]
    code, out = api("POST", f"{k}/api/v1/namespaces/default/configmaps",
                    {"metadata": {"name": "a", "namespace": "kube-system"}})
    assert code == 400 and out["reason"] == "BadRequest"
    code, out = api("POST", f"{k}/api/v1/namespaces",
                    {"metadata": {"name": "gpu", "labels": {"pod-security.kubernetes.io/enforce": "lenient"}}})
    assert code == 403 and "must be one of privileged, baseline, restricted" in out["message"]
    code, out = api("POST", f"{k}/api/v1/namespaces", {"metadata": {"name": "gpu"}})
    assert code == 201 and out["metadata"]["uid"] and out["metadata"]["resourceVersion"]
    code, out = api("POST", f"{k}/api/v1/namespaces/gpu/configmaps", {"metadata": {"generateName": "cm-"}})
    assert code == 201 and out["metadata"]["name"].startswith("cm-") and out["metadata"]["namespace"] == "gpu"
    body = {"metadata": {"name": "a"}}
    assert api("POST", f"{k}/api/v1/namespaces/gpu/configmaps", body)[0] == 201
    code, out = api("POST", f"{k}/api/v1/namespaces/gpu/configmaps", body)
    assert code == 409 and out["reason"] == "AlreadyExists"


def test_k8s_replace_refusals(fake, api):
    cid = _cluster_with_node(fake, api)
    col = f"/k8s/clusters/{cid}/apis/apps/v1/namespaces/kube-system/daemonsets"
    spec = {"selector": {"matchLabels": {"app": "ds"}},
            "template": {"metadata": {"labels": {"app": "ds"}}, "spec": {"containers": [{"name": "c", "image": "i"}]}}}
    code, created = api("POST", col, {"metadata": {"name": "ds"}, "spec": spec})
    assert code == 201
    assert api("PUT", f"{col}/missing", {"metadata": {"name": "missing"}})[0] == 404
    code, out = api("PUT", f"{col}/ds", {"metadata": {"name": "other"}})
    assert code == 400 and "does not match the name on the URL" in out["message"]
    code, out = api("PUT", f"{col}/ds", {"metadata": {"name": "ds", "namespace": "default"}})
    assert code == 400
    code, updated = api("PUT", f"{col}/ds", created)  # current resourceVersion: accepted
    assert code == 200 and updated["metadata"]["uid"] == created["metadata"]["uid"]
    assert updated["metadata"]["resourceVersion"] != created["metadata"]["resourceVersion"]
    code, out = api("PUT", f"{col}/ds", created)  # stale now
    assert code == 409 and out["reason"] == "Conflict"
    assert api("DELETE", f"{col}/missing")[0] == 404
    # the API server's order: existence, then the precondition, then the new content
    invalid = {"metadata": {"name": "ds"}, "spec": {}}
    assert api("PUT", f"{col}/missing", dict(invalid, metadata={"name": "missing"}))[0] == 404
    stale = dict(invalid, metadata=dict(created["metadata"]))
    assert api("PUT", f"{col}/ds", stale)[0] == 409
    current = api("GET", f"{col}/ds")[1]
    code, out = api("PUT", f"{col}/ds", dict(invalid, metadata=dict(current["metadata"])))
    assert code == 422 and "spec.template.spec.containers" in out["message"]


def test_k8s_node_patch_and_eviction_refusals(fake, api):
    cid = _cluster_with_node(fake, api)
    k = f"/k8s/clusters/{cid}"
    node = api("GET", f"{k}/api/v1/nodes")[1]["items"][0]
    assert api("PATCH", f"{k}/api/v1/nodes/ghost", {"metadata": {"labels": {"a": "b"}}})[0] == 404
    assert api("PATCH", f"{k}/api/v1/nodes/n1", ["not", "an", "object"])[0] == 400
    rv = node["metadata"]["resourceVersion"]
    assert api("PATCH", f"{k}/api/v1/nodes/n1", {"metadata": {"resourceVersion": rv, "labels": {"a": "1"}}})[0] == 200
    code, out = api("PATCH", f"{k}/api/v1/nodes/n1", {"metadata": {"resourceVersion": rv, "labels": {"a": "2"}}})
    assert code == 409 and out["reason"] == "Conflict"
    assert api("GET", f"{k}/api/v1/nodes")[1]["items"][0]["metadata"]["labels"]["a"] == "1"
    assert api("POST", f"{k}/api/v1/namespaces/default/pods/ghost/eviction", {})[0] == 404
    pod = {"metadata": {"name": "p", "annotations": {FakeRancher.PDB_ANNOTATION: "always"}},
           "spec": {"nodeName": "n1", "containers": [{"name": "c", "image": "busybox"}]}}
    assert api("POST", f"{k}/api/v1/namespaces/default/pods", pod)[0] == 201
    code, out = api("POST", f"{k}/api/v1/namespaces/default/pods/p/eviction", {})
    assert code == 429 and out["reason"] == "TooManyRequests"
    assert fake.state.evictions_refused == 1


# --- admission ------------------------------------------------------------------------------------
def _pod(name, **spec):
    return {"metadata": {"name": name}, "spec": dict({"containers": [{"name": "c", "image": "busybox"}]}, **spec)}


def test_admission_pod_security_levels(fake, api):
    cid = _cluster_with_node(fake, api)
    k = f"/k8s/clusters/{cid}"
    for level in ("baseline", "restricted"):
        assert api("POST", f"{k}/api/v1/namespaces",
                   {"metadata": {"name": level, "labels": {"pod-security.kubernetes.io/enforce": level}}})[0] == 201
    host = _pod("host", hostNetwork=True, volumes=[{"name": "dev", "hostPath": {"path": "/dev"}}])
    assert api("POST", f"{k}/api/v1/namespaces/default/pods", host)[0] == 201  # privileged by default
    code, out = api("POST", f"{k}/api/v1/namespaces/baseline/pods", host)
    assert code == 403 and 'violates PodSecurity "baseline:latest"' in out["message"]
    assert "hostNetwork" in out["message"] and "hostPath" in out["message"]
    assert api("POST", f"{k}/api/v1/namespaces/baseline/pods", _pod("plain"))[0] == 201
    code, out = api("POST", f"{k}/api/v1/namespaces/restricted/pods", _pod("plain"))
    assert code == 403 and "runAsNonRoot" in out["message"] and "drop ALL" in out["message"]
    hardened = _pod("hard", securityContext={"runAsNonRoot": True, "seccompProfile": {"type": "RuntimeDefault"}})
    hardened["spec"]["containers"][0]["securityContext"] = {"allowPrivilegeEscalation": False,
                                                           "capabilities": {"drop": ["ALL"]}}
    assert api("POST", f"{k}/api/v1/namespaces/restricted/pods", hardened)[0] == 201


def test_admission_cluster_default_level_applies_to_unlabelled_namespaces():
    with FakeRancher(bootstrap_password="bootstrap-pw-0123", default_pod_security="baseline") as fake:
        code, out = Api(fake)("POST", "/v3-public/localProviders/local?action=login",
                              {"username": "admin", "password": "bootstrap-pw-0123"})
        api = Api(fake, out["token"])
        cid = _cluster_with_node(fake, api)
        code, out = api("POST", f"/k8s/clusters/{cid}/api/v1/namespaces/default/pods", _pod("p", hostPID=True))
        assert code == 403 and "baseline" in out["message"]
    with pytest.raises(ValueError):
        FakeRancher(default_pod_security="lenient")


def test_admission_webhook_failure_policy(fake, api):
    cid = _cluster_with_node(fake, api)
    k = f"/k8s/clusters/{cid}"
    hook = {"name": "inject.example.com", "sideEffects": "None", "admissionReviewVersions": ["v1"],
            "rules": [{"operations": ["CREATE"], "apiGroups": [""],
                                                     "apiVersions": ["v1"], "resources": ["pods"]}],
            "clientConfig": {"service": {"name": "nowhere", "namespace": "kube-system", "path": "/mutate"},
                             "caBundle": base64.b64encode(b"").decode()},
            "namespaceSelector": {"matchExpressions": [{"key": "inject", "operator": "In", "values": ["yes"]}]}}
    cfgs = f"{k}/apis/admissionregistration.k8s.io/v1/mutatingwebhookconfigurations"
    assert api("POST", cfgs, {"metadata": {"name": "fail"}, "webhooks": [dict(hook, failurePolicy="Fail")]})[0] == 201
    assert api("POST", f"{k}/api/v1/namespaces", {"metadata": {"name": "inj", "labels": {"inject": "yes"}}})[0] == 201
    # the selector does not match default: the unreachable webhook is never called
    assert api("POST", f"{k}/api/v1/namespaces/default/pods", _pod("a"))[0] == 201
    code, out = api("POST", f"{k}/api/v1/namespaces/inj/pods", _pod("b"))
    assert code == 400 and "failed calling webhook inject.example.com" in out["message"]
    assert api("GET", f"{k}/api/v1/namespaces/inj/pods/b")[0] == 404  # nothing stored
    assert api("GET", f"{k}/api/v1/namespaces/inj/pods")[1]["items"] == []
    # under Ignore the same failure lets the pod through unmodified
    ignore = api("GET", f"{cfgs}/fail")[1]
    ignore["webhooks"][0]["failurePolicy"] = "Ignore"
    assert api("PUT", f"{cfgs}/fail", ignore)[0] == 200
    assert api("POST", f"{k}/api/v1/namespaces/inj/pods", _pod("b"))[0] == 201


def test_client_upgrade_rereads_on_conflict(fake, api):
    """The provisioning controllers write the object too: the client's read-modify-write
    of ``spec.kubernetesVersion`` meets a 409 when one did so in between, re-reads and
    applies again instead of failing the upgrade."""
    from triton_kubernetes_amd.rancher.client import RancherClient

    obj = _rke2(api)
    user, _, secret = api.token.partition(":")
    client = RancherClient(fake.url, user, secret)
    real = fake._v2_cluster
    raced = []

    def controller_writes_first(method, key, body=None):
        if method == "PUT" and not raced:  # a status update lands between the read and the write
            raced.append(key)
            with fake.state.mu:
                fake.state.v2_clusters[key]["metadata"]["resourceVersion"] = fake._next_rv()
        return real(method, key, body)

    fake._v2_cluster = controller_writes_first
    client.upgrade_cluster(obj["status"]["clusterName"], RKE2_NEW)
    assert raced and fake.state.v2_clusters[f"{FLEET_NAMESPACE}/r1"]["spec"]["kubernetesVersion"] == RKE2_NEW
    assert [m for m, p in fake.state.log if m == "PUT"] == ["PUT", "PUT"]  # the 409, then the retry


def test_k8s_webhook_configuration_validation(fake, api):
    cid = _cluster_with_node(fake, api)
    cfgs = f"/k8s/clusters/{cid}/apis/admissionregistration.k8s.io/v1/mutatingwebhookconfigurations"
    good = {"name": "inject.amd.example.com", "sideEffects": "None", "admissionReviewVersions": ["v1"],
            "clientConfig": {"service": {"name": "s", "namespace": "kube-system"}}, "failurePolicy": "Ignore",
            "rules": []}
    for change, want in (({"sideEffects": "Unknown"}, "sideEffects"),
                         ({"admissionReviewVersions": []}, "admissionReviewVersions"),
                         ({"name": "inject"}, "three segments"),
                         ({"clientConfig": {}}, "exactly one of url or service"),
                         ({"clientConfig": {"url": "https://x", "service": {"name": "s"}}}, "exactly one"),
                         ({"failurePolicy": "Retry"}, "failurePolicy")):
        code, out = api("POST", cfgs, {"metadata": {"name": "bad"}, "webhooks": [dict(good, **change)]})
        assert code == 422 and want in out["message"], (change, out)
    code, out = api("POST", cfgs, {"metadata": {"name": "dup"}, "webhooks": [good, good]})
    assert code == 422 and "Duplicate" in out["message"]
    assert api("POST", cfgs, {"metadata": {"name": "ok"}, "webhooks": [good]})[0] == 201
    # the framework's own injector configuration passes the same validation
    from triton_kubernetes_amd.rancher.fake.k8s import _webhook_config_problem
    from triton_kubernetes_amd.k8s.addons import rendered_addons

    mine = [obj for path, obj in rendered_addons({"gpu_count": 8}) if obj.get("kind") == "MutatingWebhookConfiguration"]
    assert mine and all(_webhook_config_problem(o) == "" for o in mine)


def test_k8s_workload_validation(fake, api):
    cid = _cluster_with_node(fake, api)
    k = f"/k8s/clusters/{cid}"
    tmpl = {"metadata": {"labels": {"app": "x"}}, "spec": {"containers": [{"name": "c", "image": "busybox"}]}}
    ds = f"{k}/apis/apps/v1/namespaces/kube-system/daemonsets"
    code, out = api("POST", ds, {"metadata": {"name": "a"}, "spec": {"template": tmpl}})
    assert code == 422 and "spec.selector: Required" in out["message"]
    code, out = api("POST", ds, {"metadata": {"name": "a"}, "spec": {"selector": {"matchLabels": {"app": "y"}},
                                                                      "template": tmpl}})
    assert code == 422 and "does not match template" in out["message"]
    bare = {"metadata": {"labels": {"app": "x"}}, "spec": {"containers": [{"name": "c"}]}}
    code, out = api("POST", ds, {"metadata": {"name": "a"}, "spec": {"selector": {"matchLabels": {"app": "x"}},
                                                                      "template": bare}})
    assert code == 422 and "name and image" in out["message"]
    assert api("POST", ds, {"metadata": {"name": "a"}, "spec": {"selector": {"matchLabels": {"app": "x"}},
                                                                 "template": tmpl}})[0] == 201
    jobs = f"{k}/apis/batch/v1/namespaces/default/jobs"
    code, out = api("POST", jobs, {"metadata": {"name": "j"}, "spec": {"template": tmpl}})  # restartPolicy Always
    assert code == 422 and "restartPolicy" in out["message"]
    never = json.loads(json.dumps(tmpl))
    never["spec"]["restartPolicy"] = "Never"
    assert api("POST", jobs, {"metadata": {"name": "j"}, "spec": {"template": never}})[0] == 201
    # the framework's own add-ons pass the same validation
    from triton_kubernetes_amd.k8s.addons import rendered_addons
    from triton_kubernetes_amd.rancher.fake.k8s import _workload_problem

    for path, obj in rendered_addons({"gpu_count": 8, "node_labeller_image": "rocm/k8s-device-plugin:labeller-x"}):
        kind = path.rsplit("/", 1)[-1]
        if kind in ("daemonsets", "deployments", "jobs"):
            assert _workload_problem(kind, obj) == "", (path, obj["metadata"]["name"])


def test_k8s_core_object_validation(fake, api):
    cid = _cluster_with_node(fake, api)
    ns = f"/k8s/clusters/{cid}/api/v1/namespaces/kube-system"
    cases = [
        ("secrets", {"metadata": {"name": "s"}, "data": {"k": "not base64!"}}, "illegal base64"),
        ("secrets", {"metadata": {"name": "s"}, "type": "kubernetes.io/tls", "data": {"tls.crt": "eA=="}},
         "data[tls.key]: Required"),
        ("secrets", {"metadata": {"name": "s"}, "type": "kubernetes.io/service-account-token"},
         "service-account.name"),
        ("configmaps", {"metadata": {"name": "c"}, "data": {"bad key": "v"}}, "valid config key"),
        ("services", {"metadata": {"name": "svc"}, "spec": {"ports": [{"port": 70000}]}}, "between 1 and 65535"),
    ]
    for kind, body, want in cases:
        code, out = api("POST", f"{ns}/{kind}", body)
        assert code == 422 and want in out["message"], (kind, out)
    rb = f"/k8s/clusters/{cid}/apis/rbac.authorization.k8s.io/v1/clusterrolebindings"
    code, out = api("POST", rb, {"metadata": {"name": "b"}, "roleRef": {"kind": "ClusterRole", "name": "r"}})
    assert code == 422 and "roleRef.apiGroup" in out["message"]
    # the framework's own add-ons pass the same validation
    from triton_kubernetes_amd.k8s.addons import rendered_addons
    from triton_kubernetes_amd.k8s.tls import serving_cert
    from triton_kubernetes_amd.rancher.fake.k8s import _core_problem

    for path, obj in rendered_addons({"gpu_count": 8}, serving_cert("rccl-env-injector", "kube-system")):
        assert _core_problem(path.rsplit("/", 1)[-1], obj) == "", (path, obj["metadata"]["name"])
