#!/bin/bash
# S4 as a Terraform data "external" program (operator machine): find the cluster by
# name or create it, then its registration token (reused when the cluster existed) and
# the checksum of the Rancher CA bundle.  Query keys: name, version, network,
# distribution (rke2 | rke1), api_url, access_key, secret_key, registry,
# registry_username, registry_password.  RKE2: a provisioning.cattle.io/v1 Cluster in
# fleet-default whose management cluster (status.clusterName) holds the token; RKE1:
# the v3 cluster with rancherKubernetesEngineConfig (the reference's flow).
# Query key operation (the executor's tk_operation): apply finds or creates; destroy and
# read only find -- a destroy must never re-create a cluster removed out of band -- and
# a Rancher that is gone or unreachable then yields empty outputs instead of an error.
exec python3 -c '
import base64, hashlib, json, re, ssl, sys, time, urllib.error, urllib.parse, urllib.request

q = json.load(sys.stdin)
# TLS verified against the CA pinned for the manager (query key ca_pem = tk_rancher_ca,
# rendered by the executor; rancher/trust.py); none pinned: a publicly trusted certificate
pinned = q.get("ca_pem", "").strip()
pinned = pinned + "\n" if pinned else ""
ctx = ssl.create_default_context(cadata=pinned) if pinned else ssl.create_default_context()
if pinned:
    ctx.check_hostname = False  # the chain to this server s own CA; rancher/trust.py RancherTrust.context
auth = "Basic " + base64.b64encode((q["access_key"] + ":" + q["secret_key"]).encode()).decode()


def call(method, path, body=None):
    req = urllib.request.Request(q["api_url"].rstrip("/") + path, method=method,
                                 data=None if body is None else json.dumps(body).encode(),
                                 headers={"Authorization": auth, "Accept": "application/json",
                                          "Content-Type": "application/json"})
    try:
        with urllib.request.urlopen(req, context=ctx, timeout=60) as resp:
            return json.load(resp)
    except urllib.error.URLError as exc:
        if isinstance(exc.reason, ssl.SSLCertVerificationError):
            sys.exit("the Rancher server at %s presented a certificate that does not verify against %s (%s): "
                     "refusing to send the API key. If its CA was rotated on purpose, pin the new one with "
                     "rancher_ca_file=<PEM bundle>" % (q["api_url"], "the CA pinned for this cluster manager"
                                                       if pinned else "the system trust store", exc.reason))
        raise


def get_or_none(path):
    try:
        return call("GET", path)
    except urllib.error.HTTPError as exc:
        if exc.code == 404:
            return None
        raise


def k8s_version(requested, rke2=False):
    # requested if the server offers it, else its newest release of the same minor
    if rke2:
        offered = [r.get("version") or r.get("id") for r in call("GET", "/v1-rke2-release/releases").get("data", [])]
    else:
        offered = [v for v in call("GET", "/v3/settings/k8s-versions-current").get("value", "").split(",") if v]
    if not offered or requested in offered:
        return requested
    minor = requested.split(".")[:2]
    same = [v for v in offered if v.split(".")[:2] == minor]
    if not same:
        sys.exit("Kubernetes version %s is not offered by the Rancher server (offered: %s)"
                 % (requested, ", ".join(offered)))
    return max(same, key=lambda v: [int(x) for x in re.findall(r"[0-9]+", v)])


def ca_checksum():
    # the checksum nodes pin: of the pinned bundle (read on the manager host), not of what the
    # server says now
    cacerts = pinned or call("GET", "/v3/settings/cacerts").get("value", "")
    if cacerts and not cacerts.endswith("\n"):
        cacerts += "\n"  # Rancher hashes the bundle with one trailing newline, as /cacerts serves it
    return hashlib.sha256(cacerts.encode()).hexdigest() if cacerts else ""


op = q.get("operation", "apply")
if op != "apply":
    out = {"cluster_id": "", "registration_token": "", "ca_checksum": ""}
    try:
        found = call("GET", "/v3/clusters?name=" + urllib.parse.quote(q["name"])).get("data") or []
        if found:
            out["cluster_id"] = found[0]["id"]
            toks = call("GET", "/v3/clusters/%s/clusterregistrationtokens" % found[0]["id"]).get("data") or []
            out["registration_token"] = (toks[0].get("token") or "") if toks else ""
            out["ca_checksum"] = ca_checksum()
    except Exception as exc:  # noqa: BLE001 - find-only: nothing to create, nothing to fail
        sys.stderr.write("ensure_cluster (%s): %s\n" % (op, exc))
    print(json.dumps(out))
    sys.exit(0)

dist = q.get("distribution", "rke2")
v3 = call("GET", "/v3/clusters?name=" + urllib.parse.quote(q["name"])).get("data") or []
if v3 and ("rke2" if v3[0].get("driver") == "rke2" else "rke1") != dist:
    sys.exit("cluster %s already exists as an %s cluster; it cannot be reused as %s"
             % (q["name"], "RKE1" if dist == "rke2" else "RKE2", dist.upper()))


def ensure_rke2():
    v2 = "/v1/provisioning.cattle.io.clusters"
    path = v2 + "/fleet-default/" + urllib.parse.quote(q["name"])
    existing = get_or_none(path)
    found = [existing] if existing else []
    if not found:
        rke = {"machineGlobalConfig": {"cni": q["network"]}, "machinePools": []}
        if q.get("registry"):
            conf = {}
            if q.get("registry_username"):
                # credentials: a basic-auth Secret in fleet-default that the config names
                b64 = lambda v: base64.b64encode(v.encode()).decode()
                secret = call("POST", "/v1/secrets", {
                    "type": "kubernetes.io/basic-auth",
                    "metadata": {"generateName": "registryconfig-auth-", "namespace": "fleet-default"},
                    "data": {"username": b64(q["registry_username"]), "password": b64(q.get("registry_password", ""))}})
                conf["authConfigSecretName"] = secret["metadata"]["name"]
            rke["registries"] = {"mirrors": {"docker.io": {"endpoint": ["https://" + q["registry"]]}},
                                 "configs": {q["registry"]: conf}}
        call("POST", v2, {"apiVersion": "provisioning.cattle.io/v1", "kind": "Cluster",
                          "metadata": {"name": q["name"], "namespace": "fleet-default"},
                          "spec": {"kubernetesVersion": k8s_version(q["version"], True), "rkeConfig": rke}})
    cluster_id, delay, deadline = "", 0.05, time.time() + 120
    while not cluster_id and time.time() < deadline:
        # the provisioning controller creates the management cluster (c-m-...) after the create
        cluster_id = ((get_or_none(path) or {}).get("status") or {}).get("clusterName", "")
        if not cluster_id:
            time.sleep(delay)
            delay = min(2.0, delay * 2)
    return found, cluster_id


def ensure_rke1():
    found = v3
    if found:
        return found, found[0]["id"]
    rke = {"type": "rancherKubernetesEngineConfig", "kubernetesVersion": k8s_version(q["version"]),
           "ignoreDockerVersion": False, "sshAgentAuth": False,
           "authentication": {"type": "authnConfig", "strategy": "x509"},
           "network": {"type": "networkConfig", "plugin": q["network"]},
           "services": {"type": "rkeConfigServices",
                        "kubeApi": {"type": "kubeAPIService", "podSecurityPolicy": False}}}
    if q.get("registry"):
        rke["privateRegistries"] = [{"url": q["registry"], "user": q.get("registry_username", ""),
                                     "password": q.get("registry_password", "")}]
    return found, call("POST", "/v3/cluster", {"type": "cluster", "name": q["name"],
                                               "rancherKubernetesEngineConfig": rke}).get("id", "")


found, cluster_id = ensure_rke2() if dist == "rke2" else ensure_rke1()
if not cluster_id:
    sys.exit("Unable to create cluster!")
tokens = call("GET", "/v3/clusters/%s/clusterregistrationtokens" % cluster_id).get("data") if found else []
token = tokens[0].get("token") if tokens else ""
if not token:
    created = call("POST", "/v3/clusterregistrationtoken", {"type": "clusterRegistrationToken",
                                                             "clusterId": cluster_id})
    token, delay, deadline = created.get("token"), 0.05, time.time() + 120
    while not token and created.get("id") and time.time() < deadline:
        # the server fills the value in after the create returns
        time.sleep(delay)
        delay = min(2.0, delay * 2)
        token = call("GET", "/v3/clusterregistrationtokens/" + created["id"]).get("token")
if not token:
    sys.exit("Unable to create cluster registration token!")
print(json.dumps({"cluster_id": cluster_id, "registration_token": token, "ca_checksum": ca_checksum()}))
'
