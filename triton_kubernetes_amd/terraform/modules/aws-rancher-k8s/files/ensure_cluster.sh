#!/bin/bash
# S4 as a Terraform data "external" program (operator machine): find the RKE cluster
# by name or create it, then its registration token (reused when the cluster existed)
# and the checksum of the Rancher CA bundle.  Query keys: name, version, network,
# api_url, access_key, secret_key, registry, registry_username, registry_password.
exec python3 -c '
import base64, hashlib, json, re, ssl, sys, time, urllib.parse, urllib.request

q = json.load(sys.stdin)
ctx = ssl.create_default_context()
ctx.check_hostname, ctx.verify_mode = False, ssl.CERT_NONE  # self-signed Rancher certificates
auth = "Basic " + base64.b64encode((q["access_key"] + ":" + q["secret_key"]).encode()).decode()


def call(method, path, body=None):
    req = urllib.request.Request(q["api_url"].rstrip("/") + path, method=method,
                                 data=None if body is None else json.dumps(body).encode(),
                                 headers={"Authorization": auth, "Accept": "application/json",
                                          "Content-Type": "application/json"})
    with urllib.request.urlopen(req, context=ctx, timeout=60) as resp:
        return json.load(resp)


def k8s_version(requested):
    # requested if the server offers it, else its newest release of the same minor
    offered = [v for v in call("GET", "/v3/settings/k8s-versions-current").get("value", "").split(",") if v]
    if not offered or requested in offered:
        return requested
    minor = requested.split(".")[:2]
    same = [v for v in offered if v.split(".")[:2] == minor]
    if not same:
        sys.exit("Kubernetes version %s is not offered by the Rancher server (offered: %s)"
                 % (requested, ", ".join(offered)))
    return max(same, key=lambda v: [int(x) for x in re.findall(r"[0-9]+", v)])


found = call("GET", "/v3/clusters?name=" + urllib.parse.quote(q["name"])).get("data") or []
if found:
    cluster_id = found[0]["id"]
else:
    rke = {"type": "rancherKubernetesEngineConfig", "kubernetesVersion": k8s_version(q["version"]),
           "ignoreDockerVersion": False, "sshAgentAuth": False,
           "authentication": {"type": "authnConfig", "strategy": "x509"},
           "network": {"type": "networkConfig", "plugin": q["network"]},
           "services": {"type": "rkeConfigServices",
                        "kubeApi": {"type": "kubeAPIService", "podSecurityPolicy": False}}}
    if q.get("registry"):
        rke["privateRegistries"] = [{"url": q["registry"], "user": q.get("registry_username", ""),
                                     "password": q.get("registry_password", "")}]
    cluster_id = call("POST", "/v3/cluster", {"type": "cluster", "name": q["name"],
                                              "rancherKubernetesEngineConfig": rke}).get("id", "")
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
cacerts = call("GET", "/v3/settings/cacerts").get("value", "")
print(json.dumps({"cluster_id": cluster_id, "registration_token": token,
                  "ca_checksum": hashlib.sha256((cacerts + "\n").encode()).hexdigest()}))
'
