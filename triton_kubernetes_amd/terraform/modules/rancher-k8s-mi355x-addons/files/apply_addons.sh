#!/bin/bash
# MI355X cluster add-ons: wait for the cluster, then create the manifests in
# $MANIFEST_DIR through Rancher's Kubernetes proxy (PUT on 409).  TLS is verified against
# the manager's pinned CA (RANCHER_CA; empty: the system trust store).  With a private CA the
# chain is checked, not the hostname (rancher/trust.py RancherTrust.context): curl has no
# such mode, so the calls are Python's.
set -euo pipefail
exec python3 -c '
import base64, glob, json, os, ssl, sys, time, urllib.error, urllib.request

ca = os.environ.get("RANCHER_CA", "").strip()
if ca:
    ctx = ssl.create_default_context(cadata=ca + "\n")
    ctx.check_hostname = False  # the chain to this manager s own CA
else:
    ctx = ssl.create_default_context()
url, cid = os.environ["RANCHER_URL"].rstrip("/"), os.environ["CLUSTER_ID"]
auth = "Basic " + base64.b64encode((os.environ["RANCHER_ACCESS_KEY"] + ":" +
                                    os.environ["RANCHER_SECRET_KEY"]).encode()).decode()


def call(method, path, body=None):
    req = urllib.request.Request(url + path, method=method, data=None if body is None else json.dumps(body).encode(),
                                 headers={"Authorization": auth, "Content-Type": "application/json",
                                          "Accept": "application/json"})
    try:
        with urllib.request.urlopen(req, context=ctx, timeout=60) as resp:
            return resp.status, resp.read()
    except urllib.error.HTTPError as exc:
        return exc.code, exc.read()


state = ""
for _ in range(3600):
    try:
        code, raw = call("GET", "/v3/clusters/" + cid)
        state = json.loads(raw).get("state", "") if code == 200 else ""
    except (OSError, ValueError) as exc:
        if isinstance(getattr(exc, "reason", None), ssl.SSLError) or isinstance(exc, ssl.SSLError):
            sys.exit("the Rancher server certificate does not verify against the CA pinned for this cluster "
                     "manager: " + str(exc))
        state = ""
    if state == "active":
        break
    time.sleep(1)
if state != "active":
    sys.exit("cluster " + cid + " not active")
for f in sorted(glob.glob(os.path.join(os.environ["MANIFEST_DIR"], "*.json"))):
    doc = json.load(open(f))
    path, obj = doc["path"], doc["object"]
    code, raw = call("POST", "/k8s/clusters/" + cid + path, obj)
    if code == 409:
        code, raw = call("PUT", "/k8s/clusters/" + cid + path + "/" + obj["metadata"]["name"], obj)
    if code >= 300:
        sys.exit("applying " + f + ": HTTP " + str(code))
'
