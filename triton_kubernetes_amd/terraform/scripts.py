"""Bootstrap scripts and templates shipped inside the Terraform modules (S1-S6 + MI355X).

Terraform ``templatefile`` syntax: ``${var}`` is substituted, ``$${x}`` is a
literal ``${x}`` and ``%{ if }`` directives are available.  These are fresh
scripts for a current Rancher 2.x / Docker, not the reference's 0.11-era
templates, and they fix the reference quirks Q10
(hard-coded ``/home/ubuntu``, ``/etc/fstab`` overwritten with ``tee``).
"""

from ..node.hosttune import shell_check as _host_tuning_check
from ..parallel.hostkeys import GO_HOSTKEY_ALGORITHMS
from ..node.metrics import textfile_script as _metrics_textfile
from ..node.tools import NODE_TOOLS_FN, PREBUILT_DIR
from ..rancher.trust import HOST_CA_READ as _HOST_CA_READ

# download, verify (when docker_install_sha256 is set), run — no `curl | sh` of an unchecked stream
DOCKER_INSTALL = r"""if ! command -v docker >/dev/null 2>&1; then
  curl -fsSL -o /tmp/tk-install-docker.sh '${docker_engine_install_url}'
%{ if docker_install_sha256 != "" ~}
  echo '${docker_install_sha256}  /tmp/tk-install-docker.sh' | sha256sum -c - >/dev/null || { echo 'docker install script checksum mismatch' >&2; exit 1; }
%{ endif ~}
  sudo sh /tmp/tk-install-docker.sh && rm -f /tmp/tk-install-docker.sh
fi"""

INSTALL_DOCKER = r"""#!/bin/bash
# S1/S6: container runtime for a Rancher manager or node (cloud-init / remote-exec).
set -euo pipefail
if command -v firewalld >/dev/null 2>&1; then
  sudo systemctl disable --now firewalld.service || true
fi
""" + DOCKER_INSTALL + r"""
if [ ! -f /etc/docker/daemon.json ]; then
  if mountpoint -q /mnt; then
    echo '{"storage-driver": "overlay2", "data-root": "/mnt/docker"}' | sudo tee /etc/docker/daemon.json >/dev/null
  else
    echo '{"storage-driver": "overlay2"}' | sudo tee /etc/docker/daemon.json >/dev/null
  fi
  sudo systemctl restart docker || sudo service docker restart
fi
%{ if rancher_registry_username != "" ~}
echo '${rancher_registry_password}' | sudo docker login -u '${rancher_registry_username}' --password-stdin '${rancher_registry}'
%{ endif ~}
%{ if rancher_server_image != "" ~}
sudo docker pull '${rancher_server_image}'
%{ endif ~}
"""

INSTALL_RANCHER_SERVER = r"""#!/bin/bash
# S2: run the Rancher server container once docker and the image are present.
set -euo pipefail
for i in $(seq 1 600); do command -v docker >/dev/null 2>&1 && break; sleep 1; done
for i in $(seq 1 600); do sudo docker image inspect '${rancher_server_image}' >/dev/null 2>&1 && break; sudo docker pull '${rancher_server_image}' || sleep 1; done
[ -n '${bootstrap_password}' ] || { echo 'rancher_bootstrap_password is empty (the CLI passes the random one it keeps in the state backend)' >&2; exit 1; }
if ! sudo docker ps --format '{{.Image}}' | grep -x '${rancher_server_image}' >/dev/null; then
  # Rancher >= 2.6 has no admin/admin: the first login uses this bootstrap password (random,
  # kept in the state backend: rancher/bootstrap_secret.py), handed over in a 0600 env file
  # that is removed once the container runs -- never on a command line
  envf=$(umask 077; mktemp)
  trap 'rm -f "$envf"' EXIT
  cat > "$envf" <<'TK_BOOTSTRAP_EOF'
CATTLE_BOOTSTRAP_PASSWORD=${bootstrap_password}
TK_BOOTSTRAP_EOF
  sudo docker run -d --restart=unless-stopped --privileged -p 80:80 -p 443:443 --env-file "$envf" \
    '${rancher_server_image}'
  rm -f "$envf"
fi
"""

SETUP_RANCHER = r"""#!/bin/bash
# S3 on the manager: log in with the bootstrap password, create the API token
# (-> ~/rancher_api_key), set server-url, and save the server's CA bundle as served here
# (https://127.0.0.1: loopback, nothing between) to ~/rancher_cacerts.pem.  The admin
# password is set from the operator side (read_api_key.sh), over TLS verified against that
# bundle: it never reaches this host.  A re-run finds the token and only refreshes the CA.
set -euo pipefail
R='${rancher_host}'
for i in $(seq 1 900); do curl -ksf "$R/ping" >/dev/null 2>&1 && break; sleep 1; done
umask 077
curl -ksf "$R/cacerts" > ~/rancher_cacerts.pem.tmp && mv ~/rancher_cacerts.pem.tmp ~/rancher_cacerts.pem
[ -s ~/rancher_api_key ] && exit 0
json() { python3 -c "import json,sys; print(json.load(sys.stdin)$1)"; }
login=$(curl -ksf -X POST -H 'Content-Type: application/json' --data-binary @- \
  "$R/v3-public/localProviders/local?action=login" <<'TK_EOF'
{"username":"admin","password":${jsonencode(bootstrap_password)},"ttl":60000,"description":"Initial Token"}
TK_EOF
)
initial=$(printf '%s' "$login" | json '["token"]')
tok=$(curl -ksf -u "$initial" -X POST -H 'Content-Type: application/json' \
  -d '{"type":"token","name":"triton-kubernetes","description":"Managed by triton-kubernetes","ttl":0}' "$R/v3/token")
printf '%s' "$tok" > ~/rancher_api_key
ak=$(printf '%s' "$tok" | json '["name"]')
sk=$(printf '%s' "$tok" | json '["token"].split(":",1)[1]')
curl -ksf -u "$ak:$sk" -X PUT -H 'Content-Type: application/json' \
  -d '{"name":"server-url","value":"${host_registration_url}"}' "$R/v3/settings/server-url" >/dev/null
"""

SSH_PINNED = r"""# SSH with the cluster manager's pinned host keys (query key known_hosts, the executor's
# tk_known_hosts; parallel/hostkeys.py): a known host's key must match, an unknown one is
# pinned on this first contact and reported back (result key known_hosts).
kh=$(mktemp); err=$(mktemp); trap 'rm -f "$kh" "$err"' EXIT
printf '%s\n' "${known_hosts:-}" > "$kh"
# host key algorithms in Go's order (Terraform's client): the key pinned here is the type
# Terraform's provisioner connections negotiate; UpdateHostKeys pins the host's other keys
ko=(-o "UserKnownHostsFile=$kh" -o StrictHostKeyChecking=accept-new -o HashKnownHosts=no -o GlobalKnownHostsFile=/dev/null
    -o "HostKeyAlgorithms=@@HKA@@" -o UpdateHostKeys=yes)
key="${key_path/#\~/$HOME}"
opts=(-o BatchMode=yes -o LogLevel=ERROR "${ko[@]}" -i "$key")
if [ -n "${bastion_host:-}" ]; then
  opts+=(-o "ProxyCommand=ssh -o BatchMode=yes -o LogLevel=ERROR $(printf '%q ' "${ko[@]}" -i "$key")-W %h:%p $(printf '%q' "$ssh_user@$bastion_host")")
fi
pinned_for() { python3 -c 'import sys; hs=set(sys.argv[2:]); print("".join(l for l in open(sys.argv[1]) if l.split() and l.split()[0] in hs), end="")' "$kh" "$host" ${bastion_host:+"$bastion_host"}; }
refused() {
  if grep -q -e 'Host key verification failed' -e 'REMOTE HOST IDENTIFICATION HAS CHANGED' "$err"; then
    echo "the SSH host key of $host${bastion_host:+ (or its bastion $bastion_host)} does not match the key pinned for this cluster manager; refusing to $1. If the machine was reinstalled, run 'triton-kubernetes forget host-key' with host=$host and retry." >&2
  else
    cat "$err" >&2
    echo "could not $1 ($host)" >&2
  fi
  exit 1
}
""".replace("@@HKA@@", ",".join(GO_HOSTKEY_ALGORITHMS))

READ_API_KEY = r"""#!/bin/bash
# data "external" program (operator machine): read the manager's ~/rancher_api_key and the
# server's CA bundle (~/rancher_cacerts.pem, saved on the host from its own loopback) over
# the pinned SSH session, then -- on apply -- set the admin password: a curl on the host
# against its loopback, with the credentials and the request body on curl's stdin (a
# config, "-K -"), which is this SSH session's stdin.  The admin password is never on a
# command line, in a file or in a rendered script on the host (rancher/bootstrap_secret.py).
# Replaces the reference's matti/outputs/shell registry module.  Outside an apply (query
# key operation = destroy | read, the executor's tk_operation) a manager that cannot be
# reached yields empty keys instead of an error: destroying what is left of a manager whose
# host is gone must not depend on that host.
set -euo pipefail
eval "$(python3 -c 'import json,shlex,sys; q=json.load(sys.stdin); print(" ".join(f"{k}={shlex.quote(str(v))}" for k,v in q.items()))')"
""" + SSH_PINNED + r"""if ! tok=$(ssh "${opts[@]}" "$ssh_user@$host" 'cat ~/rancher_api_key' 2>"$err"); then
  if [ "${operation:-apply}" != apply ]; then echo '{"access_key": "", "secret_key": "", "known_hosts": "", "ca_certs": ""}'; exit 0; fi
  refused "read the Rancher API key"
fi
# the bundle as saved on the host, or -- an older install that never saved it -- read there
# now from the server's own loopback (rancher/trust.py HOST_CA_READ).  Empty only when the
# server's cacerts setting is (a publicly trusted certificate); a failed read fails here
# rather than pinning an empty bundle
if ! ca=$(ssh "${opts[@]}" "$ssh_user@$host" 'bash -s' 2>"$err" <<'TK_CA_EOF'
@@HOST_CA_READ@@TK_CA_EOF
); then
  if [ "${operation:-apply}" != apply ]; then echo '{"access_key": "", "secret_key": "", "known_hosts": "", "ca_certs": ""}'; exit 0; fi
  refused "read the Rancher CA bundle"
fi
if [ "${operation:-apply}" = apply ] && [ -n "${admin_password:-}" ] && [ "${admin_password:-}" != "${bootstrap_password:-}" ]; then
  # curl config on stdin: user (the API token), the JSON body with both passwords
  cfg=$(printf '%s' "$tok" | TKQ_admin="$admin_password" TKQ_boot="$bootstrap_password" python3 -c '
import json, os, sys
t = json.load(sys.stdin)
q = lambda v: json.dumps(v)  # a curl config string: double-quoted, backslash escapes
body = json.dumps({"currentPassword": os.environ["TKQ_boot"], "newPassword": os.environ["TKQ_admin"]})
print("user = " + q(t["token"]))
print("header = " + q("Content-Type: application/json"))
print("data = " + q(body))')
  code=$(printf '%s
' "$cfg" | ssh "${opts[@]}" "$ssh_user@$host" \
    'curl -ks -K - -o /dev/null -w "%{http_code}" -X POST "https://127.0.0.1/v3/users?action=changepassword"' 2>"$err") \
    || refused "set the Rancher admin password"
  # 422: the current password is no longer the bootstrap one -- set by an earlier run, or the
  # bootstrap password is wrong: the admin password must then log in, or this is an error
  case "$code" in
    2??|"") ;;
    422)
      login_cfg=$(TKQ_admin="$admin_password" python3 -c '
import json, os
print("header = " + json.dumps("Content-Type: application/json"))
print("data = " + json.dumps(json.dumps({"username": "admin", "password": os.environ["TKQ_admin"], "ttl": 60000,
                                          "description": "triton-kubernetes admin password check"})))')
      lc=$(printf '%s\n' "$login_cfg" | ssh "${opts[@]}" "$ssh_user@$host" \
        'curl -ks -K - -o /dev/null -w "%{http_code}" -X POST "https://127.0.0.1/v3-public/localProviders/local?action=login"' \
        2>"$err") || refused "check the Rancher admin password"
      case "$lc" in 2??) ;; *) echo "setting the Rancher admin password on $host: the server refused the bootstrap password and the admin password does not log in (HTTP $lc): is rancher_bootstrap_password the server's?" >&2; exit 1 ;; esac ;;
    *) echo "setting the Rancher admin password on $host: HTTP $code" >&2; exit 1 ;;
  esac
fi
printf '%s' "$tok" | KH="$(pinned_for)" CA="$ca" python3 -c '
import json, os, sys
t = json.load(sys.stdin)
ca = os.environ["CA"].strip()
print(json.dumps({"access_key": t["name"], "secret_key": t["token"].split(":", 1)[1], "known_hosts": os.environ["KH"],
                  "ca_certs": ca + "\n" if ca else ""}))'
"""

READ_API_KEY = READ_API_KEY.replace("@@HOST_CA_READ@@", _HOST_CA_READ)

RANCHER_CLUSTER = r"""#!/bin/bash
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
"""

# How a node joins its cluster: RKE2 -> the server's rancher-system-agent installer (RKE2
# brings its own containerd: no Docker); RKE1 -> docker run rancher/rancher-agent.
JOIN_CLUSTER = r"""%{ if k8s_distribution == "rke2" ~}
# the installer over TLS verified against the server's CA, which must first match the
# cluster's CA checksum (an empty CA: a publicly trusted certificate)
installer=$(mktemp); ca=$(mktemp)
curl -fsSLk -o "$ca" '${rancher_api_url}/cacerts'
if [ -s "$ca" ]; then
  [ "$(sha256sum < "$ca" | cut -d' ' -f1)" = '${rancher_cluster_ca_checksum}' ] || { echo 'the Rancher CA does not match the cluster CA checksum' >&2; exit 1; }
  curl -fsSL --cacert "$ca" -o "$installer" '${rancher_api_url}/system-agent-install.sh'
else
  curl -fsSL -o "$installer" '${rancher_api_url}/system-agent-install.sh'
fi
sudo sh "$installer" --server '${rancher_api_url}' --label 'cattle.io/os=linux' \
  --token '${rancher_cluster_registration_token}' --ca-checksum '${rancher_cluster_ca_checksum}' \
  --node-name '${hostname}' --${rancher_node_role}${extra_agent_args}
rm -f "$installer" "$ca"
%{ else ~}
sudo docker run -d --privileged --restart=unless-stopped --net=host \
  -v /etc/kubernetes:/etc/kubernetes -v /var/run:/var/run '${rancher_agent_image}' \
  --server '${rancher_api_url}' --token '${rancher_cluster_registration_token}' \
  --ca-checksum '${rancher_cluster_ca_checksum}' --${rancher_node_role}${extra_agent_args}
%{ endif ~}"""

INSTALL_RANCHER_AGENT = r"""#!/bin/bash
# S5: join a node to the cluster (user-data or remote-exec).
set -euo pipefail
if command -v firewalld >/dev/null 2>&1; then sudo systemctl disable --now firewalld.service || true; fi
%{ if k8s_distribution == "rke1" ~}
""" + DOCKER_INSTALL + r"""
if [ ! -f /etc/docker/daemon.json ]; then
  echo '{"storage-driver": "overlay2"}' | sudo tee /etc/docker/daemon.json >/dev/null
  sudo systemctl restart docker || sudo service docker restart
fi
%{ endif ~}
sudo hostnamectl set-hostname '${hostname}'
grep -q ' ${hostname}$' /etc/hosts || echo '127.0.0.1 ${hostname}' | sudo tee -a /etc/hosts >/dev/null
%{ if rancher_registry_username != "" && k8s_distribution == "rke1" ~}
echo '${rancher_registry_password}' | sudo docker login -u '${rancher_registry_username}' --password-stdin '${rancher_registry}'
%{ endif ~}
%{ if disk_device != "" && disk_mount_path != "" ~}
# data disk: first of the candidate device names that exists; appended to fstab (never overwritten)
for dev in ${disk_device}; do
  if [ -b "$dev" ]; then
    if ! sudo blkid "$dev" >/dev/null 2>&1; then sudo mkfs.ext4 -q -E nodiscard "$dev"; fi
    sudo mkdir -p '${disk_mount_path}'
    uuid=$(sudo blkid -s UUID -o value "$dev")
    grep -q "$uuid" /etc/fstab || echo "UUID=$uuid ${disk_mount_path} ext4 defaults,noatime,nofail 0 2" | sudo tee -a /etc/fstab >/dev/null
    sudo mount -a
    break
  fi
done
%{ endif ~}
""" + JOIN_CLUSTER + "\n"

# Single-target RCCL, shell form of ops/rccl_slim.py (nodes delivered by SSH / Terraform).
# OPT-IN (rccl_slim = "on"): a copy of librccl whose .hip_fatbin holds only the gfx950 code
# object, uncompressed and without DWARF, so a cold process's first communicator init skips
# decompressing every GPU target.  It is a modified vendor binary, so by default nothing
# uses it: rccl-ready loads /opt/rocm/lib/librccl.so (RUNPATH).  When enabled,
# tk_rccl_slim_enable verifies the copy with a one-rank all-reduce that must map it, and
# only then installs the rccl-ready-slim wrapper, which uses the copy while it still
# matches the installed librccl (a ROCm upgrade falls back to the installed RCCL with a
# warning).  Written without brace expansions: the same text is a Terraform templatefile
# fragment and plain bash.
RCCL_SLIM_ROOT = "/var/lib/triton-kubernetes/rccl-slim"
RCCL_SLIM_FN = r"""tk_rccl_slim() { # <cache root> <rocm dir>: prints the slim runtime directory
  local root=$1 rocm=$2 llvm real key out tmp sec off size nb f n
  llvm=$rocm/lib/llvm/bin; [ -x $llvm/clang-offload-bundler ] || llvm=$rocm/llvm/bin
  for f in clang-offload-bundler llvm-objcopy llvm-readelf; do
    [ -x $llvm/$f ] || { echo "rccl slim: $f not found" >&2; return 1; }
  done
  real=$(readlink -f $rocm/lib/librccl.so) || return 1
  key=$(stat -c '%s-%Y' "$real")-$(head -c 1048576 "$real" | sha256sum | cut -c1-16)
  out=$root/gfx950-sh-$key
  if [ ! -f $out/slim.json ]; then
    mkdir -p $root && tmp=$(mktemp -d $root/.tmp-XXXXXX) && chmod 755 $tmp || return 1
    sec=$($llvm/llvm-readelf -S -W "$real" | sed 's/^ *\[ *[0-9]*\] *//' | awk '$1 == ".hip_fatbin" {print $4, $5}')
    if [ -z "$sec" ]; then rm -rf $tmp; echo "rccl slim: no .hip_fatbin in $real" >&2; return 1; fi
    off=$((16#$(echo $sec | cut -d' ' -f1))); size=$((16#$(echo $sec | cut -d' ' -f2))); nb=$size
    # a compressed bundle (CCOB) may be shorter than its section: its header holds the size
    if [ "$(head -c $((off + 4)) "$real" | tail -c 4)" = CCOB ]; then
      case $(od -An -t u2 -j $((off + 4)) -N 2 "$real" | tr -d ' ') in
        2) nb=$(od -An -t u4 -j $((off + 8)) -N 4 "$real" | tr -d ' ') ;;
        1) ;;
        *) nb=$(od -An -t u8 -j $((off + 8)) -N 8 "$real" | tr -d ' ') ;;
      esac
    fi
    dd if="$real" of=$tmp/fat.bin iflag=skip_bytes,count_bytes skip=$off count=$nb status=none
    : > $tmp/host
    if ! { $llvm/clang-offload-bundler --unbundle --type=o --input=$tmp/fat.bin \
             --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$tmp/full.co &&
           $llvm/llvm-objcopy --strip-debug $tmp/full.co $tmp/gfx950.co &&
           env -u OFFLOAD_BUNDLER_COMPRESS $llvm/clang-offload-bundler --type=o --bundle-align=4096 \
             --targets=host-x86_64-unknown-linux-gnu-,hipv4-amdgcn-amd-amdhsa--gfx950 \
             --input=$tmp/host --input=$tmp/gfx950.co --output=$tmp/new.bin &&
           [ $(stat -c %s $tmp/new.bin) -le $size ]; }; then
      rm -rf $tmp; echo 'rccl slim: cannot build the gfx950 bundle' >&2; return 1
    fi
    nb=$(stat -c %s $tmp/new.bin)
    cp "$real" $tmp/librccl.so
    head -c $size /dev/zero | dd of=$tmp/librccl.so oflag=seek_bytes seek=$off conv=notrunc status=none
    dd if=$tmp/new.bin of=$tmp/librccl.so oflag=seek_bytes seek=$off conv=notrunc status=none
    rm -f $tmp/fat.bin $tmp/full.co $tmp/gfx950.co $tmp/host $tmp/new.bin
    for f in $rocm/lib/lib*.so*; do
      n=$(basename $f)
      case $n in
        librccl.so) ;;
        librccl.so*) ln -s librccl.so $tmp/$n ;;
        *) ln -s "$(readlink -f $f)" $tmp/$n ;;
      esac
    done
    printf '{"source": "%s", "arch": "gfx950", "form": "shell", "bundle_bytes": %s}\n' "$real" $nb > $tmp/slim.json
    mv -T $tmp $out 2>/dev/null || rm -rf $tmp
  fi
  echo $out
}"""

# written next to the node tools by tk_rccl_slim_enable: the verified copy and its source
RCCL_SLIM_ENV = "rccl-slim.env"
RCCL_SLIM_ENABLE_FN = r"""tk_rccl_slim_enable() { # <cache root> <rocm dir> <tools dir>: opt-in, verified before use
  local dir real
  rm -f $3/""" + RCCL_SLIM_ENV + r""" $3/rccl-ready-slim
  dir=$(tk_rccl_slim $1 $2) || return 1
  real=$(readlink -f $2/lib/librccl.so) || return 1
  if ! LD_LIBRARY_PATH=$dir $3/rccl-ready --ngpus 1 --max-mib 4 --iters 2 --expect-rccl $dir/librccl.so >/dev/null; then
    echo "rccl slim: $dir failed its one-rank verified all-reduce; not enabled" >&2; return 1
  fi
  printf 'TK_RCCL_SLIM_DIR=%s\nTK_RCCL_SLIM_SOURCE=%s\nTK_RCCL_SLIM_KEY=%s\n' $dir "$real" "$(stat -c %s-%Y "$real")" \
    > $3/""" + RCCL_SLIM_ENV + r"""
  cat > $3/rccl-ready-slim <<'TK_SLIM_EOF'
#!/bin/sh
# rccl-ready on the verified single-target RCCL copy while it matches the installed librccl
. "$(dirname "$0")/""" + RCCL_SLIM_ENV + r""""
rocm=/opt/rocm; [ -n "$ROCM_PATH" ] && rocm=$ROCM_PATH
real=$(readlink -f "$rocm/lib/librccl.so")
if [ "$real" = "$TK_RCCL_SLIM_SOURCE" ] && [ "$(stat -c %s-%Y "$real")" = "$TK_RCCL_SLIM_KEY" ]; then
  if [ -n "$LD_LIBRARY_PATH" ]; then LD_LIBRARY_PATH=$TK_RCCL_SLIM_DIR:$LD_LIBRARY_PATH; else LD_LIBRARY_PATH=$TK_RCCL_SLIM_DIR; fi
  export LD_LIBRARY_PATH
else
  echo "rccl-ready-slim: librccl changed since the single-target copy was verified; using the installed RCCL (re-run the rccl_slim step)" >&2
fi
exec "$(dirname "$0")/rccl-ready" "$@"
TK_SLIM_EOF
  chmod 755 $3/rccl-ready-slim
  echo $dir
}"""

INSTALL_MI355X_NODE = r"""#!/bin/bash
# MI355X worker bootstrap: ROCm preflight, topology labels (N1), burn-in,
# RCCL environment + node-level RCCL gate (N2), then the Rancher agent with
# the GPU labels.  Node tools: the CLI's prebuilt gfx950 binaries when their
# stamp matches the shipped sources (node/tools.py), else built here with hipcc.
set -euo pipefail
T=/opt/triton-kubernetes/bin
S=/opt/triton-kubernetes/src
sudo mkdir -p $T /etc/triton-kubernetes /etc/rccl
lsmod | grep '^amdgpu' >/dev/null || { echo 'amdgpu kernel module not loaded' >&2; exit 1; }
test -c /dev/kfd || { echo '/dev/kfd missing' >&2; exit 1; }
n=$(ls /dev/dri/renderD* 2>/dev/null | wc -l || true)  # pipefail: ls fails when there are none
[ "$n" -ge ${gpu_count * gpu_partitions} ] || { echo "expected ${gpu_count * gpu_partitions} GPUs (${gpu_count} x ${gpu_compute_partition}), found $n render nodes" >&2; exit 1; }
# partition modes: verified, never changed here (repartitioning resets the GPUs)
for f in /sys/class/drm/renderD*/device/current_compute_partition /sys/class/drm/renderD*/device/current_memory_partition; do
  [ -r "$f" ] || continue
  m=$(tr 'A-Z' 'a-z' < "$f")
  case $f in
    *compute*) [ "$m" = '${gpu_compute_partition}' ] || { echo "compute partition is $m, the cluster expects ${gpu_compute_partition}" >&2; exit 1; } ;;
    *) [ "$m" = '${gpu_memory_partition}' ] || { echo "memory partition is $m, the cluster expects ${gpu_memory_partition}" >&2; exit 1; } ;;
  esac
done
sudo usermod -aG video,render "$(id -un)" || true
ROCM=$${ROCM_PATH:-/opt/rocm}
""" + NODE_TOOLS_FN + r"""
tk_node_tools $T $S """ + PREBUILT_DIR + r""" $ROCM
RCCL_READY=$T/rccl-ready
sudo rm -f $T/""" + RCCL_SLIM_ENV + r""" $T/rccl-ready-slim
%{ if rccl_slim == "on" ~}
""" + RCCL_SLIM_FN + "\n" + RCCL_SLIM_ENABLE_FN + r"""
if sudo bash -c "$(declare -f tk_rccl_slim tk_rccl_slim_enable); tk_rccl_slim_enable """ + RCCL_SLIM_ROOT + r""" $ROCM $T" >/dev/null; then
  RCCL_READY=$T/rccl-ready-slim
else
  echo 'rccl slim: not enabled, the node tools load the installed RCCL' >&2
fi
%{ endif ~}
$T/amdgpu-topo-labeller | sudo tee /etc/triton-kubernetes/gpu-topology.json >/dev/null
$T/amdgpu-topo-labeller --labels | sudo tee /etc/triton-kubernetes/gpu-labels >/dev/null
sudo rm -f /etc/triton-kubernetes/gpu-burnin-labels /etc/triton-kubernetes/gpu-taints
%{ if gpu_host_tuning != "off" ~}
""" + _host_tuning_check(
    "warn", "/etc/triton-kubernetes/gpu-burnin-labels", fail='${gpu_host_tuning == "enforce" ? "exit 1" : "true"}') + r"""
%{ endif ~}
# the xGMI link check first, on idle GPUs: a full burn-in's release of ~300 GB per GPU is
# cleared by the driver for seconds after it, beside whatever runs next
%{ if gpu_count > 1 && gpu_compute_partition == "spx" ~}
$T/gpu-burnin --p2p --min-link-frac ${gpu_link_min_frac} --min-link-gbps ${gpu_link_min_gbps} --labels /tmp/tk-link-labels | sudo tee /etc/triton-kubernetes/gpu-links.json
cat /tmp/tk-link-labels | sudo tee -a /etc/triton-kubernetes/gpu-burnin-labels >/dev/null
%{ endif ~}
%{ if gpu_health != "off" ~}
# GPU health (RAS): exit 3 = an unhealthy GPU; fail the node or join it tainted
health_rc=0
$T/amdgpu-topo-labeller --health --max-uncorrectable ${gpu_max_uncorrectable_ecc} --max-bad-pages ${gpu_max_retired_pages} > /tmp/tk-gpu-health.json || health_rc=$?
sudo install -m 0644 /tmp/tk-gpu-health.json /etc/triton-kubernetes/gpu-health.json
{ $T/amdgpu-topo-labeller --health --labels --max-uncorrectable ${gpu_max_uncorrectable_ecc} --max-bad-pages ${gpu_max_retired_pages} || true; } | sudo tee -a /etc/triton-kubernetes/gpu-burnin-labels >/dev/null
case $health_rc in
  0) ;;
%{ if gpu_health == "taint" ~}
  3) echo 'amd.com/gpu-health=unhealthy:NoSchedule' | sudo tee /etc/triton-kubernetes/gpu-taints >/dev/null ;;
%{ else ~}
  3) echo 'unhealthy GPUs (gpu_health = fail):' >&2; cat /tmp/tk-gpu-health.json >&2; exit 1 ;;
%{ endif ~}
  *) echo "GPU health check failed (exit $health_rc)" >&2; exit 1 ;;
esac
%{ endif ~}
%{ if gpu_metrics_textfile != "" ~}
# GPU health as Prometheus text for node_exporter's textfile collector, every minute
""" + _metrics_textfile("/opt/triton-kubernetes/bin", "${gpu_metrics_textfile}", "${gpu_max_uncorrectable_ecc}",
                        "${gpu_max_retired_pages}") + r"""
%{ endif ~}
{ $T/amdgpu-topo-labeller --rccl-env || true; cat <<'TK_RCCL_EOF'
${rccl_env_file}
TK_RCCL_EOF
} | sudo tee /etc/rccl/rccl.env >/dev/null
%{ if gpu_count * gpu_partitions > 1 ~}
set -a; . /etc/rccl/rccl.env; set +a
$RCCL_READY --ngpus ${gpu_count * gpu_partitions} --min-busbw ${rccl_min_busbw}
%{ endif ~}
# the burn-in last of the GPU steps: the driver clears the ~300 GB per GPU a full burn-in
# releases for seconds afterwards, and an RCCL communicator started meanwhile waits behind it
%{ if gpu_burnin != "off" ~}
$T/gpu-burnin --all --level '${gpu_burnin}' --compute-partition ${gpu_compute_partition} --memory-partition ${gpu_memory_partition} --labels /tmp/tk-burnin-labels | sudo tee /etc/triton-kubernetes/gpu-burnin.json
sudo tee -a /etc/triton-kubernetes/gpu-burnin-labels < /tmp/tk-burnin-labels >/dev/null
%{ endif ~}
labels=$(cat /etc/triton-kubernetes/gpu-labels $([ -r /etc/triton-kubernetes/gpu-burnin-labels ] && echo /etc/triton-kubernetes/gpu-burnin-labels) | sed 's/^/--label /' | tr '\n' ' ')
if [ -r /etc/triton-kubernetes/gpu-taints ]; then labels="$labels $(sed 's/^/--taints /' /etc/triton-kubernetes/gpu-taints | tr '\n' ' ')"; fi
%{ if k8s_distribution == "rke1" ~}
""" + DOCKER_INSTALL + r"""
%{ endif ~}
sudo hostnamectl set-hostname '${hostname}'
%{ if rancher_registry_username != "" && k8s_distribution == "rke1" ~}
echo '${rancher_registry_password}' | sudo docker login -u '${rancher_registry_username}' --password-stdin '${rancher_registry}'
%{ endif ~}
""" + JOIN_CLUSTER.replace("${extra_agent_args}", " $labels") + "\n"

READ_REMOTE_LABELS = r"""#!/bin/bash
# data "external" program: the GPU labels a MI355X node computed, as one JSON string.
set -euo pipefail
eval "$(python3 -c 'import json,shlex,sys; q=json.load(sys.stdin); print(" ".join(f"{k}={shlex.quote(str(v))}" for k,v in q.items()))')"
""" + SSH_PINNED + r"""if ! raw=$(ssh "${opts[@]}" "$ssh_user@$host" 'cat /etc/triton-kubernetes/gpu-labels; cat /etc/triton-kubernetes/gpu-burnin-labels 2>/dev/null || true' 2>"$err"); then
  # outside an apply (operation destroy | read) a node that is gone has no labels to report
  if [ "${operation:-apply}" != apply ]; then echo '{"labels": "{}", "known_hosts": ""}'; exit 0; fi
  refused "read the GPU labels"
fi
printf '%s\n' "$raw" | KH="$(pinned_for)" python3 -c '
import json, os, sys
labels = dict(l.strip().split("=", 1) for l in sys.stdin if "=" in l)
print(json.dumps({"labels": json.dumps(labels, sort_keys=True), "known_hosts": os.environ["KH"]}))'
"""

APPLY_ADDONS = r"""#!/bin/bash
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
"""
