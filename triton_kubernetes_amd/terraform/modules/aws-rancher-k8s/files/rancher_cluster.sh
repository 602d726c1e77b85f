#!/bin/bash
# S4: data "external" program run on the operator machine.  Idempotent
# find-or-create of the RKE cluster, its registration token and CA checksum.
set -euo pipefail
eval "$(python3 -c 'import json,shlex,sys; q=json.load(sys.stdin); print(" ".join(f"{k}={shlex.quote(str(v))}" for k,v in q.items()))')"
api() { curl -ksf -u "$rancher_access_key:$rancher_secret_key" -H 'Accept: application/json' -H 'Content-Type: application/json' "$@"; }
py() { python3 -c "$1"; }
search=$(api "$rancher_api_url/v3/clusters?name=$name")
cluster_id=$(printf '%s' "$search" | py 'import json,sys; d=json.load(sys.stdin)["data"]; print(d[0]["id"] if d else "")')
existed=true
if [ -z "$cluster_id" ]; then
  existed=false
  body=$(NAME="$name" VER="$k8s_version" NET="$k8s_network_provider" REG="${k8s_registry:-}" \
         REGU="${k8s_registry_username:-}" REGP="${k8s_registry_password:-}" py '
import json, os
rke = {"ignoreDockerVersion": False, "sshAgentAuth": False, "type": "rancherKubernetesEngineConfig",
       "kubernetesVersion": os.environ["VER"], "authentication": {"type": "authnConfig", "strategy": "x509"},
       "network": {"type": "networkConfig", "plugin": os.environ["NET"]},
       "services": {"type": "rkeConfigServices", "kubeApi": {"podSecurityPolicy": False, "type": "kubeAPIService"}}}
if os.environ["REG"]:
    rke["privateRegistries"] = [{"url": os.environ["REG"], "user": os.environ["REGU"], "password": os.environ["REGP"]}]
print(json.dumps({"type": "cluster", "name": os.environ["NAME"], "rancherKubernetesEngineConfig": rke}))')
  cluster_id=$(api -X POST -d "$body" "$rancher_api_url/v3/cluster" | py 'import json,sys; print(json.load(sys.stdin).get("id",""))')
fi
[ -n "$cluster_id" ] || { echo "Unable to create cluster!" >&2; exit 1; }
token=""
if [ "$existed" = true ]; then
  token=$(api "$rancher_api_url/v3/clusters/$cluster_id/clusterregistrationtokens" | py 'import json,sys; d=json.load(sys.stdin)["data"]; print(d[0]["token"] if d else "")')
fi
if [ -z "$token" ]; then
  token=$(api -X POST -d "{\"type\":\"clusterRegistrationToken\",\"clusterId\":\"$cluster_id\"}" \
          "$rancher_api_url/v3/clusterregistrationtoken" | py 'import json,sys; print(json.load(sys.stdin).get("token",""))')
fi
[ -n "$token" ] || { echo "Unable to create cluster registration token!" >&2; exit 1; }
checksum=$(api "$rancher_api_url/v3/settings/cacerts" | py 'import json,sys,hashlib; v=json.load(sys.stdin)["value"]; print(hashlib.sha256((v+"\n").encode()).hexdigest())')
CID="$cluster_id" TOK="$token" SUM="$checksum" py 'import json,os; print(json.dumps({"cluster_id": os.environ["CID"], "registration_token": os.environ["TOK"], "ca_checksum": os.environ["SUM"]}))'
