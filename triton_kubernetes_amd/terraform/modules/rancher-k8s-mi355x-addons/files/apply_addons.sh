#!/bin/bash
# MI355X cluster add-ons: wait for the cluster, then create the manifests in
# $MANIFEST_DIR through Rancher's Kubernetes proxy (PUT on 409).
set -euo pipefail
# TLS verified against the manager's pinned CA (RANCHER_CA; empty: the system trust store)
tls=()
if [ -n "${RANCHER_CA:-}" ]; then
  cafile=$(mktemp); trap 'rm -f "$cafile"' EXIT
  printf '%s\n' "$RANCHER_CA" > "$cafile"
  tls=(--cacert "$cafile")
fi
api() { curl -sf "${tls[@]}" -u "$RANCHER_ACCESS_KEY:$RANCHER_SECRET_KEY" -H 'Content-Type: application/json' "$@"; }
for i in $(seq 1 3600); do
  state=$(api "$RANCHER_URL/v3/clusters/$CLUSTER_ID" | python3 -c 'import json,sys; print(json.load(sys.stdin).get("state",""))' || true)
  [ "$state" = active ] && break
  sleep 1
done
[ "$state" = active ] || { echo "cluster $CLUSTER_ID not active" >&2; exit 1; }
for f in "$MANIFEST_DIR"/*.json; do
  path=$(python3 -c 'import json,sys; print(json.load(open(sys.argv[1]))["path"])' "$f")
  obj=$(python3 -c 'import json,sys; print(json.dumps(json.load(open(sys.argv[1]))["object"]))' "$f")
  name=$(python3 -c 'import json,sys; print(json.load(open(sys.argv[1]))["object"]["metadata"]["name"])' "$f")
  code=$(curl -s "${tls[@]}" -o /dev/null -w '%{http_code}' -u "$RANCHER_ACCESS_KEY:$RANCHER_SECRET_KEY" \
         -H 'Content-Type: application/json' -X POST -d "$obj" "$RANCHER_URL/k8s/clusters/$CLUSTER_ID$path")
  if [ "$code" = 409 ]; then api -X PUT -d "$obj" "$RANCHER_URL/k8s/clusters/$CLUSTER_ID$path/$name" >/dev/null
  elif [ "$code" -ge 300 ]; then echo "applying $f: HTTP $code" >&2; exit 1; fi
done
