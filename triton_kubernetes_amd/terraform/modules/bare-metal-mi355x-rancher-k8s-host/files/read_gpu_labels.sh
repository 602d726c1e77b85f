#!/bin/bash
# data "external" program: the GPU labels a MI355X node computed, as one JSON string.
set -euo pipefail
eval "$(python3 -c 'import json,shlex,sys; q=json.load(sys.stdin); print(" ".join(f"{k}={shlex.quote(str(v))}" for k,v in q.items()))')"
opts=(-o BatchMode=yes -o StrictHostKeyChecking=no -o UserKnownHostsFile=/dev/null -o LogLevel=ERROR -i "${key_path/#\~/$HOME}")
if [ -n "${bastion_host:-}" ]; then opts+=(-J "$ssh_user@$bastion_host"); fi
if ! raw=$(ssh "${opts[@]}" "$ssh_user@$host" 'cat /etc/triton-kubernetes/gpu-labels; cat /etc/triton-kubernetes/gpu-burnin-labels 2>/dev/null || true'); then
  # outside an apply (operation destroy | read) a node that is gone has no labels to report
  if [ "${operation:-apply}" != apply ]; then echo '{"labels": "{}"}'; exit 0; fi
  echo "could not read the GPU labels of $host" >&2
  exit 1
fi
printf '%s\n' "$raw" | python3 -c '
import json, sys
labels = dict(l.strip().split("=", 1) for l in sys.stdin if "=" in l)
print(json.dumps({"labels": json.dumps(labels, sort_keys=True)}))'
