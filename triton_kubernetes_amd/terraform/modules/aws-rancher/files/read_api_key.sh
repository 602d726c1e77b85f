#!/bin/bash
# data "external" program: read the manager's ~/rancher_api_key over SSH.
# Replaces the reference's matti/outputs/shell registry module.
set -euo pipefail
eval "$(python3 -c 'import json,shlex,sys; q=json.load(sys.stdin); print(" ".join(f"{k}={shlex.quote(str(v))}" for k,v in q.items()))')"
opts=(-o BatchMode=yes -o StrictHostKeyChecking=no -o UserKnownHostsFile=/dev/null -o LogLevel=ERROR -i "${key_path/#\~/$HOME}")
if [ -n "${bastion_host:-}" ]; then opts+=(-J "$ssh_user@$bastion_host"); fi
tok=$(ssh "${opts[@]}" "$ssh_user@$host" 'cat ~/rancher_api_key')
printf '%s' "$tok" | python3 -c '
import json, sys
t = json.load(sys.stdin)
print(json.dumps({"access_key": t["name"], "secret_key": t["token"].split(":", 1)[1]}))'
