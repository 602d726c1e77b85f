#!/bin/bash
# data "external" program: read the manager's ~/rancher_api_key over SSH.
# Replaces the reference's matti/outputs/shell registry module.
# Outside an apply (query key operation = destroy | read, the executor's tk_operation)
# a manager that cannot be reached yields empty keys instead of an error: destroying
# what is left of a manager whose host is gone must not depend on that host.
set -euo pipefail
eval "$(python3 -c 'import json,shlex,sys; q=json.load(sys.stdin); print(" ".join(f"{k}={shlex.quote(str(v))}" for k,v in q.items()))')"
opts=(-o BatchMode=yes -o StrictHostKeyChecking=no -o UserKnownHostsFile=/dev/null -o LogLevel=ERROR -i "${key_path/#\~/$HOME}")
if [ -n "${bastion_host:-}" ]; then opts+=(-J "$ssh_user@$bastion_host"); fi
if ! tok=$(ssh "${opts[@]}" "$ssh_user@$host" 'cat ~/rancher_api_key'); then
  if [ "${operation:-apply}" != apply ]; then echo '{"access_key": "", "secret_key": ""}'; exit 0; fi
  echo "could not read the Rancher API key from $host" >&2
  exit 1
fi
printf '%s' "$tok" | python3 -c '
import json, sys
t = json.load(sys.stdin)
print(json.dumps({"access_key": t["name"], "secret_key": t["token"].split(":", 1)[1]}))'
