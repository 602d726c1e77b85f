#!/bin/bash
# data "external" program: the GPU labels a MI355X node computed, as one JSON string.
set -euo pipefail
eval "$(python3 -c 'import json,shlex,sys; q=json.load(sys.stdin); print(" ".join(f"{k}={shlex.quote(str(v))}" for k,v in q.items()))')"
# SSH with the cluster manager's pinned host keys (query key known_hosts, the executor's
# tk_known_hosts; parallel/hostkeys.py): a known host's key must match, an unknown one is
# pinned on this first contact and reported back (result key known_hosts).
kh=$(mktemp); err=$(mktemp); trap 'rm -f "$kh" "$err"' EXIT
printf '%s\n' "${known_hosts:-}" > "$kh"
# host key algorithms in Go's order (Terraform's client): the key pinned here is the type
# Terraform's provisioner connections negotiate; UpdateHostKeys pins the host's other keys
ko=(-o "UserKnownHostsFile=$kh" -o StrictHostKeyChecking=accept-new -o HashKnownHosts=no -o GlobalKnownHostsFile=/dev/null
    -o "HostKeyAlgorithms=ecdsa-sha2-nistp256,ecdsa-sha2-nistp384,ecdsa-sha2-nistp521,rsa-sha2-512,rsa-sha2-256,ssh-ed25519" -o UpdateHostKeys=yes)
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
if ! raw=$(ssh "${opts[@]}" "$ssh_user@$host" 'cat /etc/triton-kubernetes/gpu-labels; cat /etc/triton-kubernetes/gpu-burnin-labels 2>/dev/null || true' 2>"$err"); then
  # outside an apply (operation destroy | read) a node that is gone has no labels to report
  if [ "${operation:-apply}" != apply ]; then echo '{"labels": "{}", "known_hosts": ""}'; exit 0; fi
  refused "read the GPU labels"
fi
printf '%s\n' "$raw" | KH="$(pinned_for)" python3 -c '
import json, os, sys
labels = dict(l.strip().split("=", 1) for l in sys.stdin if "=" in l)
print(json.dumps({"labels": json.dumps(labels, sort_keys=True), "known_hosts": os.environ["KH"]}))'
