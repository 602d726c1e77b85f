#!/bin/bash
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
if ! tok=$(ssh "${opts[@]}" "$ssh_user@$host" 'cat ~/rancher_api_key' 2>"$err"); then
  if [ "${operation:-apply}" != apply ]; then echo '{"access_key": "", "secret_key": "", "known_hosts": "", "ca_certs": ""}'; exit 0; fi
  refused "read the Rancher API key"
fi
# the bundle as saved on the host, or -- an older install that never saved it -- read there
# now from the server's own loopback (rancher/trust.py HOST_CA_READ).  Empty only when the
# server's cacerts setting is (a publicly trusted certificate); a failed read fails here
# rather than pinning an empty bundle
if ! ca=$(ssh "${opts[@]}" "$ssh_user@$host" 'bash -s' 2>"$err" <<'TK_CA_EOF'
f=~/rancher_cacerts.pem
if [ ! -e "$f" ]; then
  umask 077
  if ! curl -ksf https://127.0.0.1/cacerts > "$f.tmp"; then
    rm -f "$f.tmp"
    echo "no $f on this host and https://127.0.0.1/cacerts cannot be read: is the Rancher server running? (or give rancher_ca_file)" >&2
    exit 3
  fi
  mv "$f.tmp" "$f"
fi
cat "$f"
TK_CA_EOF
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
