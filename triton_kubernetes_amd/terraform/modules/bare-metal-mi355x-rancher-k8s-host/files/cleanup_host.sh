#!/bin/bash
# triton-kubernetes host cleanup (node/cleanup.py): uninstall the cluster's agent and
# Kubernetes distribution, keep the node tools and the container runtime
set -uo pipefail
R=${TK_HOST_ROOT:-}
rc=0
_tk_mark() { echo "::tk-cleanup $1 $2"; }
if [ "${TK_NODE_CLEANUP:-true}" = false ]; then
  # the host module's node_cleanup = false (Terraform's destroy-time provisioner): keep the host
  echo "::tk-cleanup node_cleanup skipped"
  echo "::tk-cleanup-done 0"
  exit 0
fi
for f in /usr/local/bin/rancher-system-agent-uninstall.sh /opt/rancher-system-agent/bin/rancher-system-agent-uninstall.sh /usr/local/bin/rke2-killall.sh /usr/local/bin/rke2-uninstall.sh /opt/rke2/bin/rke2-killall.sh /opt/rke2/bin/rke2-uninstall.sh; do
  [ -x "$R$f" ] || continue
  if sudo "$R$f" >/dev/null 2>&1; then _tk_mark "$f" ok; else _tk_mark "$f" failed; rc=1; fi
done
if command -v docker >/dev/null 2>&1; then
  # RKE1 (node/cleanup.py RKE1_LABELS, RKE1_REPOS): labelled containers, and containers of the
  # agent's or RKE's image repositories with any registry prefix, tag or digest
  _tk_repo() { local i="${1%%@*}" l; l="${i##*/}"; case "$l" in *:*) i="${i%:*}";; esac; echo "$i"; }
  repos="rancher/rancher-agent rancher/rke-tools rancher/hyperkube"
  rec_img=$(sed -n 's/.*"agent_image": *"\([^"]*\)".*/\1/p' "$R/etc/triton-kubernetes/joined.json" 2>/dev/null || true)
  for img in "${TK_AGENT_IMAGE:-}" "$rec_img"; do [ -n "$img" ] && repos="$repos $(_tk_repo "$img")"; done
  ids=$( { for lab in io.rancher.rke.container.name io.kubernetes.pod.namespace; do sudo docker ps -aq --filter "label=$lab" 2>/dev/null || true; done
           sudo docker ps -a --format '{{.ID}} {{.Image}}' 2>/dev/null | awk -v repos="$repos" '
             BEGIN { n = split(repos, want, " ") }
             { img = $2; sub(/@.*/, "", img); k = split(img, p, "/"); if (p[k] ~ /:/) sub(/:[^:\/]*$/, "", img)
               for (j = 1; j <= n; j++) { w = want[j]
                 if (img == w || (length(img) > length(w) && substr(img, length(img) - length(w)) == "/" w)) { print $1; break } } }' || true
         } | sort -u)
  if [ -n "$ids" ]; then
    if sudo docker rm -f $ids >/dev/null 2>&1; then _tk_mark rke1-containers ok; else _tk_mark rke1-containers failed; rc=1; fi
  fi
fi
# the kubelet's mounts (RKE1; rke2-killall.sh unmounts its own), deepest first
mounts=$(awk -v p="$R/var/lib/kubelet" 'index($2, p) == 1 {print $2}' /proc/mounts 2>/dev/null | sort -r)
for m in $mounts; do sudo umount "$m" >/dev/null 2>&1 || sudo umount -l "$m" >/dev/null 2>&1 || true; done
for d in /etc/rancher /var/lib/rancher /etc/kubernetes /var/lib/etcd /var/lib/kubelet /etc/cni /opt/cni /var/lib/cni /var/run/calico /run/flannel /etc/triton-kubernetes/joined.json; do
  [ -e "$R$d" ] || continue
  if sudo rm -rf "$R$d"; then _tk_mark "$d" removed; else _tk_mark "$d" failed; rc=1; fi
done
echo "::tk-cleanup-done $rc"
exit $rc
