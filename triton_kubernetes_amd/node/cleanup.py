"""Host teardown and the join record: a reused bare-metal host can join another cluster.

Bare-metal MI355X hosts are never re-imaged, so ``destroy cluster``
followed by ``create cluster`` on the same host is the normal path.  The reference never
uninstalled anything (Q7: ``destroy/node.go:167-168`` only drops the module;
``terraform/modules/bare-metal-rancher-k8s-host/main.tf:24-42`` has no destroy-time
provisioner), so the second join met a live agent and kubelet of the first cluster.

Two halves, one definition each, rendered for every delivery path:

* **teardown** (:func:`cleanup_script` for SSH and Terraform's destroy-time provisioner,
  :func:`cleanup_host` for the node agent's fixed-argv ``POST /v1/cleanup``), in order:

  1. ``rancher-system-agent-uninstall.sh`` (RKE2 custom clusters: stops the agent that
     would otherwise re-apply the old cluster's plan);
  2. ``rke2-killall.sh`` then ``rke2-uninstall.sh`` (RKE2 itself: containers, mounts,
     interfaces, binaries, ``/var/lib/rancher/rke2``);
  3. the RKE1 containers (``rancher/rancher-agent`` and RKE-managed ones) when docker is
     there, and the kubelet's mounts;
  4. what is left of the Kubernetes / Rancher / CNI state directories (:data:`CLEAN_DIRS`)
     and this framework's join record.

  Kept: the node agent itself, the node tools (``/opt/triton-kubernetes/bin``) and the
  container runtime -- the next join needs them, and they belong to no cluster.

* **join record** (:data:`JOIN_RECORD`): written after a successful join, checked before
  the next one.  A host whose record names another cluster is refused with a message that
  says how to clean it, instead of joining with the old cluster's RKE2 state in place
  (which fails far later, as a node that never turns Ready).  A host without a record
  (joined by an older version, or never) is not refused.

Cleanup is the default on destroy for bare-metal hosts (``node_cleanup``, default true:
the host outlives the cluster); cloud host modules delete their instance instead.  A
cleanup that fails (host unreachable, an uninstaller erroring) does not block the destroy
-- Terraform's provisioner runs ``on_failure = continue`` -- it is reported, and the join
record then stops a later join on that host with the reason.

``TK_HOST_ROOT`` (default empty, i.e. ``/``) prefixes every path the scripts touch: a host
filesystem mounted elsewhere (an image being prepared in a chroot) and the tests' host
models use it.
"""

import hashlib
import json
import os
import shlex
import shutil
import subprocess
import time
from typing import Any, Callable, Dict, List, Optional

JOIN_RECORD = "/etc/triton-kubernetes/joined.json"

# in the order they run; absent ones are skipped (a host of the other distribution)
UNINSTALLERS = (
    "/usr/local/bin/rancher-system-agent-uninstall.sh",
    "/opt/rancher-system-agent/bin/rancher-system-agent-uninstall.sh",
    "/usr/local/bin/rke2-killall.sh",
    "/usr/local/bin/rke2-uninstall.sh",
    "/opt/rke2/bin/rke2-killall.sh",
    "/opt/rke2/bin/rke2-uninstall.sh",
)

# left-overs of either distribution, removed after the uninstallers (which remove most)
CLEAN_DIRS = (
    "/etc/rancher", "/var/lib/rancher", "/etc/kubernetes", "/var/lib/etcd", "/var/lib/kubelet",
    "/etc/cni", "/opt/cni", "/var/lib/cni", "/var/run/calico", "/run/flannel",
)

# RKE1: what the teardown removes, decided from what ``docker ps -a`` shows.  Not an
# untagged ``--filter ancestor=rancher/rancher-agent``: Docker reads that as
# ``rancher/rancher-agent:latest``, which matches no agent running a tagged image (the
# pinned ``rancher/rancher-agent:v2.10.3``, or one behind a registry), so the agent -- run
# with ``--restart=unless-stopped`` -- survived and kept the node in its old cluster.
# * containers carrying either label: RKE's own (kubelet, etcd, kube-proxy, service-sidekick)
#   and every container the kubelet started for a pod (``k8s_*`` and their ``k8s_POD_*``
#   sandboxes: flannel, cattle-node-agent, the device plugin);
# * containers whose image repository -- any registry prefix, any tag or digest -- is the
#   agent's (``rancher/rancher-agent``, plus the exact image the join record names or
#   Terraform passes as ``TK_AGENT_IMAGE``) or one of RKE's (its helper containers such as
#   the port listeners and log linkers carry no label).
RKE1_LABELS = ("io.rancher.rke.container.name", "io.kubernetes.pod.namespace")
RKE1_REPOS = ("rancher/rancher-agent", "rancher/rke-tools", "rancher/hyperkube")


def image_repository(ref: str) -> str:
    """``[registry/]path`` of an image reference, without its tag or digest
    (``reg:5000/rancher/rancher-agent:v2.10.3`` -> ``reg:5000/rancher/rancher-agent``)."""
    ref = ref.split("@", 1)[0]
    head, _, last = ref.rpartition("/")
    last = last.split(":", 1)[0]
    return f"{head}/{last}" if head else last


def rke1_repos(record: Optional[Dict[str, Any]] = None, agent_image: str = "") -> List[str]:
    """The image repositories whose containers an RKE1 teardown removes."""
    repos = list(RKE1_REPOS)
    for img in ((record or {}).get("agent_image", ""), agent_image):
        if img and image_repository(img) not in repos:
            repos.append(image_repository(img))
    return repos


def repo_matches(image: str, repos: List[str]) -> bool:
    """``image`` (as ``docker ps`` shows it) is of one of ``repos``, with any registry prefix."""
    r = image_repository(image)
    return any(r == w or r.endswith("/" + w) for w in repos)


def cluster_identity(server: str, token: str) -> str:
    """Which cluster a join is for: the Rancher server and the cluster's registration
    token (hashed: the record holds no secret)."""
    return hashlib.sha256(f"{server.rstrip('/')}\n{token}".encode()).hexdigest()[:24]


def join_record(server: str, token: str, distribution: str, hostname: str,
                agent_image: str = "") -> Dict[str, Any]:
    """What a successful join records; ``agent_image``: the RKE1 agent image it ran (the
    teardown removes that repository's containers whatever its registry and tag)."""
    rec = {"cluster": cluster_identity(server, token), "server": server.rstrip("/"),
           "distribution": distribution, "hostname": hostname}
    if agent_image:
        rec["agent_image"] = agent_image
    return rec


def refusal(record: Optional[Dict[str, Any]], server: str, token: str) -> Optional[str]:
    """Why a join for ``(server, token)`` must not run on a host holding ``record``."""
    if not record or not record.get("cluster"):
        return None
    if record["cluster"] == cluster_identity(server, token):
        return None  # a re-join of the same cluster (re-apply, retry): idempotent
    return (f"this host is still a node of another cluster ({record.get('distribution', '?')} "
            f"'{record.get('hostname', '?')}' of {record.get('server', '?')}): clean it up first "
            f"(destroy that node or cluster with node_cleanup on, the default for bare metal; "
            f"or uninstall its rancher-system-agent / RKE2 and remove {JOIN_RECORD})")


# --- shell renderings ------------------------------------------------------------------------


def join_guard_shell(server: str, token: str) -> str:
    """Shell lines for the start of a join step: refuse a host whose join record names
    another cluster (:func:`refusal`)."""
    ident = cluster_identity(server, token)
    return (
        f"_tk_rec=\"${{TK_HOST_ROOT:-}}{JOIN_RECORD}\"\n"
        "if [ -r \"$_tk_rec\" ]; then\n"
        "  _tk_prev=$(sed -n 's/.*\"cluster\": *\"\\([0-9a-f]*\\)\".*/\\1/p' \"$_tk_rec\")\n"
        f"  if [ -n \"$_tk_prev\" ] && [ \"$_tk_prev\" != {ident} ]; then\n"
        "    echo \"this host is still a node of another cluster ($(cat \"$_tk_rec\")): clean it up first "
        f"(destroy that node or cluster with node_cleanup on, the default for bare metal; or uninstall its "
        f"rancher-system-agent / RKE2 and remove {JOIN_RECORD})\" >&2\n"
        "    exit 1\n"
        "  fi\n"
        "fi\n")


def join_record_shell(server: str, token: str, distribution: str, hostname: str, agent_image: str = "") -> str:
    """Shell lines for the end of a successful join step: write the join record."""
    doc = json.dumps(join_record(server, token, distribution, hostname, agent_image), sort_keys=True)
    # quoted for the shell whatever the fields hold (a quote in a server URL stays data)
    return (f"sudo mkdir -p \"${{TK_HOST_ROOT:-}}{os.path.dirname(JOIN_RECORD)}\"\n"
            f"printf '%s\\n' {shlex.quote(doc)} | sudo tee \"${{TK_HOST_ROOT:-}}{JOIN_RECORD}\" >/dev/null\n")


def cleanup_script() -> str:
    """The host teardown as a script (SSH ``bash -s``, Terraform ``remote-exec``).  Prints
    ``::tk-cleanup <what> <status>`` per action; exits non-zero if an uninstaller failed."""
    uninstallers = " ".join(UNINSTALLERS)
    dirs = " ".join(CLEAN_DIRS + (JOIN_RECORD,))
    return f"""#!/bin/bash
# triton-kubernetes host cleanup (node/cleanup.py): uninstall the cluster's agent and
# Kubernetes distribution, keep the node tools and the container runtime
set -uo pipefail
R=${{TK_HOST_ROOT:-}}
rc=0
_tk_mark() {{ echo "::tk-cleanup $1 $2"; }}
if [ "${{TK_NODE_CLEANUP:-true}}" = false ]; then
  # the host module's node_cleanup = false (Terraform's destroy-time provisioner): keep the host
  echo "::tk-cleanup node_cleanup skipped"
  echo "::tk-cleanup-done 0"
  exit 0
fi
for f in {uninstallers}; do
  [ -x "$R$f" ] || continue
  if sudo "$R$f" >/dev/null 2>&1; then _tk_mark "$f" ok; else _tk_mark "$f" failed; rc=1; fi
done
if command -v docker >/dev/null 2>&1; then
  # RKE1 (node/cleanup.py RKE1_LABELS, RKE1_REPOS): labelled containers, and containers of the
  # agent's or RKE's image repositories with any registry prefix, tag or digest
  _tk_repo() {{ local i="${{1%%@*}}" l; l="${{i##*/}}"; case "$l" in *:*) i="${{i%:*}}";; esac; echo "$i"; }}
  repos="{" ".join(RKE1_REPOS)}"
  rec_img=$(sed -n 's/.*"agent_image": *"\\([^"]*\\)".*/\\1/p' "$R{JOIN_RECORD}" 2>/dev/null || true)
  for img in "${{TK_AGENT_IMAGE:-}}" "$rec_img"; do [ -n "$img" ] && repos="$repos $(_tk_repo "$img")"; done
  ids=$( {{ for lab in {" ".join(RKE1_LABELS)}; do sudo docker ps -aq --filter "label=$lab" 2>/dev/null || true; done
           sudo docker ps -a --format '{{{{.ID}}}} {{{{.Image}}}}' 2>/dev/null | awk -v repos="$repos" '
             BEGIN {{ n = split(repos, want, " ") }}
             {{ img = $2; sub(/@.*/, "", img); k = split(img, p, "/"); if (p[k] ~ /:/) sub(/:[^:\\/]*$/, "", img)
               for (j = 1; j <= n; j++) {{ w = want[j]
                 if (img == w || (length(img) > length(w) && substr(img, length(img) - length(w)) == "/" w)) {{ print $1; break }} }} }}' || true
         }} | sort -u)
  if [ -n "$ids" ]; then
    if sudo docker rm -f $ids >/dev/null 2>&1; then _tk_mark rke1-containers ok; else _tk_mark rke1-containers failed; rc=1; fi
  fi
fi
# the kubelet's mounts (RKE1; rke2-killall.sh unmounts its own), deepest first
mounts=$(awk -v p="$R/var/lib/kubelet" 'index($2, p) == 1 {{print $2}}' /proc/mounts 2>/dev/null | sort -r)
for m in $mounts; do sudo umount "$m" >/dev/null 2>&1 || sudo umount -l "$m" >/dev/null 2>&1 || true; done
for d in {dirs}; do
  [ -e "$R$d" ] || continue
  if sudo rm -rf "$R$d"; then _tk_mark "$d" removed; else _tk_mark "$d" failed; rc=1; fi
done
echo "::tk-cleanup-done $rc"
exit $rc
"""


def parse_cleanup_markers(output: str) -> Dict[str, Any]:
    """``::tk-cleanup`` markers of a :func:`cleanup_script` run -> a report."""
    actions: List[Dict[str, str]] = []
    done = None
    for line in output.splitlines():
        parts = line.split()
        if len(parts) >= 3 and parts[0] == "::tk-cleanup":
            actions.append({"what": parts[1], "status": parts[2]})
        elif len(parts) >= 2 and parts[0] == "::tk-cleanup-done":
            done = parts[1] == "0"
    ok = done if done is not None else all(a["status"] != "failed" for a in actions)
    return {"ok": bool(ok), "actions": actions, "complete": done is not None,
            "rke1": {"labels": list(RKE1_LABELS), "repositories": list(RKE1_REPOS)}}


# --- the node agent's teardown (fixed argv lists, no shell text) -------------------------------


def cleanup_host(path: Callable[[str], str], run_argv: Callable[[List[str]], str],
                 docker: Optional[str] = None, env: Optional[Dict[str, str]] = None) -> Dict[str, Any]:
    """:func:`cleanup_script` for the node agent: the same actions, each a fixed argv.

    ``path`` maps a host path to where it is (``NodeAgent.path``: ``/`` in exec mode, the
    agent's root in sim mode); ``run_argv`` runs an argv and raises on failure; ``docker``
    is the docker binary (None: no docker); ``env`` is the uninstallers' environment."""
    t0 = time.perf_counter()
    actions: List[Dict[str, str]] = []
    ok = True
    for f in UNINSTALLERS:
        p = path(f)
        if not (os.path.isfile(p) and os.access(p, os.X_OK)):
            continue
        try:
            if env is None:
                run_argv([p])
            else:
                proc = subprocess.run([p], env=env, capture_output=True, text=True, timeout=600, check=False)
                if proc.returncode != 0:
                    raise RuntimeError(f"{f} exited {proc.returncode}: {(proc.stderr or proc.stdout)[-500:]}")
            actions.append({"what": f, "status": "ok"})
        except Exception as exc:  # noqa: BLE001 - reported per action, the rest still runs
            actions.append({"what": f, "status": "failed", "error": str(exc)[-500:]})
            ok = False
    if docker:
        try:
            found = set()
            for lab in RKE1_LABELS:
                found.update(run_argv([docker, "ps", "-aq", "--filter", f"label={lab}"]).split())
            repos = rke1_repos(read_join_record(path))
            for line in run_argv([docker, "ps", "-a", "--format", "{{.ID}} {{.Image}}"]).splitlines():
                parts = line.split()
                if len(parts) >= 2 and repo_matches(parts[1], repos):
                    found.add(parts[0])
            ids = sorted(found)
            if ids:
                run_argv([docker, "rm", "-f", *ids])
                actions.append({"what": "rke1-containers", "status": "ok", "count": str(len(ids))})
        except Exception as exc:  # noqa: BLE001
            actions.append({"what": "rke1-containers", "status": "failed", "error": str(exc)[-500:]})
            ok = False
    for d in CLEAN_DIRS + (JOIN_RECORD,):
        p = path(d)
        if not os.path.lexists(p):
            continue
        try:
            if os.path.isdir(p) and not os.path.islink(p):
                shutil.rmtree(p)
            else:
                os.unlink(p)
            actions.append({"what": d, "status": "removed"})
        except OSError as exc:
            actions.append({"what": d, "status": "failed", "error": str(exc)})
            ok = False
    return {"ok": ok, "actions": actions, "ms": round((time.perf_counter() - t0) * 1e3, 1)}


def read_join_record(path: Callable[[str], str]) -> Optional[Dict[str, Any]]:
    try:
        with open(path(JOIN_RECORD), "r", encoding="utf-8") as fh:
            doc = json.load(fh)
        return doc if isinstance(doc, dict) else None
    except (OSError, ValueError):
        return None


def write_join_record(path: Callable[[str], str], record: Dict[str, Any]) -> None:
    p = path(JOIN_RECORD)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    tmp = p + ".tmp"
    with open(tmp, "w", encoding="utf-8") as fh:
        json.dump(record, fh, sort_keys=True)
        fh.write("\n")
    os.replace(tmp, p)
