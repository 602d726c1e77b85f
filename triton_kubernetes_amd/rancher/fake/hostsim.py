"""What joining a cluster leaves on a host, for the fakes (sim-mode node agents, the fake
Rancher's installer, the tests' SSH hosts).

A real ``system-agent-install.sh`` installs ``rancher-system-agent`` (binary, systemd unit,
``/etc/rancher/agent``, its uninstaller) and the agent then installs RKE2 for the node's
role (``/var/lib/rancher/rke2``, ``/etc/rancher/rke2``, ``rke2-killall.sh``,
``rke2-uninstall.sh``).  The agent keeps its connection to the server it joined in
``/var/lib/rancher/agent/rancher2_connection_info.json``.

Joining a second cluster while that installation is in place does not work: the new
system-agent configuration is written, but the RKE2 left behind still holds the first
cluster's datastore, certificates and server address, and the node never turns Ready.
The model refuses such a join at once with that reason (a fake may refuse what the real
system fails on later; ``tests/test_host_teardown.py`` pins it), and models the vendor
uninstallers: each removes what its component installed.

Everything lives under a host root (``TK_HOST_ROOT`` for the shell side).  Without one
(an empty root or ``/``) nothing is modelled: the fakes never write to the machine they
run on.
"""

import json
import os
import stat
from typing import Optional

CONNECTION_INFO = "/var/lib/rancher/agent/rancher2_connection_info.json"

# the vendor uninstallers as this model installs them: each removes its component
UNINSTALLERS = {
    "/usr/local/bin/rancher-system-agent-uninstall.sh": """#!/bin/sh
R=${TK_HOST_ROOT:-}
rm -rf "$R/etc/rancher/agent" "$R/var/lib/rancher/agent" "$R/usr/local/bin/rancher-system-agent" \\
  "$R/etc/systemd/system/rancher-system-agent.service"
rm -f "$0"
""",
    "/usr/local/bin/rke2-killall.sh": """#!/bin/sh
R=${TK_HOST_ROOT:-}
rm -f "$R/run/rke2-running"
""",
    "/usr/local/bin/rke2-uninstall.sh": """#!/bin/sh
R=${TK_HOST_ROOT:-}
[ -e "$R/run/rke2-running" ] && "$R/usr/local/bin/rke2-killall.sh"
rm -rf "$R/etc/rancher/rke2" "$R/var/lib/rancher/rke2" "$R/var/lib/kubelet" "$R/usr/local/bin/rke2" \\
  "$R/usr/local/bin/rke2-killall.sh"
rm -f "$0"
""",
}

RKE2_STATE = "/var/lib/rancher/rke2"
LEFTOVER = ("RKE2 of an earlier cluster is still installed on this host (/var/lib/rancher/rke2): run "
            "rke2-uninstall.sh before it joins another cluster")
REFUSAL = ("rancher-system-agent is already installed on this host and connected to {server}: "
           "its RKE2 still holds that cluster's datastore and certificates, so the node cannot join "
           "another cluster until rancher-system-agent-uninstall.sh and rke2-uninstall.sh have run")


def _p(root: str, path: str) -> str:
    return os.path.join(root, path.lstrip("/"))


def conflict(root: str, server: str, token: str) -> Optional[str]:
    """The refusal for a join of ``(server, token)`` on the host at ``root``, or None."""
    try:
        with open(_p(root, CONNECTION_INFO), "r", encoding="utf-8") as fh:
            info = json.load(fh)
    except (OSError, ValueError):
        # no agent connection, but an RKE2 datastore left behind (agent uninstalled only)
        return LEFTOVER if os.path.exists(_p(root, RKE2_STATE)) else None
    if info.get("server") == server.rstrip("/") and info.get("token") == token:
        return None  # re-registration with the same cluster
    return REFUSAL.format(server=info.get("server", "?"))


def install(root: str, server: str, token: str, distribution: str = "rke2") -> None:
    """Leave on the host at ``root`` what a completed join leaves."""
    files = {CONNECTION_INFO: json.dumps({"server": server.rstrip("/"), "token": token,
                                          "distribution": distribution}) + "\n"}
    if distribution == "rke2":
        files.update({"/etc/rancher/agent/config.yaml": "workDirectory: /var/lib/rancher/agent/work\n",
                      "/usr/local/bin/rancher-system-agent": "#!/bin/sh\n",
                      "/etc/rancher/rke2/config.yaml.d/50-rancher.yaml": f"server: {server}\n",
                      "/var/lib/rancher/rke2/server/db/etcd/member": "",
                      "/usr/local/bin/rke2": "#!/bin/sh\n",
                      "/run/rke2-running": ""})
        files.update(UNINSTALLERS)
    else:  # RKE1: the agent container's state (the containers themselves live in docker)
        files.update({"/etc/kubernetes/ssl/kube-node.pem": "", "/var/lib/etcd/member": ""})
    for path, text in files.items():
        full = _p(root, path)
        os.makedirs(os.path.dirname(full), exist_ok=True)
        with open(full, "w", encoding="utf-8") as fh:
            fh.write(text)
        if text.startswith("#!"):
            os.chmod(full, os.stat(full).st_mode | stat.S_IXUSR | stat.S_IXGRP | stat.S_IXOTH)


def installer_shell() -> str:
    """The same model for the fake's ``system-agent-install.sh`` (after its flags are parsed:
    ``$server``, ``$token``): refuse a conflicting join, else record the installation."""
    lines = [
        'R=${TK_HOST_ROOT:-}',
        f'ci="$R{CONNECTION_INFO}"',
        'if [ -r "$ci" ]; then',
        '  prev_server=$(sed -n \'s/.*"server": "\\([^"]*\\)".*/\\1/p\' "$ci")',
        '  prev_token=$(sed -n \'s/.*"token": "\\([^"]*\\)".*/\\1/p\' "$ci")',
        '  if [ "$prev_server" != "${server%/}" ] || [ "$prev_token" != "$token" ]; then',
        '    echo "system-agent-install: ' + REFUSAL.replace("{server}", "$prev_server").replace('"', '\\"')
        + '" >&2',
        '    exit 1',
        '  fi',
        f'elif [ -e "$R{RKE2_STATE}" ]; then',
        f'  echo "system-agent-install: {LEFTOVER}" >&2',
        '  exit 1',
        'fi',
        '_tk_install_files() {',
        f'  mkdir -p "$(dirname "$ci")" "$R/etc/rancher/agent" "$R/etc/rancher/rke2/config.yaml.d" '
        f'"$R/var/lib/rancher/rke2/server/db/etcd" "$R/usr/local/bin" "$R/run"',
        '  printf \'{"server": "%s", "token": "%s", "distribution": "rke2"}\\n\' "${server%/}" "$token" > "$ci"',
        '  echo "workDirectory: /var/lib/rancher/agent/work" > "$R/etc/rancher/agent/config.yaml"',
        '  echo "server: $server" > "$R/etc/rancher/rke2/config.yaml.d/50-rancher.yaml"',
        '  : > "$R/var/lib/rancher/rke2/server/db/etcd/member"; : > "$R/run/rke2-running"',
        '  printf \'#!/bin/sh\\n\' > "$R/usr/local/bin/rancher-system-agent"',
        '  printf \'#!/bin/sh\\n\' > "$R/usr/local/bin/rke2"',
    ]
    for path, text in UNINSTALLERS.items():
        lines.append(f"  cat > \"$R{path}\" <<'TK_UNINSTALL_EOF'")
        lines.extend(text.rstrip("\n").splitlines())
        lines.append("TK_UNINSTALL_EOF")
        lines.append(f'  chmod +x "$R{path}"')
    lines.append("}")
    return "\n".join(lines) + "\n"
