"""Manager-host scripts for the DirectExecutor's SSH path.

Re-designs of the reference's manager bootstrap (S1-S3,
``terraform/modules/files/*.sh.tpl``) for a current Rancher 2.x:

* install the container runtime only if absent (the reference always pipes a
  pinned 17.03 installer into ``sh``), data-root on ``/mnt/docker`` only when
  that mount exists (the reference hard-codes ``/home/ubuntu``, Q10);
* ``docker run rancher/rancher`` with ``CATTLE_BOOTSTRAP_PASSWORD`` from a 0600 env
  file (Rancher ≥2.6 has no admin/admin; a random password kept in the state backend,
  ``rancher/bootstrap_secret.py``) — polling with a 1 s interval instead of 5 s;
* :func:`manager_setup_script` is the on-host variant of S3 used with
  ``rancher_bootstrap: remote`` (operator cannot reach port 443).
"""

import json
import shlex
from typing import Any, Dict

from ..versions import DOCKER_INSTALL_URL as DEFAULT_DOCKER_INSTALL_URL
from ..versions import SERVER_IMAGE as DEFAULT_SERVER_IMAGE


def _q(v: Any) -> str:
    return shlex.quote(str(v))


def docker_install_lines(url: str, sha256: str = "") -> str:
    """Install the container runtime when absent: download, verify (when a checksum is
    configured), then run — never ``curl | sh`` of an unchecked stream."""
    check = (f"  echo {_q(sha256 + '  /tmp/tk-install-docker.sh')} | sha256sum -c - >/dev/null || "
             f"{{ echo 'docker install script checksum mismatch' >&2; exit 1; }}\n") if sha256 else ""
    return (f"if ! command -v docker >/dev/null 2>&1; then\n"
            f"  curl -fsSL -o /tmp/tk-install-docker.sh {_q(url)}\n{check}"
            f"  sudo sh /tmp/tk-install-docker.sh && rm -f /tmp/tk-install-docker.sh\n"
            f"fi\n")


def manager_install_script(cfg: Dict[str, Any], bootstrap_pw: str) -> str:
    url = cfg.get("docker_engine_install_url") or DEFAULT_DOCKER_INSTALL_URL
    image = cfg.get("rancher_server_image") or DEFAULT_SERVER_IMAGE
    reg, user, pw = (cfg.get("rancher_registry", ""), cfg.get("rancher_registry_username", ""),
                     cfg.get("rancher_registry_password", ""))
    login = f"echo {_q(pw)} | sudo docker login -u {_q(user)} --password-stdin {_q(reg)}\n" if user else ""
    return f"""#!/bin/bash
set -euo pipefail
if command -v firewalld >/dev/null 2>&1; then sudo systemctl disable --now firewalld.service || true; fi
{docker_install_lines(url, cfg.get("docker_install_sha256", ""))}if mountpoint -q /mnt && [ ! -f /etc/docker/daemon.json ]; then
  echo '{{"storage-driver": "overlay2", "data-root": "/mnt/docker"}}' | sudo tee /etc/docker/daemon.json >/dev/null
  sudo systemctl restart docker
fi
{login}sudo docker pull {_q(image)}
if ! sudo docker ps --format '{{{{.Image}}}}' | grep -x {_q(image)} >/dev/null; then
  # the first-login password through a 0600 env file, removed once the container runs:
  # never on a command line (ps) -- rancher/bootstrap_secret.py
  envf=$(umask 077; mktemp)
  trap 'rm -f "$envf"' EXIT
  cat > "$envf" <<'TK_BOOTSTRAP_EOF'
CATTLE_BOOTSTRAP_PASSWORD={bootstrap_pw}
TK_BOOTSTRAP_EOF
  sudo docker run -d --restart=unless-stopped --privileged -p 80:80 -p 443:443 --env-file "$envf" {_q(image)}
  rm -f "$envf"
fi
for i in $(seq 1 600); do
  if curl -ksf https://127.0.0.1/ping >/dev/null 2>&1; then
    # the server's CA as served on this host (loopback: nothing between us and it); the
    # CLI reads it over the pinned SSH session and verifies the server against it
    curl -ksf https://127.0.0.1/cacerts > ~/rancher_cacerts.pem.tmp && mv ~/rancher_cacerts.pem.tmp ~/rancher_cacerts.pem
    exit 0
  fi
  sleep 1
done
echo 'rancher server did not come up' >&2; exit 1
"""


def manager_setup_script(cfg: Dict[str, Any], server_url: str, bootstrap_pw: str) -> str:
    """On-host API bootstrap (S3, ``rancher_bootstrap: remote``: the operator cannot reach
    port 443); prints the token JSON as the last line.  Logs in with the bootstrap password,
    or -- re-run after the change -- with the admin password.  The request bodies carrying a
    password reach curl on its stdin (a quoted heredoc), never its command line: the script
    itself travels over the pinned SSH session's stdin and is never written to the host."""
    pw = cfg.get("rancher_admin_password", "")
    token_req = json.dumps({"type": "token", "description": "Managed by triton-kubernetes",
                            "name": "triton-kubernetes", "ttl": 0})
    url_req = json.dumps({"name": "server-url", "value": server_url})
    pw_req = json.dumps({"currentPassword": bootstrap_pw, "newPassword": pw})
    login_req = json.dumps({"username": "admin", "password": bootstrap_pw, "ttl": 60000})
    relogin_req = json.dumps({"username": "admin", "password": pw, "ttl": 60000})
    post = "curl -ksf -X POST -H 'Content-Type: application/json' --data-binary @-"
    return f"""#!/bin/bash
set -euo pipefail
R=https://127.0.0.1
changed=0
login=$({post} "$R/v3-public/localProviders/local?action=login" <<'TK_EOF'
{login_req}
TK_EOF
) || {{
  login=$({post} "$R/v3-public/localProviders/local?action=login" <<'TK_EOF'
{relogin_req}
TK_EOF
)
  changed=1
}}
initial=$(printf '%s' "$login" | python3 -c 'import json,sys; print(json.load(sys.stdin)["token"])')
tok=$(curl -ksf -u "$initial" -X POST -H 'Content-Type: application/json' -d {_q(token_req)} "$R/v3/token")
(umask 077; printf '%s' "$tok" > ~/rancher_api_key)
ak=$(printf '%s' "$tok" | python3 -c 'import json,sys; print(json.load(sys.stdin)["name"])')
sk=$(printf '%s' "$tok" | python3 -c 'import json,sys; print(json.load(sys.stdin)["token"].split(":",1)[1])')
if [ "$changed" != 1 ]; then
  curl -ksf -u "$ak:$sk" -X POST -H 'Content-Type: application/json' --data-binary @- "$R/v3/users?action=changepassword" >/dev/null <<'TK_EOF'
{pw_req}
TK_EOF
fi
curl -ksf -u "$ak:$sk" -X PUT -H 'Content-Type: application/json' -d {_q(url_req)} "$R/v3/settings/server-url" >/dev/null
printf '%s\\n' "$tok"
"""
