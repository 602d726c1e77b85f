#!/bin/bash
# Container-runtime installer for cluster hosts (S6 equivalent).
#
#   DOCKER_VERSION=24.0 ./install-docker.sh [--mirror Aliyun|AzureChinaCloud] [--dry-run]
#
# Installs docker-ce <DOCKER_VERSION>.* from the Docker package repository for
# the running distribution (Ubuntu/Debian via apt, RHEL/Rocky/Alma/CentOS/Fedora
# via dnf/yum), pins it, enables the service and sets the overlay2 storage
# driver.  Idempotent: exits early when the requested major.minor is present.
set -euo pipefail

DOCKER_VERSION=${DOCKER_VERSION:-24.0}
REPO_BASE=https://download.docker.com
DRY_RUN=0
while [ $# -gt 0 ]; do
  case "$1" in
    --mirror)
      case "${2:-}" in
        Aliyun) REPO_BASE=https://mirrors.aliyun.com/docker-ce ;;
        AzureChinaCloud) REPO_BASE=https://mirror.azure.cn/docker-ce ;;
        *) echo "unknown mirror '${2:-}' (Aliyun, AzureChinaCloud)" >&2; exit 64 ;;
      esac
      shift 2 ;;
    --dry-run) DRY_RUN=1; shift ;;
    *) echo "unknown option $1" >&2; exit 64 ;;
  esac
done

run() { if [ "$DRY_RUN" = 1 ]; then echo "+ $*"; else "$@"; fi; }
as_root() { if [ "$(id -u)" = 0 ]; then run "$@"; else run sudo "$@"; fi; }

if command -v docker >/dev/null 2>&1; then
  have=$(docker version --format '{{.Server.Version}}' 2>/dev/null || docker --version | sed 's/.*version \([0-9.]*\).*/\1/')
  case "$have" in
    "$DOCKER_VERSION"|"$DOCKER_VERSION".*) echo "docker $have already installed"; exit 0 ;;
  esac
fi

[ -r /etc/os-release ] || { echo "cannot detect the distribution (/etc/os-release missing)" >&2; exit 1; }
. /etc/os-release
ID_LIKE=${ID_LIKE:-}
case "$ID $ID_LIKE" in
  *ubuntu*|*debian*)
    distro=$ID; [ "$distro" = ubuntu ] || [ "$distro" = debian ] || distro=$(case "$ID_LIKE" in *ubuntu*) echo ubuntu;; *) echo debian;; esac)
    codename=${VERSION_CODENAME:-${UBUNTU_CODENAME:-}}
    [ -n "$codename" ] || { echo "no VERSION_CODENAME in /etc/os-release" >&2; exit 1; }
    as_root apt-get update -qq
    as_root apt-get install -y -qq ca-certificates curl gnupg
    as_root install -m 0755 -d /etc/apt/keyrings
    if [ "$DRY_RUN" = 1 ]; then echo "+ curl $REPO_BASE/linux/$distro/gpg | gpg --dearmor > /etc/apt/keyrings/docker.gpg"
    else curl -fsSL "$REPO_BASE/linux/$distro/gpg" | as_root gpg --dearmor --yes -o /etc/apt/keyrings/docker.gpg; fi
    line="deb [arch=$(dpkg --print-architecture) signed-by=/etc/apt/keyrings/docker.gpg] $REPO_BASE/linux/$distro $codename stable"
    if [ "$DRY_RUN" = 1 ]; then echo "+ echo '$line' > /etc/apt/sources.list.d/docker.list"
    else echo "$line" | as_root tee /etc/apt/sources.list.d/docker.list >/dev/null; fi
    as_root apt-get update -qq
    pkgver=$(apt-cache madison docker-ce 2>/dev/null | awk -v v="$DOCKER_VERSION" '$3 ~ ("^[0-9]+:" v "\\.") {print $3; exit}')
    [ -n "$pkgver" ] || [ "$DRY_RUN" = 1 ] || { echo "docker-ce $DOCKER_VERSION.* not found in $REPO_BASE" >&2; exit 1; }
    pkgver=${pkgver:-$DOCKER_VERSION}
    as_root apt-get install -y -qq "docker-ce=$pkgver" "docker-ce-cli=$pkgver" containerd.io
    as_root apt-mark hold docker-ce docker-ce-cli
    ;;
  *rhel*|*centos*|*fedora*|*rocky*|*almalinux*)
    pm=$(command -v dnf || command -v yum)
    repo_distro=centos; [ "$ID" = fedora ] && repo_distro=fedora
    as_root "$pm" install -y -q dnf-plugins-core 2>/dev/null || as_root "$pm" install -y -q yum-utils
    as_root "$pm" config-manager --add-repo "$REPO_BASE/linux/$repo_distro/docker-ce.repo"
    as_root "$pm" install -y -q "docker-ce-$DOCKER_VERSION.*" "docker-ce-cli-$DOCKER_VERSION.*" containerd.io
    ;;
  *)
    echo "unsupported distribution '$ID'" >&2; exit 1 ;;
esac

as_root mkdir -p /etc/docker
if [ ! -f /etc/docker/daemon.json ]; then
  if [ "$DRY_RUN" = 1 ]; then echo "+ write /etc/docker/daemon.json (overlay2)"
  else echo '{"storage-driver": "overlay2", "log-driver": "json-file", "log-opts": {"max-size": "100m"}}' | as_root tee /etc/docker/daemon.json >/dev/null; fi
fi
as_root systemctl enable --now docker
if [ -n "${SUDO_USER:-}" ]; then as_root usermod -aG docker "$SUDO_USER" || true; fi
echo "docker $DOCKER_VERSION installed"
