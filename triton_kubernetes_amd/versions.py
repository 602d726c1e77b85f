"""Pinned component versions: one place, used by every delivery path.

The reference pairs ``rancher/server:v2.0.0-beta2`` with the RKE releases that
server shipped (``create/cluster.go:349-356``,
``terraform/modules/triton-rancher/variables.tf:14-22``).  This framework pins
Rancher v2.10.3 and offers the Kubernetes releases of that Rancher line for its two
custom-cluster distributions:

* **RKE2** (default): ``provisioning.cattle.io/v1`` ``Cluster`` objects with an
  ``rkeConfig``; nodes join by running the server's ``system-agent-install.sh``
  (``rancher-system-agent``), no Docker needed.  Current Rancher lines provision
  RKE2 / K3s only;
* **RKE1** (compatibility with reference-era documents, ``workflows/migrate.py``): the
  v3 ``cluster`` with ``rancherKubernetesEngineConfig`` and ``docker run
  rancher/rancher-agent`` -- RKE1 is end-of-life, kept because v2.10 still runs it.

The distribution follows from the release string (``v1.31.6+rke2r1`` vs
``v1.31.6-rancher1-1``) unless ``k8s_distribution`` says otherwise.  The CLI choices,
the module defaults and validations, the Rancher client, the DirectExecutor and the
bench all read these lists, and the fake Rancher server rejects anything else
(``rancher/fake/``).

Rancher ≥2.6 no longer starts with admin/admin: it takes the first admin
password from ``CATTLE_BOOTSTRAP_PASSWORD`` (or generates a random one).  Every
manager path starts the server with :func:`bootstrap_password` — derived from the
manager name and the admin password, so a re-run of a half-finished bootstrap
(the container already running) logs in with the same value — and then changes it
to ``rancher_admin_password``.  The Terraform modules compute the same value
(``sha256("tk-bootstrap:<name>:<password>")``, first 32 hex digits).
"""

import hashlib
import re
from typing import List, Optional, Sequence, Tuple

RANCHER_VERSION = "v2.10.3"
SERVER_IMAGE = f"rancher/rancher:{RANCHER_VERSION}"
AGENT_IMAGE = f"rancher/rancher-agent:{RANCHER_VERSION}"

# RKE1 Kubernetes releases of the Rancher v2.10.3 line (display name, kubernetesVersion).
# The server's own list (setting ``k8s-versions-current``) is authoritative at create
# time: a pinned patch release the server no longer offers is replaced by the server's
# release of the same minor (RancherClient.resolve_k8s_version).
K8S_VERSIONS: List[Tuple[str, str]] = [
    ("v1.31", "v1.31.6-rancher1-1"),
    ("v1.30", "v1.30.10-rancher1-1"),
    ("v1.29", "v1.29.14-rancher1-1"),
    ("v1.28", "v1.28.15-rancher1-1"),
]
DEFAULT_RKE1_VERSION = K8S_VERSIONS[0][1]
K8S_MINORS = tuple(d for d, _ in K8S_VERSIONS)

# RKE2 releases of the same Rancher line (the server's ``/v1-rke2-release/releases``,
# from its KDM data, is authoritative at create time)
RKE2_VERSIONS: List[Tuple[str, str]] = [
    ("v1.31", "v1.31.6+rke2r1"),
    ("v1.30", "v1.30.10+rke2r1"),
    ("v1.29", "v1.29.14+rke2r1"),
]
DEFAULT_RKE2_VERSION = RKE2_VERSIONS[0][1]
RKE2_MINORS = tuple(d for d, _ in RKE2_VERSIONS)

DISTRIBUTIONS = ("rke2", "rke1")
DEFAULT_DISTRIBUTION = "rke2"
DEFAULT_K8S_VERSION = DEFAULT_RKE2_VERSION
# RKE2 custom clusters live in this namespace of the Rancher management cluster
FLEET_NAMESPACE = "fleet-default"
SYSTEM_AGENT_INSTALL_PATH = "/system-agent-install.sh"
RKE2_CNIS = ("canal", "calico", "cilium", "flannel")

# container runtime: Rancher's install script for a Docker release RKE1 v1.5 supports
DOCKER_VERSION = "24.0"
DOCKER_INSTALL_URL = f"https://releases.rancher.com/install-docker/{DOCKER_VERSION}.sh"

# MI355X add-ons (pinned tags, never :latest)
DEVICE_PLUGIN_IMAGE = "rocm/k8s-device-plugin:1.31.0.6"
NODE_LABELLER_IMAGE = "rocm/k8s-device-plugin:labeller-1.31.0.6"  # opt-in (node_labeller_image)
# the RCCL readiness Job runs the node's installed rccl-ready (hostPath /opt/triton-kubernetes
# and /opt/rocm), so any small glibc image serves; pinned by tag
RCCL_PROBE_IMAGE = "ubuntu:22.04"
# the RCCL-env injector (mutating admission webhook, k8s/webhook.py) runs the stdlib server
WEBHOOK_IMAGE = "python:3.11-slim"

# Rancher ≥2.6 refuses shorter admin passwords (setting password-min-length)
PASSWORD_MIN_LENGTH = 12

_K8S_RE = re.compile(r"^v(\d+)\.(\d+)(?:\.(\d+))?(-rancher\d+-\d+|\+rke2r\d+)?$")


def bootstrap_password(manager_name: str, admin_password: str) -> str:
    """First-login password handed to the server as ``CATTLE_BOOTSTRAP_PASSWORD``."""
    return hashlib.sha256(f"tk-bootstrap:{manager_name}:{admin_password}".encode()).hexdigest()[:32]


def k8s_minor(version: str) -> Optional[str]:
    """``v1.28.10-rancher1-1`` / ``v1.28`` -> ``v1.28``; None if not a version string."""
    m = _K8S_RE.fullmatch(version or "")
    return f"v{m.group(1)}.{m.group(2)}" if m else None


def distribution_of(version: str) -> Optional[str]:
    """``rke2`` for ``...+rke2rN``, ``rke1`` for ``...-rancherN-N``, None for a bare
    ``vX.Y[.Z]`` (the distribution then comes from ``k8s_distribution``)."""
    if "+rke2r" in (version or ""):
        return "rke2"
    if "-rancher" in (version or ""):
        return "rke1"
    return None


def releases(distribution: str) -> List[Tuple[str, str]]:
    return RKE2_VERSIONS if distribution == "rke2" else K8S_VERSIONS


def default_version(distribution: str) -> str:
    return DEFAULT_RKE2_VERSION if distribution == "rke2" else DEFAULT_RKE1_VERSION


def resolve_distribution(version: str = "", distribution: str = "") -> str:
    """The distribution a cluster is created with: explicit ``distribution``, else the
    one the release string names, else the default (RKE2).  A release string of the
    other distribution is an error."""
    implied = distribution_of(version)
    chosen = (distribution or "").strip().lower() or implied or DEFAULT_DISTRIBUTION
    if chosen not in DISTRIBUTIONS:
        raise ValueError(f"k8s_distribution must be one of {', '.join(DISTRIBUTIONS)}. Found '{chosen}'.")
    if implied and implied != chosen:
        raise ValueError(f"Kubernetes version '{version}' is an {implied.upper()} release; "
                         f"k8s_distribution is {chosen}")
    return chosen


def normalize_k8s_version(value: str, distribution: str = "") -> str:
    """Map a display name to its pinned release of ``distribution`` and reject releases
    outside the pinned Rancher line (a v1.9 cluster cannot be created on Rancher 2.10)."""
    dist = resolve_distribution(value, distribution)
    pinned = releases(dist)
    for display, full in pinned:
        if value == display:
            return full
    minor = k8s_minor(value)
    if minor is None or minor not in tuple(d for d, _ in pinned) or distribution_of(value) is None:
        offered = ", ".join(full for _, full in pinned)
        raise ValueError(f"Kubernetes version '{value}' is not an {dist.upper()} release offered by Rancher "
                         f"{RANCHER_VERSION}; choose one of: {offered}")
    return value


def resolve_against(requested: str, offered: Sequence[str]) -> Tuple[str, str]:
    """``(version, note)``: ``requested`` if the server offers it, else the server's newest
    release of the same minor (note says so).  Raises ValueError when the minor is absent."""
    offered = [v for v in offered if v]
    if not offered or requested in offered:
        return requested, ""
    minor = k8s_minor(requested)
    same = [v for v in offered if k8s_minor(v) == minor]
    if not same:
        raise ValueError(f"Kubernetes version '{requested}' is not offered by the Rancher server "
                         f"(offered: {', '.join(offered)})")

    def key(v: str) -> Tuple[int, ...]:
        return tuple(int(x) for x in re.findall(r"\d+", v))

    best = max(same, key=key)
    return best, f"{requested} is not offered by the server; using {best}"


def running_version(release: str, distribution: str) -> str:
    """The version Rancher (``version.gitVersion``) and the kubelets (``kubeletVersion``)
    report for a cluster running ``release``: RKE1 reports the upstream Kubernetes version
    (``v1.30.10`` for ``v1.30.10-rancher1-1``), RKE2 the release itself (``v1.31.6+rke2r1``)."""
    return re.sub(r"-rancher\d+-\d+$", "", release) if distribution == "rke1" else release
