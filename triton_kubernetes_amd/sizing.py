"""Machine sizes and OS images the pinned stack (Rancher v2.8.5, Docker 24.0) can run on.

One table for the CLI defaults and the module variable defaults
(``terraform/generate.py``), so the two cannot drift: the reference's CLI default
``t2.micro`` (1 GiB, ``create/manager_aws.go``) silently overrode its module's size, and
a Rancher v2.8 server does not start in 1 GiB.

* the Rancher server (manager) needs at least :data:`SERVER_MIN_GIB` of memory;
* a downstream node (etcd / control plane / worker) at least :data:`NODE_MIN_GIB`;
* a size the framework knows to be smaller is refused with the reason (sizes it does not
  know, or that a cloud listing reports with memory, are checked when the memory is
  known);
* OS images are the Ubuntu LTS release the Docker 24.0 install script supports (22.04);
  the reference's filter was xenial 16.04 for its Docker 17.03.
"""

from typing import Dict, Optional, Tuple

from .errors import ConfigError
from .versions import RANCHER_VERSION

SERVER_MIN_GIB = 4.0  # Rancher v2.8 server (single node, small)
NODE_MIN_GIB = 4.0    # RKE node with etcd / control plane / kubelet

# (provider, "manager" | "host") -> (module variable, default)
DEFAULT_SIZES: Dict[Tuple[str, str], Tuple[str, str]] = {
    ("aws", "manager"): ("aws_instance_type", "t3.medium"),
    ("aws", "host"): ("aws_instance_type", "t3.large"),
    ("gcp", "manager"): ("gcp_machine_type", "n1-standard-2"),
    ("gcp", "host"): ("gcp_machine_type", "n1-standard-4"),
    ("azure", "manager"): ("azure_size", "Standard_D4s_v5"),
    ("azure", "host"): ("azure_size", "Standard_D4s_v5"),
    ("triton", "manager"): ("master_triton_machine_package", "k4-highcpu-kvm-7.75G"),
    ("triton", "host"): ("triton_machine_package", "k4-highcpu-kvm-7.75G"),
    ("vsphere", "host"): ("vsphere_memory_mb", "4096"),
}
VSPHERE_DEFAULT_CPUS = "2"

# memory (GiB) of the sizes the framework names or that the reference defaulted to
KNOWN_MEMORY_GIB: Dict[str, float] = {
    "t2.nano": 0.5, "t2.micro": 1, "t2.small": 2, "t2.medium": 4, "t2.large": 8,
    "t3.nano": 0.5, "t3.micro": 1, "t3.small": 2, "t3.medium": 4, "t3.large": 8, "t3.xlarge": 16,
    "m5.large": 8, "m5.xlarge": 16,
    "n1-standard-1": 3.75, "n1-standard-2": 7.5, "n1-standard-4": 15, "e2-small": 2, "e2-medium": 4,
    "e2-standard-2": 8,
    "Standard_A0": 0.75, "Standard_A1": 1.75, "Standard_B1s": 1, "Standard_B2s": 4, "Standard_D2s_v5": 8,
    "Standard_D4s_v5": 16,
    "k4-highcpu-kvm-1.75G": 1.75, "k4-highcpu-kvm-3.75G": 3.75, "k4-highcpu-kvm-7.75G": 7.75,
}

# Ubuntu LTS the Docker 24.0 install script supports (versions.DOCKER_INSTALL_URL)
UBUNTU_LTS = "22.04"
AWS_AMI_FILTER = "*hvm-ssd/ubuntu-jammy-22.04-amd64-server*"
GCP_IMAGE_PREFIX = "ubuntu-2204"
TRITON_IMAGE_PREFIX = "ubuntu-certified-22.04"


def default_size(provider: str, kind: str) -> Tuple[str, str]:
    return DEFAULT_SIZES[(provider, kind)]


def memory_gib(provider: str, value: str) -> Optional[float]:
    """Memory of a size value, when known (vSphere: the value is the memory in MB)."""
    if provider == "vsphere":
        try:
            return int(value) / 1024.0
        except ValueError:
            return None
    return KNOWN_MEMORY_GIB.get(value)


def check_size(provider: str, kind: str, value: str, memory: Optional[float] = None) -> None:
    """Refuse a size whose memory (given, or known) is below the minimum for ``kind``."""
    mem = memory if memory is not None else memory_gib(provider, value)
    floor = SERVER_MIN_GIB if kind == "manager" else NODE_MIN_GIB
    if mem is not None and mem < floor:
        what = f"the Rancher {RANCHER_VERSION} server" if kind == "manager" else "a Kubernetes node"
        key = DEFAULT_SIZES[(provider, kind)][0]
        raise ConfigError(f"{key} '{value}' has {mem:g} GiB of memory; {what} needs at least {floor:g} GiB "
                          f"(default: {DEFAULT_SIZES[(provider, kind)][1]}).")


__all__ = ["SERVER_MIN_GIB", "NODE_MIN_GIB", "DEFAULT_SIZES", "KNOWN_MEMORY_GIB", "default_size", "memory_gib",
           "check_size", "AWS_AMI_FILTER", "GCP_IMAGE_PREFIX", "TRITON_IMAGE_PREFIX", "UBUNTU_LTS"]
