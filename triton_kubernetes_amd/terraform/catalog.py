"""Catalog of the Terraform module library (``terraform/modules/*``).

The 17 reference modules keep their names, input
variables and outputs — the module name is part of the ``main.tf.json``
``source`` contract.  Two MI355X modules are added:

* ``bare-metal-mi355x-rancher-k8s-host`` — bare-metal 8xMI355X worker: ROCm /
  amdgpu preflight, ``/dev/kfd`` + ``/dev/dri`` passthrough, native topology
  labeller (N1) feeding agent ``--label`` flags, RCCL environment file;
* ``rancher-k8s-mi355x-addons`` — cluster add-on step run once the cluster is
  active: ROCm k8s device plugin + node labeller DaemonSets, xGMI affinity
  example, RCCL readiness Job (N2).

Executors use the catalog to know which outputs a module exposes (root outputs
for Terraform >= 0.12, whose ``terraform output -module`` no longer exists).
"""

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

MODULES_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "modules")

MANAGER_OUTPUTS = ("rancher_url", "rancher_access_key", "rancher_secret_key")
CLUSTER_OUTPUTS = ("rancher_cluster_id", "rancher_cluster_registration_token", "rancher_cluster_ca_checksum")


@dataclass(frozen=True)
class ModuleInfo:
    name: str
    kind: str  # manager | cluster | host | addon
    provider: str  # triton | aws | gcp | azure | baremetal | vsphere
    outputs: Tuple[str, ...] = ()
    mi355x: bool = False
    # which provider-network outputs a host module consumes from its cluster
    consumes: Tuple[str, ...] = field(default_factory=tuple)

    @property
    def path(self) -> str:
        return f"terraform/modules/{self.name}"

    @property
    def local_dir(self) -> str:
        return os.path.join(MODULES_DIR, self.name)


_MODULES: List[ModuleInfo] = [
    # managers (T1-T5)
    ModuleInfo("triton-rancher", "manager", "triton", MANAGER_OUTPUTS),
    ModuleInfo("aws-rancher", "manager", "aws", MANAGER_OUTPUTS),
    ModuleInfo("gcp-rancher", "manager", "gcp", MANAGER_OUTPUTS),
    ModuleInfo("azure-rancher", "manager", "azure", MANAGER_OUTPUTS),
    ModuleInfo("bare-metal-rancher", "manager", "baremetal", MANAGER_OUTPUTS),
    # clusters (T6-T11)
    ModuleInfo("triton-rancher-k8s", "cluster", "triton", CLUSTER_OUTPUTS),
    ModuleInfo("aws-rancher-k8s", "cluster", "aws",
               CLUSTER_OUTPUTS + ("aws_subnet_id", "aws_security_group_id", "aws_key_name")),
    ModuleInfo("gcp-rancher-k8s", "cluster", "gcp",
               CLUSTER_OUTPUTS + ("gcp_compute_network_name", "gcp_compute_firewall_host_tag")),
    ModuleInfo("azure-rancher-k8s", "cluster", "azure",
               CLUSTER_OUTPUTS + ("azure_resource_group_name", "azure_network_security_group_id", "azure_subnet_id")),
    ModuleInfo("bare-metal-rancher-k8s", "cluster", "baremetal", CLUSTER_OUTPUTS),
    ModuleInfo("vsphere-rancher-k8s", "cluster", "vsphere",
               CLUSTER_OUTPUTS + ("vsphere_datacenter_name", "vsphere_datastore_name", "vsphere_resource_pool_name",
                                  "vsphere_network_name")),
    # hosts (T12-T17)
    ModuleInfo("triton-rancher-k8s-host", "host", "triton"),
    ModuleInfo("aws-rancher-k8s-host", "host", "aws",
               consumes=("aws_subnet_id", "aws_security_group_id", "aws_key_name")),
    ModuleInfo("gcp-rancher-k8s-host", "host", "gcp",
               consumes=("gcp_compute_network_name", "gcp_compute_firewall_host_tag")),
    ModuleInfo("azure-rancher-k8s-host", "host", "azure",
               consumes=("azure_resource_group_name", "azure_network_security_group_id", "azure_subnet_id")),
    ModuleInfo("bare-metal-rancher-k8s-host", "host", "baremetal"),
    ModuleInfo("vsphere-rancher-k8s-host", "host", "vsphere",
               consumes=("vsphere_datacenter_name", "vsphere_datastore_name", "vsphere_resource_pool_name",
                         "vsphere_network_name")),
    # MI355X additions
    ModuleInfo("bare-metal-mi355x-rancher-k8s-host", "host", "baremetal", ("gpu_node_labels",), mi355x=True),
    ModuleInfo("rancher-k8s-mi355x-addons", "addon", "baremetal", ("addons_applied",), mi355x=True),
]

CATALOG: Dict[str, ModuleInfo] = {m.name: m for m in _MODULES}
REFERENCE_MODULES = [m.name for m in _MODULES if not m.mi355x]


def module_source(source_url: str, module_path: str, source_ref: str) -> str:
    """``<url>//<path>?ref=<ref>`` (``create/manager.go:160-171``)."""
    return f"{source_url}//{module_path}?ref={source_ref}"


def module_from_source(source: str) -> Optional[ModuleInfo]:
    """Identify the catalog module a ``source`` string points at."""
    path = source.split("?", 1)[0]
    name = path.rstrip("/").rsplit("/", 1)[-1]
    return CATALOG.get(name)


def outputs_for_source(source: str) -> Tuple[str, ...]:
    info = module_from_source(source)
    return info.outputs if info else ()
