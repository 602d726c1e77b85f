"""vSphere provider: cluster (C29) and node (C36).  No manager (``create/manager.go:119``).

Reference: ``create/cluster_vsphere.go:12-210``, ``create/node_vsphere.go:16-170``.
All vSphere names are free text (the reference has TODOs to list them).  Note
the reference's trailing period in ``"vsphere_user must be specified."`` is kept.
Deliberate fix: node CPU / memory are configurable
(``vsphere_num_cpus`` / ``vsphere_memory_mb``; the reference hard-codes 2/2048).
"""

from typing import Dict, List

from .. import sizing
from ..config.context import Context, expand_home, file_exists, not_blank
from ..state import State
from .common import add_nodes, base_cluster_config, base_node_config, omit_empty

CLUSTER_MODULE = "terraform/modules/vsphere-rancher-k8s"
NODE_MODULE = "terraform/modules/vsphere-rancher-k8s-host"

_CLUSTER_FIELDS = [
    ("vsphere_user", "vSphere User", "Invalid vSphere user", False),
    ("vsphere_password", "vSphere Password", "", True),
    ("vsphere_server", "vSphere Server", "Invalid vSphere server", False),
    ("vsphere_datacenter_name", "vSphere Datacenter Name", "Invalid vSphere datacenter name", False),
    ("vsphere_datastore_name", "vSphere Datastore Name", "Invalid vSphere datastore name", False),
    ("vsphere_resource_pool_name", "vSphere Resource Pool Name", "Invalid vSphere resource pool name", False),
    ("vsphere_network_name", "vSphere Network Name", "Invalid vSphere network name", False),
]


def new_cluster(ctx: Context, backend, state: State) -> str:
    cfg = base_cluster_config(ctx, CLUSTER_MODULE)
    for key, label, invalid, mask in _CLUSTER_FIELDS:
        cfg[key] = ctx.resolve(key, label, mask=mask, validate=not_blank(invalid) if invalid else None,
                               missing_message=f"{key} must be specified.")
    state.add_cluster("vsphere", cfg["name"], cfg)
    return cfg["name"]


def new_node(ctx: Context, manager: str, cluster: str, backend, state: State) -> List[str]:
    base = base_node_config(ctx, NODE_MODULE, cluster, state)
    extra: Dict = {k: state.get(f"module.{cluster}.{k}") for k in ("vsphere_user", "vsphere_password",
                                                                   "vsphere_server")}
    for k in ("vsphere_datacenter_name", "vsphere_datastore_name", "vsphere_resource_pool_name",
              "vsphere_network_name"):
        extra[k] = f"${{module.{cluster}.{k}}}"
    extra["vsphere_template_name"] = ctx.resolve("vsphere_template_name", "VM Template Name",
                                                 validate=not_blank("Invalid template name"))
    extra["ssh_user"] = ctx.resolve("ssh_user", "SSH User", validate=not_blank("Invalid SSH user"))
    extra["key_path"] = expand_home(ctx.resolve("key_path", "Private Key Path", default="~/.ssh/id_rsa",
                                                validate=file_exists()))
    for key in ("vsphere_num_cpus", "vsphere_memory_mb"):
        if ctx.is_set(key):
            extra[key] = ctx.get_string(key)
    if "vsphere_memory_mb" in extra:
        sizing.check_size("vsphere", "host", extra["vsphere_memory_mb"])
    omit_empty(extra, ["vsphere_user", "vsphere_password", "vsphere_server", "vsphere_template_name"])
    return add_nodes(state, cluster, base, extra)
