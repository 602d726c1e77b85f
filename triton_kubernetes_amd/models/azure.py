"""Azure provider: manager (C21), cluster (C27), node (C34).

Reference: ``create/manager_azure.go:21-437``, ``create/cluster_azure.go:19-250``,
``create/node_azure.go:23-314``.  Service-principal credentials, environment in
{public, government, german, china}, location and VM size validated against
ARM listings.  ``azure_resource_group_name`` is emitted empty for the manager
(never prompted in the reference) and the image fields are omitted.
"""

from typing import Dict, List, Optional

from ..cloud.azure import ENVIRONMENTS
from ..config.context import Context, expand_home, file_exists, not_blank
from .. import sizing
from ..errors import ConfigError
from ..state import State
from .cloudctx import cloud, validation_enabled
from .common import add_nodes, base_cluster_config, base_manager_config, base_node_config, positive_int

MANAGER_MODULE = "terraform/modules/azure-rancher"
CLUSTER_MODULE = "terraform/modules/azure-rancher-k8s"
NODE_MODULE = "terraform/modules/azure-rancher-k8s-host"
AZURE_ENVIRONMENTS = ["public", "government", "german", "china"]


def _creds(ctx: Context) -> Dict[str, str]:
    out = {
        "azure_subscription_id": ctx.resolve("azure_subscription_id", "Azure Subscription ID",
                                             validate=not_blank("Invalid Azure Subscription ID")),
        "azure_client_id": ctx.resolve("azure_client_id", "Azure Client ID",
                                       validate=not_blank("Invalid Azure Client ID")),
        "azure_client_secret": ctx.resolve("azure_client_secret", "Azure Client Secret", mask=True,
                                           validate=not_blank("Invalid Azure Client Secret")),
        "azure_tenant_id": ctx.resolve("azure_tenant_id", "Azure Tenant ID",
                                       validate=not_blank("Invalid Azure Tenant ID")),
    }
    env = ctx.resolve_choice("azure_environment", "Azure Environment", AZURE_ENVIRONMENTS)
    if env not in ENVIRONMENTS:
        raise ConfigError(f"Invalid azure_environment '{env}', must be one of the following: "
                          "'public', 'government', 'german', or 'china'")
    out["azure_environment"] = env
    return out


def _api(ctx: Context, creds: Dict[str, str]):
    if not validation_enabled(ctx):
        return None
    return cloud(ctx).azure(creds["azure_subscription_id"], creds["azure_client_id"],
                            creds["azure_client_secret"], creds["azure_tenant_id"], creds["azure_environment"])


def _validated(ctx: Context, key: str, label: str, items: Optional[List[str]]) -> str:
    if ctx.is_set(key):
        value = ctx.get_string(key)
        if items is not None and value not in items:
            raise ConfigError(f"Invalid {key} '{value}', must be one of the following: {', '.join(items)}")
        return value
    if ctx.non_interactive:
        raise ConfigError(f"{key} must be specified")
    if not items:
        return ctx.prompter.prompt(label)
    _, value = ctx.prompter.select(label, items, searchable=True)
    return value


def _location(ctx: Context, api) -> str:
    return _validated(ctx, "azure_location", "Azure Location", api.locations() if api else None)


def _size(ctx: Context, api, location: str, kind: str) -> str:
    value = _validated(ctx, "azure_size", "Azure Size", api.vm_sizes(location) if api else None)
    sizing.check_size("azure", kind, value)
    return value


def _ssh(ctx: Context, with_private: bool) -> Dict[str, str]:
    out = {"azure_ssh_user": ctx.resolve("azure_ssh_user", "Azure SSH User", default="ubuntu")}
    out["azure_public_key_path"] = expand_home(ctx.resolve(
        "azure_public_key_path", "Azure Public Key Path", default="~/.ssh/id_rsa.pub", validate=file_exists()))
    if with_private:
        out["azure_private_key_path"] = expand_home(ctx.resolve(
            "azure_private_key_path", "Azure Private Key Path", default="~/.ssh/id_rsa", validate=file_exists()))
    return out


def new_manager(ctx: Context, state: State, name: str) -> None:
    cfg = base_manager_config(ctx, MANAGER_MODULE, name)
    creds = _creds(ctx)
    api = _api(ctx, creds)
    location = _location(ctx, api)
    size = _size(ctx, api, location, "manager")
    ssh = _ssh(ctx, with_private=True)
    cfg.update(creds)
    cfg.update({"azure_location": location, "azure_resource_group_name": "", "azure_size": size})
    cfg.update(ssh)
    state.set_manager(cfg)


def new_cluster(ctx: Context, backend, state: State) -> str:
    cfg = base_cluster_config(ctx, CLUSTER_MODULE)
    creds = _creds(ctx)
    cfg.update(creds)
    cfg["azure_location"] = _location(ctx, _api(ctx, creds))
    state.add_cluster("azure", cfg["name"], cfg)
    return cfg["name"]


def _disk(ctx: Context) -> Dict[str, str]:
    s = ctx.settings
    out = {"azure_disk_mount_path": "", "azure_disk_size": ""}
    mount_set, size_set = s.is_set("azure_disk_mount_path"), s.is_set("azure_disk_size")
    if ctx.non_interactive:
        if mount_set and not size_set:
            raise ConfigError("If azure_disk_mount_path is set, then azure_disk_size must also be set.")
        if mount_set:
            out["azure_disk_mount_path"] = s.get_string("azure_disk_mount_path")
            out["azure_disk_size"] = s.get_string("azure_disk_size")
        return out
    if not ctx.prompter.confirm("Create a disk for this node", "Disk created"):
        return out
    out["azure_disk_mount_path"] = s.get_string("azure_disk_mount_path") if mount_set else \
        ctx.prompter.prompt("Azure Disk Mount Path")
    out["azure_disk_size"] = s.get_string("azure_disk_size") if size_set else \
        ctx.prompter.prompt("Azure Disk Size in GB", validate=positive_int)
    return out


def new_node(ctx: Context, manager: str, cluster: str, backend, state: State) -> List[str]:
    base = base_node_config(ctx, NODE_MODULE, cluster, state)
    creds = {k: state.get(f"module.{cluster}.{k}") for k in
             ("azure_subscription_id", "azure_client_id", "azure_client_secret", "azure_tenant_id",
              "azure_environment", "azure_location")}
    api = _api(ctx, creds) if creds["azure_environment"] in ENVIRONMENTS else None
    extra: Dict = dict(creds)
    extra.update({
        "azure_resource_group_name": f"${{module.{cluster}.azure_resource_group_name}}",
        "azure_network_security_group_id": f"${{module.{cluster}.azure_network_security_group_id}}",
        "azure_subnet_id": f"${{module.{cluster}.azure_subnet_id}}",
        "azure_size": _size(ctx, api, creds["azure_location"], "host"),
    })
    extra.update(_ssh(ctx, with_private=False))
    extra.update(_disk(ctx))
    return add_nodes(state, cluster, base, extra)
