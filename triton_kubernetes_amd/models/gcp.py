"""GCP provider: manager (C20), cluster (C26), node (C33).

Reference: ``create/manager_gcp.go:21-422``, ``create/cluster_gcp.go:22-168``,
``create/node_gcp.go:20-377``.  ``gcp_project_id`` is read from the credentials
JSON; region / zone (filtered by region) / machine type / image are validated
against Compute listings.  Node disks: the reference emits ``gcp_disk_*`` as
empty strings (its prompts are commented out, ``node_gcp.go:241-342``); we
accept them from config (``gcp_disk_type/size/mount_path``) and the rewritten
host module attaches the disk.
"""

from typing import Dict, List, Optional

from ..config.context import Context, expand_home, file_exists
from .. import sizing
from ..errors import ConfigError
from ..state import State
from ..cloud.gcp import project_id_from_credentials
from .cloudctx import cloud, validation_enabled
from .common import add_nodes, base_cluster_config, base_manager_config, base_node_config

MANAGER_MODULE = "terraform/modules/gcp-rancher"
CLUSTER_MODULE = "terraform/modules/gcp-rancher-k8s"
NODE_MODULE = "terraform/modules/gcp-rancher-k8s-host"
GCP_DISK_TYPES = ["pd-standard", "pd-ssd"]


def _credentials(ctx: Context) -> Dict[str, str]:
    raw = ctx.resolve("gcp_path_to_credentials", "Path to Google Cloud Platform Credentials File",
                      validate=file_exists())
    path = expand_home(raw)
    return {"gcp_path_to_credentials": path, "gcp_project_id": project_id_from_credentials(path)}


def _api(ctx: Context, creds: Dict[str, str]):
    if not validation_enabled(ctx):
        return None
    return cloud(ctx).gcp(creds["gcp_path_to_credentials"])


def _pick(ctx: Context, key: str, label: str, items: Optional[List[str]], what: str) -> str:
    if ctx.is_set(key):
        value = ctx.get_string(key)
        if items is not None and value not in items:
            raise ConfigError(f"Selected GCP {what} '{value}' does not exist.")
        return value
    if ctx.non_interactive:
        raise ConfigError(f"{key} must be specified")
    if not items:
        return ctx.prompter.prompt(label)
    _, value = ctx.prompter.select(label, items, searchable=True)
    return value


def _region(ctx: Context, api) -> str:
    return _pick(ctx, "gcp_compute_region", "GCP Compute Region", api.regions() if api else None,
                 "Compute Region")


def _instance(ctx: Context, api, region: str, kind: str) -> Dict[str, str]:
    zone = _pick(ctx, "gcp_instance_zone", "GCP Instance Zone", api.zones(region) if api else None,
                 "Instance Zone")
    mtype = _pick(ctx, "gcp_machine_type", "GCP Machine Type", api.machine_types(zone) if api else None,
                  "Machine Type")
    sizing.check_size("gcp", kind, mtype)
    image = _pick(ctx, "gcp_image", "GCP Image", [i.name for i in api.images()] if api else None, "Image")
    return {"gcp_machine_type": mtype, "gcp_instance_zone": zone, "gcp_image": image}


def new_manager(ctx: Context, state: State, name: str) -> None:
    cfg = base_manager_config(ctx, MANAGER_MODULE, name)
    creds = _credentials(ctx)
    api = _api(ctx, creds)
    region = _region(ctx, api)
    inst = _instance(ctx, api, region, "manager")
    pub = ctx.resolve("gcp_public_key_path", "GCP Public Key Path", default="~/.ssh/id_rsa.pub",
                      validate=file_exists())
    priv = ctx.resolve("gcp_private_key_path", "GCP Private Key Path", default="~/.ssh/id_rsa",
                       validate=file_exists())
    user = ctx.resolve("gcp_ssh_user", "GCP SSH User", default="ubuntu")
    cfg.update(creds)
    cfg["gcp_compute_region"] = region
    cfg.update(inst)
    cfg.update({"gcp_public_key_path": expand_home(pub), "gcp_private_key_path": expand_home(priv),
                "gcp_ssh_user": user})
    state.set_manager(cfg)


def new_cluster(ctx: Context, backend, state: State) -> str:
    cfg = base_cluster_config(ctx, CLUSTER_MODULE)
    creds = _credentials(ctx)
    cfg.update(creds)
    cfg["gcp_compute_region"] = _region(ctx, _api(ctx, creds))
    state.add_cluster("gcp", cfg["name"], cfg)
    return cfg["name"]


def _disk(ctx: Context) -> Dict[str, str]:
    s = ctx.settings
    out = {"gcp_disk_type": "", "gcp_disk_size": "", "gcp_disk_mount_path": ""}
    if s.is_set("gcp_disk_type"):
        if not (s.is_set("gcp_disk_size") and s.is_set("gcp_disk_mount_path")):
            raise ConfigError("If gcp_disk_type is set, gcp_disk_size and gcp_disk_mount_path must also be set.")
        out["gcp_disk_type"] = s.get_string("gcp_disk_type")
        if out["gcp_disk_type"] not in GCP_DISK_TYPES:
            raise ConfigError(f"gcp_disk_type must be valid. Found '{out['gcp_disk_type']}'.")
        out["gcp_disk_size"] = s.get_string("gcp_disk_size")
        out["gcp_disk_mount_path"] = s.get_string("gcp_disk_mount_path")
    return out


def new_node(ctx: Context, manager: str, cluster: str, backend, state: State) -> List[str]:
    base = base_node_config(ctx, NODE_MODULE, cluster, state)
    creds = {k: state.get(f"module.{cluster}.{k}") for k in
             ("gcp_path_to_credentials", "gcp_project_id", "gcp_compute_region")}
    api = _api(ctx, creds)
    extra: Dict = dict(creds)
    extra.update({
        "gcp_compute_network_name": f"${{module.{cluster}.gcp_compute_network_name}}",
        "gcp_compute_firewall_host_tag": f"${{module.{cluster}.gcp_compute_firewall_host_tag}}",
    })
    extra.update(_instance(ctx, api, creds["gcp_compute_region"], "host"))
    extra.update(_disk(ctx))
    return add_nodes(state, cluster, base, extra)
