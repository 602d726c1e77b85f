"""Triton provider: manager (C18), cluster (C24), node (C31).

Reference: ``create/manager_triton.go:24-399``, ``create/cluster_triton.go:15-140``,
``create/node_triton.go:22-318``.  CloudAPI listings validate networks,
image name@version and packages; nodes reuse the cluster's credentials by
value (``node_triton.go:56-61``).  Deliberate fix: node image / package are
validated like the manager's (reference TODOs at ``node_triton.go:185,251``).
"""

from typing import Dict, List, Optional

from ..backend.select import resolve_triton_key_id
from ..config.context import Context, expand_home, file_exists, not_blank
from .. import sizing
from ..errors import ConfigError
from ..state import State
from .cloudctx import cloud, validation_enabled
from .common import add_nodes, base_cluster_config, base_manager_config, base_node_config, omit_empty

MANAGER_MODULE = "terraform/modules/triton-rancher"
CLUSTER_MODULE = "terraform/modules/triton-rancher-k8s"
NODE_MODULE = "terraform/modules/triton-rancher-k8s-host"
DEFAULT_URL = "https://us-east-1.api.joyent.com"


def credentials(ctx: Context) -> Dict[str, str]:
    account = ctx.resolve("triton_account", "Triton Account Name", validate=not_blank("Invalid Triton Account"))
    raw_path = ctx.resolve("triton_key_path", "Triton Key Path", default="~/.ssh/id_rsa", validate=file_exists())
    key_path = expand_home(raw_path)
    key_id = resolve_triton_key_id(ctx, key_path)
    url = ctx.resolve("triton_url", "Triton URL", default=DEFAULT_URL)
    return {"triton_account": account, "triton_key_path": key_path, "triton_key_id": key_id, "triton_url": url}


def _api(ctx: Context, creds: Dict[str, str]):
    return cloud(ctx).triton(creds["triton_account"], creds["triton_key_path"], creds["triton_key_id"],
                             creds["triton_url"])


def _networks(ctx: Context, api) -> List[str]:
    valid = [n.name for n in api.networks()] if api is not None else None
    if ctx.is_set("triton_network_names"):
        chosen = ctx.settings.get_string_slice("triton_network_names")
        if valid is not None:
            for net in chosen:
                if net not in valid:
                    raise ConfigError(
                        f"Invalid Triton Network '{net}', must be one of the following: {', '.join(valid)}")
        return chosen
    if ctx.non_interactive:
        raise ConfigError("triton_network_names must be specified")
    if valid is None:
        return ctx.settings.get_string_slice("triton_network_names") or [
            ctx.prompter.prompt("Triton Networks to attach (space separated)")]
    return ctx.resolve_list("triton_network_names", "Triton Networks to attach", valid)


def _image(ctx: Context, api) -> Dict[str, str]:
    images = api.images() if api is not None else None
    if ctx.is_set("triton_image_name") and ctx.is_set("triton_image_version"):
        name, version = ctx.get_string("triton_image_name"), ctx.get_string("triton_image_version")
        if images is not None and not any(i.name == name and i.version == version for i in images):
            raise ConfigError(f"Invalid Triton Image Name and Version '{name}@{version}'")
        return {"triton_image_name": name, "triton_image_version": version}
    if ctx.non_interactive:
        raise ConfigError("Both triton_image_name and triton_image_version must be specified")
    if not images:
        name = ctx.prompter.prompt("Triton Image Name")
        return {"triton_image_name": name, "triton_image_version": ctx.prompter.prompt("Triton Image Version")}
    idx, _ = ctx.prompter.select("Triton Image to use", [f"{i.name}@{i.version}" for i in images], searchable=True)
    return {"triton_image_name": images[idx].name, "triton_image_version": images[idx].version}


def _package(ctx: Context, api, key: str, label: str, invalid: str) -> str:
    packages = api.packages() if api is not None else None
    kind = "manager" if key.startswith("master_") else "host"
    if ctx.is_set(key):
        value = ctx.get_string(key)
        if packages is not None and not any(p.name == value for p in packages):
            raise ConfigError(f"{invalid} '{value}'")
    elif ctx.non_interactive:
        raise ConfigError(f"{key} must be specified")
    elif not packages:
        value = ctx.prompter.prompt(label, default=sizing.default_size("triton", kind)[1])
    else:
        _, value = ctx.prompter.select(label, [p.name for p in packages], searchable=True)
    # the package listing knows the memory (MB); otherwise the known sizes table
    mem = next((p.memory / 1024.0 for p in packages or [] if p.name == value and p.memory), None)
    sizing.check_size("triton", kind, value, mem)
    return value


def _machine_fields(ctx: Context, api, package_key: str, package_label: str, invalid: str) -> Dict:
    out: Dict = {"triton_network_names": _networks(ctx, api)}
    out.update(_image(ctx, api))
    out["triton_ssh_user"] = ctx.resolve("triton_ssh_user", "Triton SSH User", default="ubuntu")
    out[package_key] = _package(ctx, api, package_key, package_label, invalid)
    return out


def new_manager(ctx: Context, state: State, name: str) -> None:
    cfg = base_manager_config(ctx, MANAGER_MODULE, name)
    cfg.update(credentials(ctx))
    api = _api(ctx, cfg) if validation_enabled(ctx) else None
    cfg.update(_machine_fields(ctx, api, "master_triton_machine_package",
                               "Triton Machine Package to use for Rancher Master",
                               "Invalid Master Triton Machine Package"))
    state.set_manager(omit_empty(cfg, ["triton_url", "triton_network_names", "triton_image_name",
                                       "triton_image_version", "triton_ssh_user", "master_triton_machine_package"]))


def new_cluster(ctx: Context, backend, state: State) -> str:
    cfg = base_cluster_config(ctx, CLUSTER_MODULE)
    cfg.update(credentials(ctx))
    state.add_cluster("triton", cfg["name"], omit_empty(cfg, ["triton_url"]))
    return cfg["name"]


def new_node(ctx: Context, manager: str, cluster: str, backend, state: State,
             api: Optional[object] = None) -> List[str]:
    base = base_node_config(ctx, NODE_MODULE, cluster, state)
    creds = {k: state.get(f"module.{cluster}.{k}") for k in
             ("triton_account", "triton_key_path", "triton_key_id", "triton_url")}
    if api is None and validation_enabled(ctx):
        api = _api(ctx, creds)
    extra: Dict = dict(creds)
    extra.update(_machine_fields(ctx, api, "triton_machine_package", "Triton Machine Package to use for node",
                                 "Invalid Triton Machine Package"))
    omit_empty(extra, ["triton_url", "triton_network_names", "triton_image_name", "triton_image_version",
                       "triton_ssh_user", "triton_machine_package"])
    return add_nodes(state, cluster, base, extra)
