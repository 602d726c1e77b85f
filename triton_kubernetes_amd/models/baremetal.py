"""Bare-metal provider: manager, cluster and node (+ the MI355X node variant).

Reference: ``create/manager_bare_metal.go:14-150`` (C22),
``create/cluster_bare_metal.go:8-36`` (C28), ``create/node_bare_metal.go:16-181`` (C35).

MI355X additions (BASELINE.json north star):

* ``gpu: mi355x`` on a node selects ``bare-metal-mi355x-rancher-k8s-host``: the
  host bootstrap runs a ROCm/amdgpu preflight, passes ``/dev/kfd`` and
  ``/dev/dri`` to the container runtime, runs the native topology labeller (N1)
  to derive ``amd.com/*`` node labels (incl. the xGMI hive id used for pod
  affinity), writes the RCCL environment file and runs the GPU burn-in probes;
* ``gpu_addons: true`` on the cluster adds ``addons_baremetal_<name>``
  (``rancher-k8s-mi355x-addons``): ROCm device plugin + labeller DaemonSets and
  the RCCL readiness Job, applied once the cluster is active.
"""

import math
from typing import Dict, List

from ..config.context import Context, file_exists, not_blank
from ..errors import ConfigError
from ..state import MANAGER_KEY, State, cluster_key_parts
from .. import versions
from ..parallel.rccl_env import default_rccl_env, env_problems
from .common import add_nodes, base_cluster_config, base_manager_config, base_node_config, omit_empty, source_for

MANAGER_MODULE = "terraform/modules/bare-metal-rancher"
CLUSTER_MODULE = "terraform/modules/bare-metal-rancher-k8s"
NODE_MODULE = "terraform/modules/bare-metal-rancher-k8s-host"
MI355X_NODE_MODULE = "terraform/modules/bare-metal-mi355x-rancher-k8s-host"
ADDONS_MODULE = "terraform/modules/rancher-k8s-mi355x-addons"

GPU_TYPES = ["none", "mi355x"]
BURNIN_LEVELS = ["quick", "full", "off"]
DEFAULT_BURNIN = "full"


def addons_key(cluster_name: str) -> str:
    return f"addons_baremetal_{cluster_name}"


def _ssh_fields(ctx: Context) -> Dict[str, str]:
    ssh_user = ctx.resolve("ssh_user", "SSH User", default="ubuntu", validate=not_blank("Invalid SSH User"))
    bastion = ctx.resolve("bastion_host", "Bastion Host", none_sentinel="None",
                          validate=not_blank("Invalid Bastion Host"))
    key_path = ctx.resolve("key_path", "Key Path", default="~/.ssh/id_rsa", validate=file_exists())
    return {"ssh_user": ssh_user, "bastion_host": bastion, "key_path": key_path}


def new_manager(ctx: Context, state: State, name: str) -> None:
    cfg = base_manager_config(ctx, MANAGER_MODULE, name)
    cfg["host"] = ctx.resolve("host", "Host/IP for cluster manager", validate=not_blank("Invalid host/ip"))
    ssh = _ssh_fields(ctx)
    cfg["bastion_host"] = ssh["bastion_host"]
    cfg["ssh_user"] = ssh["ssh_user"]
    cfg["key_path"] = ssh["key_path"]
    # key order of bareMetalManagerTerraformConfig: host, bastion_host, ssh_user, key_path
    state.set_manager(omit_empty(cfg, ["bastion_host", "ssh_user", "key_path"]))


def new_cluster(ctx: Context, backend, state: State) -> str:
    cfg = base_cluster_config(ctx, CLUSTER_MODULE)
    name = cfg["name"]
    key = state.add_cluster("baremetal", name, cfg)
    if ctx.settings.get_bool("gpu_addons"):
        add_mi355x_addons(ctx, state, key, name)
    return name


def add_mi355x_addons(ctx: Context, state: State, cluster: str, name: str) -> str:
    s = ctx.settings
    addon = {
        "source": source_for(ctx, ADDONS_MODULE),
        "name": name,
        "rancher_api_url": f"${{module.{MANAGER_KEY}.rancher_url}}",
        "rancher_access_key": f"${{module.{MANAGER_KEY}.rancher_access_key}}",
        "rancher_secret_key": f"${{module.{MANAGER_KEY}.rancher_secret_key}}",
        "rancher_cluster_id": f"${{module.{cluster}.rancher_cluster_id}}",
        # pinned tags (versions.py), never :latest
        "device_plugin_image": s.get_string("device_plugin_image") or versions.DEVICE_PLUGIN_IMAGE,
        # opt-in: the bootstrap labeller owns amd.com/gpu.* (k8s/manifests.py:ROCM_LABELLER_ARGS)
        "node_labeller_image": s.get_string("node_labeller_image") if s.is_set("node_labeller_image") else "",
        "rccl_probe_image": s.get_string("rccl_probe_image") or versions.RCCL_PROBE_IMAGE,
        "webhook_image": s.get_string("webhook_image") or versions.WEBHOOK_IMAGE,
        "rccl_gate": "true" if s.get_bool("rccl_gate") or not s.is_set("rccl_gate") else "false",
        "rccl_env_injector": ("true" if not s.is_set("rccl_env_injector") or s.get_bool("rccl_env_injector")
                              else "false"),
    }
    key = addons_key(name)
    state.set_module(key, addon)
    return key


def _gpu_type(ctx: Context) -> str:
    if ctx.is_set("gpu"):
        value = ctx.get_string("gpu").lower()
    elif ctx.non_interactive:
        value = "none"
    else:
        _, value = ctx.prompter.select("Node GPU type", ["None", "MI355X"])
        value = value.lower()
    if value in ("", "false", "no"):
        value = "none"
    if value not in GPU_TYPES:
        raise ConfigError(f"Invalid gpu '{value}', must be one of the following: none, mi355x")
    return value


def new_node(ctx: Context, manager: str, cluster: str, backend, state: State) -> List[str]:
    cluster_key_parts(cluster)
    gpu = _gpu_type(ctx)
    module = MI355X_NODE_MODULE if gpu == "mi355x" else NODE_MODULE
    base = base_node_config(ctx, module, cluster, state)
    ssh = _ssh_fields(ctx)
    extra: Dict = {
        "host": "",
        "bastion_host": ssh["bastion_host"],
        "ssh_user": ssh["ssh_user"],
        "key_path": ssh["key_path"],
    }
    if ctx.is_set("node_cleanup"):
        # the host module's destroy-time teardown (node/cleanup.py); unset: the module's default (on)
        extra["node_cleanup"] = ctx.settings.get_bool("node_cleanup")
    if gpu == "mi355x":
        extra.update(_mi355x_fields(ctx))

    existing = list(state.nodes(cluster).keys())
    from .common import new_hostnames

    names = new_hostnames(existing, base.hostname, base.count)
    if ctx.is_set("hosts"):
        hosts = ctx.settings.get_string_slice("hosts")
    elif ctx.non_interactive:
        raise ConfigError("hosts must be specified")
    else:
        hosts = [ctx.prompter.prompt(f"Host/IP for {n}", validate=not_blank("Invalid host/ip")) for n in names]
    if len(hosts) != base.count:
        raise ConfigError("not enough hosts")
    return add_nodes(state, cluster, base, extra, per_node=[{"host": h} for h in hosts])


def _plain_number(text: str, message: str, hi: float = math.inf) -> str:
    """A finite number in [0, hi], written plainly ("38", "0.5", "1000" for "1e3"): the form
    the host module's validation accepts and its script passes to the node tools."""
    try:
        v = float(text)
        if not (math.isfinite(v) and 0.0 <= v <= hi):
            raise ValueError
    except ValueError as exc:
        raise ConfigError(f"{message}. Found '{text}'.") from exc
    out = f"{v:.6f}".rstrip("0").rstrip(".")
    return out or "0"


def _mi355x_fields(ctx: Context) -> Dict:
    s = ctx.settings
    count = s.get_string("gpu_count") if s.is_set("gpu_count") else (
        "8" if ctx.non_interactive else ctx.prompter.prompt("Expected GPUs per node", default="8"))
    try:
        if int(count) <= 0:
            raise ValueError
    except ValueError as exc:
        raise ConfigError(f"gpu_count must be greater than 0. Found '{count}'.") from exc
    # full by default: a node entering a training fleet gets every free byte of its HBM
    # memtested (~4-6 s per GPU, all GPUs at once), not the 1 GiB token check of quick
    burnin = s.get_string("gpu_burnin").lower() if s.is_set("gpu_burnin") else DEFAULT_BURNIN
    if burnin not in BURNIN_LEVELS:
        raise ConfigError(f"Invalid gpu_burnin '{burnin}', must be one of the following: quick, full, off")
    env = default_rccl_env()
    overrides = s.get("rccl_env")
    if s.is_set("rccl_env") and not isinstance(overrides, dict):
        raise ConfigError("rccl_env must be a map of NCCL_*, RCCL_* and HSA_* settings.")
    if isinstance(overrides, dict):
        bad = env_problems(overrides)
        if bad:
            raise ConfigError(f"Invalid {bad[0]}.")
        env.update({str(k): str(v) for k, v in overrides.items()})
    out = {
        "gpu_product": "MI355X",
        "gpu_count": str(int(count)),
        "gpu_burnin": burnin,
        "rccl_env": env,
    }
    if s.is_set("rccl_min_busbw"):
        out["rccl_min_busbw"] = _plain_number(s.get_string("rccl_min_busbw"),
                                              "rccl_min_busbw must be a non-negative number")
    if s.is_set("gpu_link_min_frac"):
        out["gpu_link_min_frac"] = _plain_number(s.get_string("gpu_link_min_frac"),
                                                 "gpu_link_min_frac must be a number between 0 and 1", hi=1.0)
    if s.is_set("gpu_compute_partition") or s.is_set("gpu_memory_partition"):
        from ..node.partition import normalize

        c, m = normalize(s.get_string("gpu_compute_partition") or None, s.get_string("gpu_memory_partition") or None)
        out["gpu_compute_partition"], out["gpu_memory_partition"] = c, m
    if s.is_set("gpu_link_min_gbps"):
        out["gpu_link_min_gbps"] = _plain_number(s.get_string("gpu_link_min_gbps"),
                                                 "gpu_link_min_gbps must be a non-negative number")
    # GPU health policy at bring-up (node/health.py): fail | taint | off, and its limits
    from ..node.health import limits_of, policy_of

    raw = {k: s.get_string(k) for k in ("gpu_health", "gpu_max_uncorrectable_ecc", "gpu_max_retired_pages")
           if s.is_set(k)}
    if raw:
        policy = policy_of(raw)
        max_ue, max_bad = limits_of(raw)
        out["gpu_health"] = policy
        out["gpu_max_uncorrectable_ecc"] = str(max_ue)
        out["gpu_max_retired_pages"] = "auto" if max_bad < 0 else str(max_bad)
    if s.is_set("gpu_metrics_textfile"):  # node_exporter textfile (node/metrics.py)
        from ..node.metrics import textfile_dir_of

        out["gpu_metrics_textfile"] = textfile_dir_of({"gpu_metrics_textfile": s.get_string("gpu_metrics_textfile")})
    if s.is_set("gpu_host_tuning"):  # NUMA balancing / IOMMU checks (node/hosttune.py)
        from ..node.hosttune import policy_of as tuning_policy

        out["gpu_host_tuning"] = tuning_policy({"gpu_host_tuning": s.get_string("gpu_host_tuning")})
    if s.is_set("rccl_slim"):  # opt-in verified single-target RCCL (terraform/scripts.py)
        slim = s.get_string("rccl_slim").lower()
        if slim in ("true", "yes", "1"):
            slim = "on"
        if slim in ("false", "no", "0"):
            slim = "off"
        if slim not in ("on", "off"):
            raise ConfigError(f"rccl_slim must be on or off. Found '{slim}'.")
        out["rccl_slim"] = slim
    return out
