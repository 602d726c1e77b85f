"""RCCL / HSA environment for MI355X worker nodes.

Written by the MI355X host bootstrap to ``/etc/rccl/rccl.env`` and injected into
GPU pods by the device-plugin / addon manifests.

Intra-node traffic on an 8xMI355X node is xGMI, point-to-point: each GPU has 7
links of roughly 153 GB/s, so ring collectives are per-link bound and RCCL
needs no socket/IB settings for it.  Inter-node traffic goes over RoCE/IB NICs
whose names are site specific: the node's active RDMA ports are discovered on the
host (:func:`site_env_from_topology`, ``amdgpu-topo-labeller --rccl-env``) and written
as ``NCCL_IB_HCA`` (+ the ports' RoCE v2 GID index, read from ``gid_attrs/types``);
``rccl_env`` overrides in the node
config win over both the defaults and the discovered values.

What the file may hold (:func:`env_problems`).  The node agent's service loads it
(``EnvironmentFile=``), the Terraform host script sources it, and the agent applies it at
start, all as root.  So whoever can put a setting into it would otherwise run code there:
``NCCL_NET_PLUGIN`` / ``NCCL_TUNER_PLUGIN`` / ``HSA_TOOLS_LIB`` / ``RCCL_ROCR_PATH`` load a
library, ``NCCL_DEBUG_FILE`` / ``HSA_COREDUMP_PATTERN`` write a path, and a value with a
newline or a quote adds lines of its own (``LD_PRELOAD=...``).  Only ``NCCL_*``, ``RCCL_*``
and ``HSA_*`` keys are accepted, none that names a library, plugin, file, path or
directory, and values are comma lists of plain tokens (an address range's ``/N`` allowed).
The same rules are the host module's ``rccl_env`` variable validation
(``terraform/generate.py``), the config check (``models/baremetal.py``) and the agent's
plan refusal (``node/agent.py``).
"""

import re
from typing import Any, Dict, List, Mapping

# Values chosen for MI355X nodes; every one can be overridden per node.
_DEFAULTS: Dict[str, str] = {
    # fine-grained host memory for RCCL's proxy/host buffers over PCIe
    "HSA_FORCE_FINE_GRAIN_PCIE": "1",
    # do not reclaim scratch between kernels (avoids allocator churn in
    # collective-heavy training loops)
    "HSA_NO_SCRATCH_RECLAIM": "1",
    # legacy IPC mode off: RCCL / tensor sharing across processes uses dmabuf
    "HSA_ENABLE_IPC_MODE_LEGACY": "0",
    "NCCL_DEBUG": "WARN",
    # keep collectives on the xGMI fabric inside a node
    "NCCL_P2P_LEVEL": "SYS",
}

SITE_KEYS = ("NCCL_SOCKET_IFNAME", "NCCL_IB_HCA", "NCCL_IB_GID_INDEX", "NCCL_NET_GDR_LEVEL")


def site_env_from_topology(topology: Mapping[str, Any]) -> Dict[str, str]:
    """Inter-node settings derived from the node's RDMA NICs (``topology["nics"]``, as
    discovered by the labeller): every active port in ``NCCL_IB_HCA`` (exact names), and
    the RoCE v2 GID index the Ethernet ports share (``roce_v2_gid_index``).  Mirror of
    ``csrc/tk_topo.cpp:render_rccl_env``; explicit per-node ``rccl_env`` keys override it."""
    # a port whose name is not a plain device name (sysfs gives mlx5_0, bnxt_re1, irdma0, ...)
    # is left to RCCL's own detection rather than written into a file loaded as root
    active = [n for n in topology.get("nics", []) or [] if int(n.get("port", 0) or 0) > 0
              and re.fullmatch(r"[A-Za-z0-9_.-]{1,64}", str(n.get("name", "")))]
    if not active:
        return {}
    env = {"NCCL_IB_HCA": "=" + ",".join(f"{n['name']}:{n['port']}" for n in active)}
    # the RoCE v2 GID index, when every active RoCE port has it at the same index; else
    # RCCL picks one per port itself (RoCE v2, IPv4 first, by default)
    gids = {int(n.get("roce_v2_gid_index", -1)) for n in active if str(n.get("link_layer", "")).lower() == "ethernet"}
    if len(gids) == 1 and min(gids) >= 0:
        env["NCCL_IB_GID_INDEX"] = str(min(gids))
    return env


# RE2-compatible (Terraform's regexall uses the same strings)
ENV_KEY_RE = "^(NCCL|RCCL|HSA)_[A-Z0-9_]+$"
ENV_KEY_DENY_RE = "(^|_)(PLUGIN|LIB|TOOLS|PATTERN|CONF|SCRIPT|DIR|PATH|[A-Z]*FILE)(_|$)"
ENV_ITEM_RE = "^[A-Za-z0-9_.:=^+-]*(/[0-9]{1,3})?$"
ENV_VALUE_MAX = 256


def env_problems(env: Any) -> List[str]:
    """Why ``env`` may not be a node's RCCL environment (empty: it may).  See the module
    docstring."""
    if not isinstance(env, Mapping):
        return ["rccl_env must be a map of NCCL_*, RCCL_* and HSA_* settings"]
    out = []
    for k, v in env.items():
        k, v = str(k), str(v)
        if not re.fullmatch(ENV_KEY_RE, k):
            out.append(f"rccl_env key {k[:64]!r}: only NCCL_*, RCCL_* and HSA_* settings (upper case) are accepted")
            continue
        if re.search(ENV_KEY_DENY_RE, k):
            out.append(f"rccl_env key {k}: names a library, plugin, file or path, which the node's RCCL "
                       "environment does not accept (the node agent's service loads it as root)")
        if len(v) > ENV_VALUE_MAX or not all(re.fullmatch(ENV_ITEM_RE, item) for item in v.split(",")):
            out.append(f"rccl_env {k}: value {v[:48]!r} may hold only a comma list of letters, digits and "
                       f"_ . : = ^ + - (an address range's /N allowed), at most {ENV_VALUE_MAX} characters")
    return out


def check_env(env: Mapping[str, Any]) -> None:
    bad = env_problems(env)
    if bad:
        raise ValueError("; ".join(bad))


def default_rccl_env() -> Dict[str, str]:
    return dict(_DEFAULTS)


def render_env_file(env: Mapping[str, str]) -> str:
    check_env(env)  # no writer can emit a setting, or a line, the file may not hold
    lines = ["# RCCL / HSA environment for MI355X (written by triton-kubernetes)"]
    for k in sorted(env):
        v = str(env[k]).replace('"', '\\"')
        lines.append(f'{k}="{v}"')
    return "\n".join(lines) + "\n"


def parse_env_file(text: str) -> Dict[str, str]:
    out: Dict[str, str] = {}
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith("#") or "=" not in line:
            continue
        k, _, v = line.partition("=")
        v = v.strip()
        if len(v) >= 2 and v[0] == v[-1] == '"':
            v = v[1:-1].replace('\\"', '"')
        out[k.strip()] = v
    return out
