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
"""

from typing import Any, Dict, Mapping

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
    active = [n for n in topology.get("nics", []) or [] if n.get("port", 0) > 0]
    if not active:
        return {}
    env = {"NCCL_IB_HCA": "=" + ",".join(f"{n['name']}:{n['port']}" for n in active)}
    # the RoCE v2 GID index, when every active RoCE port has it at the same index; else
    # RCCL picks one per port itself (RoCE v2, IPv4 first, by default)
    gids = {int(n.get("roce_v2_gid_index", -1)) for n in active if str(n.get("link_layer", "")).lower() == "ethernet"}
    if len(gids) == 1 and min(gids) >= 0:
        env["NCCL_IB_GID_INDEX"] = str(min(gids))
    return env


def default_rccl_env() -> Dict[str, str]:
    return dict(_DEFAULTS)


def merged_env(overrides: Mapping[str, str] = ()) -> Dict[str, str]:
    env = default_rccl_env()
    env.update({str(k): str(v) for k, v in dict(overrides).items()})
    return env


def render_env_file(env: Mapping[str, str]) -> str:
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
