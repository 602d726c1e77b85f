"""RCCL / HSA environment for MI355X worker nodes.

Written by the MI355X host bootstrap to ``/etc/rccl/rccl.env`` and injected into
GPU pods by the device-plugin / addon manifests.

Intra-node traffic on an 8xMI355X node is xGMI, point-to-point: each GPU has 7
links of roughly 153 GB/s, so ring collectives are per-link bound and RCCL
needs no socket/IB settings for it.  Inter-node traffic goes over RoCE/IB NICs
whose names are site specific: ``NCCL_SOCKET_IFNAME`` / ``NCCL_IB_HCA`` are only
written when configured (``rccl_env`` overrides in the node config).
"""

from typing import Dict, Mapping

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
