"""MI355X partition-mode policy (compute: SPX/DPX/QPX/CPX, memory: NPS1/NPS2).

An MI355X can be split into compute partitions (its 8 XCDs as 1, 2, 4 or 8 logical GPUs)
and memory partitions (its HBM as 1 or 2 NUMA pools).  Each compute partition is its own
HIP device, KFD node, render node and ``amd.com/gpu`` unit, so a node's partition modes
change what "GPU-ready" means.  The reference had no GPU notion at all; this module is the
one place the framework's rules live:

* the cluster config names the modes a node must run in (``gpu_compute_partition``,
  ``gpu_memory_partition``; default ``spx``/``nps1``), and preflight fails a node whose
  ``current_compute_partition`` / ``current_memory_partition`` (sysfs, or the labeller's
  topology document) differ -- the framework verifies, it does not repartition (that
  resets the GPUs and is the operator's call: ``amd-smi set --compute-partition``);
* readiness expects ``amd.com/gpu`` = physical GPUs x partitions per GPU, and the RCCL
  gate runs one rank per logical GPU;
* the burn-in runs on every logical GPU with its floors scaled to the partition's share
  of the chip (a CPX partition has 1/8 of the CUs), and the full memtest splits each
  memory pool between the compute partitions that share it;
* ``amd.com/xgmi.fully-connected`` is only claimed in SPX (node/labels.py): a partition
  is not a whole GPU with its own 7 links, so multi-GPU pods that need a full xGMI mesh
  (k8s/webhook.py placement) do not land on partitioned nodes.
"""

import glob
import os
from typing import Any, Dict, Optional, Tuple

from ..errors import ConfigError

COMPUTE_PARTITIONS = {"spx": 1, "dpx": 2, "qpx": 4, "cpx": 8}
MEMORY_PARTITIONS = {"nps1": 1, "nps2": 2}
DEFAULT_COMPUTE, DEFAULT_MEMORY = "spx", "nps1"


def normalize(compute: Optional[str], memory: Optional[str]) -> Tuple[str, str]:
    """Validated lower-case modes (``ConfigError`` for an unknown or impossible pair: a
    memory partition needs at least as many compute partitions)."""
    c = str(compute or DEFAULT_COMPUTE).strip().lower()
    m = str(memory or DEFAULT_MEMORY).strip().lower()
    if c not in COMPUTE_PARTITIONS:
        raise ConfigError(f"gpu_compute_partition must be one of {', '.join(COMPUTE_PARTITIONS)}. Found '{c}'.")
    if m not in MEMORY_PARTITIONS:
        raise ConfigError(f"gpu_memory_partition must be one of {', '.join(MEMORY_PARTITIONS)}. Found '{m}'.")
    if MEMORY_PARTITIONS[m] > COMPUTE_PARTITIONS[c]:
        raise ConfigError(f"gpu_memory_partition {m} needs at least {MEMORY_PARTITIONS[m]} compute partitions "
                          f"per GPU; {c} has {COMPUTE_PARTITIONS[c]}.")
    return c, m


def partitions_per_gpu(compute: Optional[str]) -> int:
    return COMPUTE_PARTITIONS[normalize(compute, None)[0]]


def modes_of(cfg: Dict[str, Any]) -> Tuple[str, str]:
    return normalize(cfg.get("gpu_compute_partition"), cfg.get("gpu_memory_partition"))


def logical_gpus(cfg: Dict[str, Any]) -> int:
    """``amd.com/gpu`` units (and RCCL ranks) a node module config implies."""
    return int(cfg.get("gpu_count", 8) or 8) * partitions_per_gpu(cfg.get("gpu_compute_partition"))


def compute_share(compute: str) -> float:
    """A compute partition's share of the chip (its CUs, its MFMA and HBM throughput)."""
    return 1.0 / COMPUTE_PARTITIONS[compute]


def memory_share(compute: str, memory: str) -> float:
    """A compute partition's share of the HBM pool it allocates from (the compute
    partitions of one memory partition share that pool)."""
    return MEMORY_PARTITIONS[memory] / COMPUTE_PARTITIONS[compute]


def topology_modes(doc: Dict[str, Any]) -> Tuple[Optional[str], Optional[str]]:
    """The node's modes from a topology document (``None`` when not reported)."""
    out = []
    for key in ("compute_partition", "memory_partition"):
        vals = {str(g.get(key, "")).lower() for g in doc.get("gpus") or [] if g.get(key)}
        out.append(vals.pop() if len(vals) == 1 else (",".join(sorted(vals)) if vals else None))
    return out[0], out[1]


def sysfs_modes(root: str = "/") -> Tuple[Optional[str], Optional[str]]:
    """Modes from ``/sys/class/drm/renderD*/device/current_{compute,memory}_partition``
    (only a GPU's first partition carries the files)."""
    out = []
    for name in ("current_compute_partition", "current_memory_partition"):
        vals = set()
        for p in glob.glob(os.path.join(root, "sys/class/drm/renderD*/device", name)):
            try:
                with open(p, "r", encoding="utf-8", errors="replace") as fh:
                    v = fh.read().strip().lower()
            except OSError:
                continue
            if v:
                vals.add(v)
        out.append(vals.pop() if len(vals) == 1 else (",".join(sorted(vals)) if vals else None))
    return out[0], out[1]


def check(want: Tuple[str, str], have: Tuple[Optional[str], Optional[str]]) -> Optional[str]:
    """Preflight verdict: None when the node runs the configured modes (a mode the node
    does not report is not held against it: older drivers lack the sysfs files)."""
    problems = []
    for what, w, h in (("compute", want[0], have[0]), ("memory", want[1], have[1])):
        if h is not None and h != w:
            problems.append(f"{what} partition is {h.upper()}, the cluster expects {w.upper()}")
    if not problems:
        return None
    return ("; ".join(problems) + " (set gpu_compute_partition / gpu_memory_partition to match, or repartition "
            "the GPUs with amd-smi before adding the node)")


def physical_count(doc: Dict[str, Any]) -> int:
    """Physical GPUs in a topology document: distinct PCI functions (a GPU's compute
    partitions share one)."""
    gpus = doc.get("gpus") or []
    return len({g.get("bdf") or f"#{i}" for i, g in enumerate(gpus)})


__all__ = ["COMPUTE_PARTITIONS", "MEMORY_PARTITIONS", "normalize", "partitions_per_gpu", "modes_of",
           "logical_gpus", "compute_share", "memory_share", "topology_modes", "sysfs_modes", "check",
           "physical_count"]
