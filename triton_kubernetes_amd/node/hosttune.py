"""MI355X host settings checked at bring-up (``gpu_preflight``).

Two host-wide kernel settings bound what an 8xMI355X node delivers to multi-GPU and
multi-node jobs, and both are invisible to the GPU burn-in:

* **NUMA auto-balancing** (``/proc/sys/kernel/numa_balancing``): the kernel unmaps and
  migrates pages it sees accessed from a remote NUMA node.  Host buffers that GPUs map
  (RCCL's proxy and host staging buffers, pinned dataloader memory) get those faults and
  moves; AMD's Instinct system-tuning guidance is to turn it off (``0``);
* **IOMMU mode** (``/proc/cmdline``, ``/sys/class/iommu``): with the IOMMU translating
  DMA, GPU peer-to-peer and GPUDirect-RDMA traffic pays an IOTLB lookup per page; the
  guidance is passthrough (``iommu=pt``), which keeps device isolation for VFIO users.

Policy ``gpu_host_tuning``: ``warn`` (default) records the facts as node labels
(``amd.com/host.numa-balancing``, ``amd.com/host.iommu``) and the problems as warnings in
the step result; ``enforce`` fails the node's preflight; ``off`` skips the check.  The
shell twin for SSH / Terraform nodes is :func:`shell_check` (same facts, same labels).
"""

import os
from typing import Callable, Dict, List, Optional

from ..errors import ConfigError

POLICIES = ("warn", "enforce", "off")


def policy_of(cfg: Dict) -> str:
    p = str(cfg.get("gpu_host_tuning") or "warn").lower()
    if p not in POLICIES:
        raise ConfigError(f"gpu_host_tuning must be one of {', '.join(POLICIES)}. Found '{p}'.")
    return p


def _reader(root: str) -> Callable[[str], Optional[str]]:
    def read(path: str) -> Optional[str]:
        full = os.path.join(root, path.lstrip("/")) if root not in ("", "/") else path
        try:
            with open(full, "r", encoding="utf-8", errors="replace") as fh:
                return fh.read().strip()
        except OSError:
            return None

    return read


def facts(root: str = "/") -> Dict[str, str]:
    """``{"numa_balancing": on|off|unknown, "iommu": pt|off|translated}`` of the host
    under ``root`` (a fixture tree in tests)."""
    read = _reader(root)
    nb = read("/proc/sys/kernel/numa_balancing")
    numa = "unknown" if nb is None else ("off" if nb == "0" else "on")
    cmdline = (read("/proc/cmdline") or "").split()
    if "iommu=pt" in cmdline or "amd_iommu=pt" in cmdline:
        iommu = "pt"
    elif "iommu=off" in cmdline or "amd_iommu=off" in cmdline:
        iommu = "off"
    else:
        units = os.path.join(root, "sys/class/iommu") if root not in ("", "/") else "/sys/class/iommu"
        try:
            iommu = "translated" if os.listdir(units) else "off"
        except OSError:
            iommu = "off"
    return {"numa_balancing": numa, "iommu": iommu}


def problems(f: Dict[str, str]) -> List[str]:
    out = []
    if f.get("numa_balancing") == "on":
        out.append("kernel.numa_balancing is on: set it to 0 (sysctl kernel.numa_balancing=0); it migrates "
                   "host pages GPUs have mapped")
    if f.get("iommu") == "translated":
        out.append("the IOMMU translates DMA: boot with iommu=pt for GPU peer-to-peer and GPUDirect RDMA")
    return out


def labels(f: Dict[str, str]) -> Dict[str, str]:
    return {"amd.com/host.numa-balancing": f["numa_balancing"], "amd.com/host.iommu": f["iommu"]}


def shell_check(policy: str, label_file: str, fail: str = "") -> str:
    """The same check as bash (SSH path and the Terraform host script): appends the
    labels to ``label_file``; warnings on stderr; ``enforce`` exits 1 on a problem
    (``fail``: the command run on a problem, e.g. a template expression)."""
    if policy == "off":
        return ""
    fail = fail or ("exit 1" if policy == "enforce" else "true")
    return f"""_tk_nb=$(cat /proc/sys/kernel/numa_balancing 2>/dev/null || echo x)
case $_tk_nb in 0) _tk_nb=off ;; x) _tk_nb=unknown ;; *) _tk_nb=on ;; esac
if grep -qwE '(amd_)?iommu=pt' /proc/cmdline; then _tk_io=pt
elif grep -qwE '(amd_)?iommu=off' /proc/cmdline; then _tk_io=off
elif [ -n "$(ls /sys/class/iommu 2>/dev/null)" ]; then _tk_io=translated
else _tk_io=off; fi
sudo mkdir -p "$(dirname {label_file})"
printf 'amd.com/host.numa-balancing=%s\\namd.com/host.iommu=%s\\n' $_tk_nb $_tk_io | sudo tee -a {label_file} >/dev/null
_tk_bad=0
[ $_tk_nb = on ] && {{ echo 'host tuning: kernel.numa_balancing is on: set it to 0 (sysctl kernel.numa_balancing=0)' >&2; _tk_bad=1; }}
[ $_tk_io = translated ] && {{ echo 'host tuning: the IOMMU translates DMA: boot with iommu=pt for GPU peer-to-peer and GPUDirect RDMA' >&2; _tk_bad=1; }}
[ $_tk_bad = 0 ] || {fail}"""


__all__ = ["POLICIES", "policy_of", "facts", "problems", "labels", "shell_check"]
