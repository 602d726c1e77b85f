"""Process / cgroup CPU accounting for bring-up diagnostics.

A bring-up step that stalls every thread of the process at once (socket(), sysfs
reads, pure-Python code alike) is usually the CPU controller throttling the
process's cgroup (CFS quota exhausted inside a period by spinning runtime threads),
not a lock.  :func:`snapshot` reads what is needed to tell: process CPU time, thread
count, and the cgroup's throttling counters (cgroup v2 ``cpu.stat`` /``cpu.max``, or
v1 ``cpu,cpuacct``), and :func:`delta` differences two snapshots.
"""

import os
import resource
from typing import Dict, Optional

_CG_CACHE: Dict[str, Optional[str]] = {}


def _read(path: str) -> Optional[str]:
    try:
        with open(path, encoding="utf-8") as fh:
            return fh.read()
    except OSError:
        return None


def cgroup_cpu_dir() -> Optional[str]:
    """Directory holding this process's CPU controller files (v2 unified or v1 cpu)."""
    if "dir" in _CG_CACHE:
        return _CG_CACHE["dir"]
    found = None
    text = _read("/proc/self/cgroup") or ""
    for line in text.splitlines():
        parts = line.split(":", 2)
        if len(parts) != 3:
            continue
        _, ctrls, path = parts
        cands = []
        # inside a cgroup namespace the listed path is relative to a root mounted at
        # /sys/fs/cgroup itself, so the mount root is a candidate too
        if ctrls == "":  # v2: the cpu controller is enabled where cpu.max exists
            cands, marker = [os.path.join("/sys/fs/cgroup", path.lstrip("/")), "/sys/fs/cgroup"], "cpu.max"
        elif "cpu" in ctrls.split(","):
            cands = [os.path.join("/sys/fs/cgroup", d, path.lstrip("/")) for d in ("cpu,cpuacct", "cpu")]
            cands += ["/sys/fs/cgroup/cpu,cpuacct", "/sys/fs/cgroup/cpu"]
            marker = "cpu.cfs_quota_us"
        for c in cands:
            if os.path.exists(os.path.join(c, marker)):
                found = c
                break
        if found and ctrls != "":
            break  # prefer the v1 cpu controller when both are listed
    _CG_CACHE["dir"] = found
    return found


def snapshot() -> Dict[str, float]:
    ru = resource.getrusage(resource.RUSAGE_SELF)
    out = {"cpu_s": ru.ru_utime + ru.ru_stime, "nvcsw": ru.ru_nvcsw, "nivcsw": ru.ru_nivcsw}
    try:
        out["fds"] = len(os.listdir("/proc/self/fd"))
    except OSError:
        pass
    status = _read("/proc/self/status") or ""
    for line in status.splitlines():
        if line.startswith("Threads:"):
            out["threads"] = int(line.split()[1])
    for res in ("cpu", "memory", "io"):  # pressure stall information (system-wide), "some" total
        psi = _read(f"/proc/pressure/{res}") or ""
        for line in psi.splitlines():
            if line.startswith("some ") and "total=" in line:
                out[f"psi_{res}_ms"] = int(line.rsplit("total=", 1)[1]) / 1e3
    d = cgroup_cpu_dir()
    stat = _read(os.path.join(d, "cpu.stat")) if d else None
    for line in (stat or "").splitlines():
        k, _, v = line.partition(" ")
        if k in ("nr_periods", "nr_throttled"):
            out["cg_" + k] = int(v)
        elif k == "throttled_usec":  # v2
            out["cg_throttled_ms"] = int(v) / 1e3
        elif k == "throttled_time":  # v1, ns
            out["cg_throttled_ms"] = int(v) / 1e6
    return out


def delta(a: Dict[str, float], b: Dict[str, float]) -> Dict[str, float]:
    """b - a for counters; the thread count is reported as of ``b``."""
    out = {}
    for k, v in b.items():
        if k == "threads":
            out[k] = v
        elif k in a:
            out[k] = round(v - a[k], 3)
    return out


def presize_fd_table(slots: int = 16384) -> int:
    """Grow this process's file-descriptor table once, up front; returns its new size.

    The kernel grows an fd table by doubling it and, before the old table may be
    freed, waits for an RCU grace period (``expand_fdtable`` -> ``synchronize_rcu``);
    every other thread that allocates a descriptor meanwhile (socket(), open(), a
    HIP allocation exporting a dma-buf) blocks on the resize.  RCCL communicators
    and the HIP runtime churn through hundreds of descriptors, so without this the
    first bring-ups of a long-lived agent hit those resizes (tens to hundreds of ms
    on a large, busy host).  The table never shrinks, so one resize here — at
    startup, before any bring-up — removes them.  Also lifts the soft RLIMIT_NOFILE
    to cover ``slots`` (within the hard limit), as long-lived daemons do.
    """
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    want = slots if hard == resource.RLIM_INFINITY else min(slots, hard)
    if soft != resource.RLIM_INFINITY and soft < want:
        try:
            resource.setrlimit(resource.RLIMIT_NOFILE, (want, hard))
            soft = want
        except (ValueError, OSError):
            pass
    top = min(want, soft if soft != resource.RLIM_INFINITY else want) - 1
    if top < 3:
        return 0
    fd = os.open("/dev/null", os.O_RDONLY | os.O_CLOEXEC)
    try:
        if top > fd:
            os.dup2(fd, top, inheritable=False)
            os.close(top)
    finally:
        os.close(fd)
    return top + 1
