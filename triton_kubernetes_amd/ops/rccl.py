"""Python front-end of the RCCL readiness probe (N2, ``csrc/tk_rccl_probe.hip``)."""

import atexit
import ctypes
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional, Sequence

from .native import load

UID_BYTES = 128
DEFAULT_SIZES = [1 << 20, 16 << 20, 256 << 20]
# MI355X: 7 xGMI links x ~153 GB/s per GPU; ring all-reduce is per-link bound.
XGMI_LINK_GBPS = 153.0
XGMI_LINKS_PER_GPU = 7


_ATEXIT = False


class RCCLError(RuntimeError):
    pass


def _lib():
    lib = load("libtk_rccl.so")
    lib.tkr_last_error.restype = ctypes.c_char_p
    lib.tkr_unique_id.argtypes = [ctypes.c_char_p]
    lib.tkr_last_init_ms.restype = ctypes.c_double
    lib.tkr_last_phase_ms.restype = ctypes.c_double
    lib.tkr_last_phase_ms.argtypes = [ctypes.c_int]
    lib.tkr_set_async_teardown.argtypes = [ctypes.c_int]
    lib.tkr_set_teardown_abort.argtypes = [ctypes.c_int]
    lib.tkr_set_teardown_quiet_ms.argtypes = [ctypes.c_double]
    dp = ctypes.POINTER(ctypes.c_double)
    lib.tkr_sweep_rank.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_size_t), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, dp, dp, dp, dp]
    lib.tkr_sweep_local.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_size_t), ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, dp, dp, dp, dp]
    lib.tkr_gate_begin.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    lib.tkr_gate_begin_ex.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_size_t]
    lib.tkr_gate_poll.argtypes = [ctypes.c_int]
    lib.tkr_gate_abort.argtypes = [ctypes.c_int]
    lib.tkr_gate_cancel.argtypes = [ctypes.c_int]
    lib.tkr_gate_sweep.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_size_t), ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_double, dp, dp, dp, dp, dp]
    global _ATEXIT
    if not _ATEXIT:
        atexit.register(lib.tkr_drain)  # join async teardowns before interpreter exit
        _ATEXIT = True
    return lib


def version() -> int:
    return int(_lib().tkr_version())


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(UID_BYTES)
    rc = _lib().tkr_unique_id(buf)
    if rc != 0:
        raise RCCLError(_lib().tkr_last_error().decode())
    return buf.raw[:UID_BYTES]


@dataclass
class SweepResult:
    world: int
    dtype: str
    sizes: List[int]
    time_us: List[float] = field(default_factory=list)
    algbw_gbps: List[float] = field(default_factory=list)
    busbw_gbps: List[float] = field(default_factory=list)
    errors: List[int] = field(default_factory=list)
    init_ms: float = 0.0  # communicator init wall time
    phase_ms: Dict[str, float] = field(default_factory=dict)  # init / alloc / sweep / teardown

    @property
    def ok(self) -> bool:
        return all(e == 0 for e in self.errors)

    @property
    def peak_busbw(self) -> float:
        return max(self.busbw_gbps) if self.busbw_gbps else 0.0

    def to_json(self) -> Dict:
        d = asdict(self)
        d["ok"] = self.ok
        d["peak_busbw_gbps"] = self.peak_busbw
        return d


# = ops/csrc/tk_rccl_verify.h: bf16 sums are verified exactly up to this many ranks
BF16_MAX_WORLD = 256


def check_dtype(dtype: str, world: int) -> None:
    """Refuse a gate whose result cannot be verified exactly (``tk_rccl_verify.h``)."""
    if dtype not in ("f32", "bf16"):
        raise ValueError(f"dtype must be f32 or bf16, not {dtype!r}")
    if dtype == "bf16" and world > BF16_MAX_WORLD:
        raise ValueError(f"a bf16 all-reduce over {world} ranks cannot be verified exactly (bf16 has 8 significant "
                         f"bits: at most {BF16_MAX_WORLD} ranks); gate in f32")


def _arrays(n: int):
    return [(ctypes.c_double * n)() for _ in range(4)]


def sweep_rank(rank: int, world: int, uid: bytes, device: int, sizes: Sequence[int] = DEFAULT_SIZES,
               iters: int = 10, warmup: int = 3, dtype: str = "f32", async_teardown: bool = False) -> SweepResult:
    """One rank of a multi-process sweep.  ``async_teardown`` moves the
    communicator destroy (~0.5 s) off this call; :func:`drain` joins it."""
    check_dtype(dtype, world)
    n = len(sizes)
    sz = (ctypes.c_size_t * n)(*sizes)
    t, alg, bus, err = _arrays(n)
    lib = _lib()
    lib.tkr_set_async_teardown(1 if async_teardown else 0)  # thread-local in the library
    try:
        rc = lib.tkr_sweep_rank(rank, world, uid, device, sz, n, iters, warmup, 1 if dtype == "bf16" else 0,
                                t, alg, bus, err)
    finally:
        lib.tkr_set_async_teardown(0)
    if rc != 0:
        raise RCCLError(f"rank {rank}/{world}: {_lib().tkr_last_error().decode()}")
    lib = _lib()
    phases = {name: round(float(lib.tkr_last_phase_ms(i)), 3)
              for i, name in enumerate(("init", "alloc", "sweep", "teardown"))}
    return SweepResult(world, dtype, list(sizes), list(t), list(alg), list(bus), [int(e) for e in err],
                       float(lib.tkr_last_init_ms()), phases)


class GateComm:
    """This process's ranks ``rank_base .. rank_base+len(devices)-1`` of a cluster-wide
    communicator (``tkr_gate_*``).  ``blocking=False`` runs the grouped
    ``ncclCommInitRank`` on a thread of its own and returns at once, so the init overlaps
    whatever the caller does next;
    :meth:`sweep` waits for the rest, runs the verified all-reduce sweep and
    consumes the handle.  :meth:`abort` releases a gate that will never run."""

    def __init__(self, uid: bytes, world: int, rank_base: int, devices: Sequence[int], blocking: bool = False,
                 prealloc_bytes: int = 0):
        self.world, self.rank_base, self.devices = world, rank_base, list(devices)
        devs = (ctypes.c_int * len(self.devices))(*self.devices)
        h = _lib().tkr_gate_begin_ex(uid, world, rank_base, len(self.devices), devs, 1 if blocking else 0,
                                     int(prealloc_bytes))
        if h < 0:
            raise RCCLError(f"ranks {rank_base}+{len(self.devices)}/{world}: {_lib().tkr_last_error().decode()}")
        self.handle = h
        self._sweeping: Optional[int] = None  # the handle a running sweep consumes

    def ready(self) -> bool:
        rc = _lib().tkr_gate_poll(self.handle)
        if rc < 0:
            raise RCCLError(_lib().tkr_last_error().decode())
        return rc == 0

    def sweep(self, sizes: Sequence[int], iters: int = 10, warmup: int = 3, dtype: str = "f32",
              timeout_s: float = 600.0, async_teardown: bool = True) -> SweepResult:
        if self.handle is None:
            raise RCCLError("gate already consumed")
        try:
            check_dtype(dtype, self.world)
        except ValueError:
            self.abort()  # every rank refuses alike: release the communicator, do not leak it
            raise
        n = len(sizes)
        sz = (ctypes.c_size_t * n)(*sizes)
        t, alg, bus, err = _arrays(n)
        ph = (ctypes.c_double * 5)()
        lib = _lib()
        lib.tkr_set_async_teardown(1 if async_teardown else 0)
        self._sweeping, self.handle = self.handle, None
        try:
            rc = lib.tkr_gate_sweep(self._sweeping, sz, n, iters, warmup, 1 if dtype == "bf16" else 0,
                                    timeout_s * 1e3, t, alg, bus, err, ph)
        finally:
            lib.tkr_set_async_teardown(0)
            self._sweeping = None
        if rc != 0:
            raise RCCLError(f"ranks {self.rank_base}+{len(self.devices)}/{self.world}: "
                            f"{lib.tkr_last_error().decode()}")
        phases = {"init_wait": round(ph[0], 3), "alloc": round(ph[1], 3), "sweep": round(ph[2], 3),
                  "teardown": round(ph[3], 3), "init_total": round(ph[4], 3)}
        if hasattr(lib, "tkr_last_footprint"):
            # device memory the init took per GPU (max over this process's ranks): the
            # communicators, then with their preallocated sweep buffers (tk_rccl_probe.hip)
            lib.tkr_last_footprint.restype = ctypes.c_double
            lib.tkr_last_footprint.argtypes = [ctypes.c_int]
            # (-1: this process's VRAM could not be read -- no KFD accounting -- so not measured)
            for i, k in enumerate(("footprint_mib", "footprint_total_mib")):
                b = float(lib.tkr_last_footprint(i))
                phases[k] = round(b / 2 ** 20, 1) if b >= 0 else -1.0
            # 1: this process's own VRAM (KFD accounting); 2: the device's used memory, which
            # counts other allocations made meanwhile (a burn-in child's span)
            phases["footprint_kind"] = float(lib.tkr_last_footprint(2))
        return SweepResult(self.world, dtype, list(sizes), list(t), list(alg), list(bus), [int(e) for e in err],
                           float(ph[4]), phases)

    def abort(self) -> None:
        if self.handle is not None:
            _lib().tkr_gate_abort(self.handle)
            self.handle = None

    def cancel(self) -> None:
        """Stop this gate from another thread: a pending one is aborted; a sweep still
        waiting for its peers returns at once with an error (``tkr_gate_cancel``)."""
        h = self._sweeping if self._sweeping is not None else self.handle
        if h is not None:
            _lib().tkr_gate_cancel(h)
            if h == self.handle:
                self.handle = None


# A failed init whose least-free GPU had less than this left ran out of memory, whatever
# RCCL called the failure ("unhandled cuda error" / "unhandled system error")
OOM_FREE_MIB = 2048
# appended to the error of an init that failed again after the agent released its held
# burn-in spans and retried (node/agent_gate.py): the cluster gate does not retry it again
OOM_RETRIED_MARK = "[gate_retry: oom, failed again after the held spans' release]"


def is_oom_error(text: str) -> bool:
    """An RCCL communicator init that failed for lack of device memory, by the error text
    libtk_rccl gives (``tk_rccl_probe.hip:annotate_init_error``): RCCL's own last error naming
    an out-of-memory allocation, or an unhandled HIP/system error with a GPU nearly full."""
    import re

    low = (text or "").lower()
    if "out of memory" in low or "outofmemory" in low:
        return True
    m = re.search(r"\(device \d+: (\d+) mib free\)", low)
    return bool(m and ("unhandled cuda error" in low or "unhandled system error" in low)
                and int(m.group(1)) < OOM_FREE_MIB)


def pending_gates() -> int:
    return int(_lib().tkr_gate_pending())


def abandoned_inits() -> int:
    """Gate inits released while still waiting for absent peers (detached threads)."""
    return int(_lib().tkr_gate_abandoned())


def inits_running() -> int:
    """Communicator inits of this process still running (0 when libtk_rccl was never loaded:
    nothing to wait for, and nothing is loaded to find out)."""
    from . import native

    lib = native._cache.get("libtk_rccl.so")
    return int(lib.tkr_inits_running()) if lib is not None else 0


def preload_device_code(devices: Sequence[int]) -> bool:
    """Start loading RCCL's device code for ``devices`` on background threads
    (``tkr_preload_device_code``); True when started."""
    devs = [int(d) for d in devices]
    if not devs:
        return False
    return _lib().tkr_preload_device_code(len(devs), (ctypes.c_int * len(devs))(*devs)) == 0


def preload_report() -> dict:
    """Which kernel handle the last :func:`preload_device_code` used and how it was found
    (``known``: one of the names /opt/rocm's librccl exports; ``scan``: found in the loaded
    librccl's dynamic symbols, ``ops/csrc/tk_elf_scan.h``), or ``none``."""
    lib = _lib()
    lib.tkr_preload_symbol.restype = ctypes.c_char_p
    lib.tkr_preload_how.restype = ctypes.c_char_p
    return {"symbol": lib.tkr_preload_symbol().decode(), "how": lib.tkr_preload_how().decode()}


def preloads_running() -> int:
    from . import native

    lib = native._cache.get("libtk_rccl.so")
    return int(lib.tkr_preloads_running()) if lib is not None else 0


def exit_now(code: int = 0) -> None:
    """Leave the process without the HIP/RCCL exit teardown, which cannot complete while an
    abandoned init thread is blocked in RCCL's bootstrap.  Flushes stdio first."""
    import os
    import sys

    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(code)


def set_teardown_quiet_ms(ms: float) -> None:
    """Run queued communicator teardowns only after ``ms`` without gate activity."""
    _lib().tkr_set_teardown_quiet_ms(float(ms))


def drain() -> int:
    """Join pending asynchronous teardowns; call before the process exits."""
    return int(_lib().tkr_drain())


def sweep_local(ndev: int, sizes: Sequence[int] = DEFAULT_SIZES, iters: int = 10, warmup: int = 3,
                dtype: str = "f32") -> SweepResult:
    n = len(sizes)
    sz = (ctypes.c_size_t * n)(*sizes)
    t, alg, bus, err = _arrays(n)
    rc = _lib().tkr_sweep_local(ndev, sz, n, iters, warmup, 1 if dtype == "bf16" else 0, t, alg, bus, err)
    if rc != 0:
        raise RCCLError(_lib().tkr_last_error().decode())
    return SweepResult(ndev, dtype, list(sizes), list(t), list(alg), list(bus), [int(e) for e in err],
                       float(_lib().tkr_last_init_ms()))
