"""Python front-end of the MI355X burn-in probes (``csrc/tk_gpu_probe.hip``).

``run_burnin(device, level)`` is what the MI355X host bootstrap executes per
GPU before the node may advertise ``amd.com/gpu``.  Thresholds are fractions of
MI355X figures (MI355X_MICROARCH.md): HBM3E ~6.3 TB/s achievable of 8 TB/s
spec, dense bf16 MFMA ~2.5 PFLOP/s, block-scaled fp8 ~5 PFLOP/s.  A GPU that
fails a threshold or the memtest marks the node not-ready.

In a node agent (:func:`set_burnin_process`) each GPU's burn-in -- and the node's xGMI
link matrix (:func:`link_matrix_process`) -- runs in a ``gpu-burnin`` child process: the
agent's own HIP runtime is busy loading RCCL's device code for the cluster gate meanwhile.
The child reports its measurements, this module judges them against the same floors as
the in-process path, and the child keeps the HBM it tested until the agent's release hold
(:func:`set_release_hold`) lets go.
"""

import contextlib
import ctypes
import json
import os
import queue
import subprocess
import threading
import time
from dataclasses import asdict, dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

from ..utils.trace import span
from . import native
from .native import load

# MI355X reference figures (dense; never the 2:1-sparsity marketing numbers)
MI355X_HBM_ACHIEVABLE_GBPS = 6300.0
MI355X_BF16_DENSE_TFLOPS = 2500.0
MI355X_FP8_DENSE_TFLOPS = 5000.0
MI355X_F32_MFMA_TFLOPS = 157.3
MI355X_CUS = 256

DTYPES = {"bf16": 0, "fp8": 1, "f32": 2}


class _DeviceInfo(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char * 128),
        ("arch", ctypes.c_char * 64),
        ("compute_units", ctypes.c_int),
        ("wavefront_size", ctypes.c_int),
        ("clock_khz", ctypes.c_int),
        ("mem_clock_khz", ctypes.c_int),
        ("mem_bus_width", ctypes.c_int),
        ("l2_bytes", ctypes.c_int),
        ("lds_per_block", ctypes.c_int),
        ("pci_domain", ctypes.c_int),
        ("pci_bus", ctypes.c_int),
        ("pci_device", ctypes.c_int),
        ("total_mem", ctypes.c_longlong),
        ("free_mem", ctypes.c_longlong),
    ]


class ProbeError(RuntimeError):
    pass


def _lib():
    lib = load("libtk_gpu_probe.so")
    lib.tkp_last_error.restype = ctypes.c_char_p
    lib.tkp_hbm_bandwidth.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_double)]
    lib.tkp_mfma_peak.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_double)]
    lib.tkp_mfma_clock.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                   ctypes.POINTER(ctypes.c_double)]
    lib.tkp_memtest.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    lib.tkp_memtest_span.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_double)]
    lib.tkp_set_async_free.argtypes = [ctypes.c_int]
    lib.tkp_set_fail_point.argtypes = [ctypes.c_char_p]
    lib.tkp_set_fail_point.restype = None
    lib.tkp_memtest_selfcheck.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_double)]
    lib.tkp_p2p_bandwidth.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_double)]
    lib.tkp_link_matrix.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
    lib.tkp_link_matrix_mode.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
    lib.tkp_link_matrix_check.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                                          ctypes.POINTER(ctypes.c_double)]
    lib.tkp_set_scratch_cache.argtypes = [ctypes.c_int]
    lib.tkp_prealloc_scratch.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t]
    lib.tkp_release_scratch.restype = ctypes.c_longlong
    lib.tkp_release_scratch_dev.argtypes = [ctypes.c_int]
    lib.tkp_release_scratch_dev.restype = ctypes.c_longlong
    return lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise ProbeError(f"{what}: {_lib().tkp_last_error().decode(errors='replace')}")


def device_count() -> int:
    n = ctypes.c_int(0)
    _check(_lib().tkp_device_count(ctypes.byref(n)), "device_count")
    return n.value


@dataclass
class DeviceInfo:
    index: int
    name: str
    arch: str
    compute_units: int
    wavefront_size: int
    clock_mhz: float
    total_mem_gib: float
    free_mem_gib: float
    l2_bytes: int
    pci_bus_id: str

    @property
    def is_gfx950(self) -> bool:
        return self.arch.split(":")[0] == "gfx950"


def device_info(dev: int) -> DeviceInfo:
    info = _DeviceInfo()
    _check(_lib().tkp_device_info(dev, ctypes.byref(info)), "device_info")
    return DeviceInfo(
        index=dev, name=info.name.decode(errors="replace"), arch=info.arch.decode(errors="replace"),
        compute_units=info.compute_units, wavefront_size=info.wavefront_size, clock_mhz=info.clock_khz / 1000.0,
        total_mem_gib=info.total_mem / 2 ** 30, free_mem_gib=info.free_mem / 2 ** 30, l2_bytes=info.l2_bytes,
        pci_bus_id=f"{info.pci_domain:04x}:{info.pci_bus:02x}:{info.pci_device:02x}.0")


def hbm_bandwidth(dev: int, nbytes: int = 1 << 30, iters: int = 5, blocks_per_cu: int = 16) -> Dict[str, float]:
    out = (ctypes.c_double * 3)()
    _check(_lib().tkp_hbm_bandwidth(dev, nbytes, iters, blocks_per_cu, out), "hbm_bandwidth")
    return {"read_gbps": out[0], "write_gbps": out[1], "copy_gbps": out[2]}


def mfma_peak(dev: int, dtype: str = "bf16", iters: int = 20000, reps: int = 3,
              blocks_per_cu: int = 2) -> Dict[str, float]:
    out = (ctypes.c_double * 2)()
    _check(_lib().tkp_mfma_peak(dev, DTYPES[dtype], iters, reps, blocks_per_cu, out), f"mfma_peak[{dtype}]")
    return {"tflops": out[0], "ms": out[1]}


# MFMA FLOP per clock per SIMD at full issue (MI355X_MICROARCH.md § Matrix cores)
MFMA_PEAK_FLOP_PER_CLK = {"bf16": 1024.0, "fp8": 2048.0, "f32": 64.0}


def mfma_clock(dev: int, dtype: str = "bf16", iters: int = 20000, warm_ms: float = 1500.0,
               blocks_per_cu: int = 2) -> Dict[str, float]:
    """Diagnostic: the in-kernel clock the chip holds under the MFMA loop (after ``warm_ms``
    of back-to-back launches) and the loop's FLOP per clock per SIMD at that clock.

    ``issue_efficiency`` near 1 means the kernel issues MFMAs at the per-clock peak, so the
    gap between measured TFLOP/s and the 2.5 / 5 PF dense figures is the clock the chip
    holds under load on random operands (DVFS), not the kernel."""
    out = (ctypes.c_double * 3)()
    _check(_lib().tkp_mfma_clock(dev, DTYPES[dtype], iters, blocks_per_cu, float(warm_ms), out),
           f"mfma_clock[{dtype}]")
    peak = MFMA_PEAK_FLOP_PER_CLK[dtype]
    return {"mhz": round(out[0], 1), "flop_per_clk_per_simd": round(out[1], 1), "tflops": round(out[2], 1),
            "issue_efficiency": round(out[1] / peak, 4) if peak else 0.0}


def memtest(dev: int, nbytes: int = 1 << 30, passes: int = 2) -> Dict[str, float]:
    out = (ctypes.c_double * 2)()
    _check(_lib().tkp_memtest(dev, nbytes, passes, out), "memtest")
    return {"errors": int(out[0]), "verify_gbps": out[1]}


def memtest_span(dev: int, nbytes: int = 0, chunk: int = 16 << 30, headroom: int = 4 << 30,
                 passes: int = 1) -> Dict[str, float]:
    """Memtest of ``nbytes`` of HBM (0: all free HBM but ``headroom``) held as ``chunk``-byte
    allocations at once, so the whole span is distinct physical memory."""
    out = (ctypes.c_double * 7)()
    _check(_lib().tkp_memtest_span(dev, nbytes, chunk, headroom, passes, out), "memtest_span")
    return {"errors": int(out[0]), "verify_gbps": out[1], "bytes": int(out[2]), "hbm_bytes": int(out[3]),
            "alloc_ms": round(out[4], 1), "test_ms": round(out[5], 1), "free_ms": round(out[6], 1)}


def set_fail_point(name: str) -> None:
    """Tests only: make the named step of the span memtest fail ("" clears it)."""
    _lib().tkp_set_fail_point(name.encode())


def free_bytes(dev: int) -> int:
    """Free HBM of ``dev`` right now (``hipMemGetInfo``)."""
    return int(device_info(dev).free_mem_gib * 2 ** 30)


def set_async_free(on: bool) -> None:
    """Release the span memtest's chunks on a background thread (long-lived agents)."""
    _lib().tkp_set_async_free(1 if on else 0)


def wait_frees(children: bool = True) -> None:
    """Join pending background releases of span-memtest memory (in this process, and --
    ``children`` -- the ``gpu-burnin`` children still releasing theirs)."""
    _lib().tkp_wait_frees()
    if children:
        _wait_span_children()


# --- the full memtest in a short-lived child process (long-lived agents) ----------------------
# A full memtest holds ~300 GB.  Releasing it costs the kernel driver's VRAM clearing (~35 GB/s
# per GPU, profiles/round4/alloc_probe.jsonl), and while a hipFree of a 16 GiB chunk waits for
# that (~0.5 s), every other HIP call of the same process waits too: in an agent, the gate's
# sweep and the plan's later GPU steps stalled for seconds behind the background release
# (profiles/round4/README.md).  So an agent runs the span in ``gpu-burnin --memtest-span``: the
# child prints its verdict as soon as it is known and releases the memory itself, outside the
# agent's HIP runtime.  The next span (and ``wait_frees``) waits for it to exit.  The child
# holds the span in 1 GiB chunks: the release then blocks other GPU users (the driver
# serialises their copies and frees behind each chunk's clearing, across processes) for
# ~30 ms at a time instead of ~0.5 s (profiles/round4/span_chunk_ab.jsonl: the gate's sweep
# after a full burn-in 4-6 ms with 1 GiB chunks, up to 0.5 s with 16 GiB ones).


def _burnin_exe() -> str:
    """``gpu-burnin`` as built from this tree (NativeUnavailable if missing or stale)."""
    return native.executable("gpu-burnin")


SPAN_CHILD_CHUNK = int(float(os.environ.get("TK_SPAN_CHUNK_GIB", "1")) * (1 << 30))
SPAN_RELEASE_TIMEOUT_S = 600.0
_SPAN_PROCESS = False
_span_children: List[Any] = []  # (device, child): children whose span may still be releasing
_span_mu = threading.Lock()
# GPU work this process started or ran that allocates device memory (burn-in children, and
# in-process burn-ins): a device-wide free-memory delta is only this process's own when no
# such work started, ran or was alive across it (:func:`activity`)
_activity_starts = 0
_activity_inproc = 0


def activity() -> Tuple[int, int]:
    """``(work started so far, work alive now)``.  Two equal snapshots with nothing alive
    bracket a window in which no burn-in of this agent allocated or released HBM."""
    with _span_mu:
        alive = sum(1 for _, p in _span_children if p.poll() is None) + _activity_inproc
        return _activity_starts, alive


class _InProcess:
    """An in-process burn-in, counted by :func:`activity`."""

    def __enter__(self):
        global _activity_starts, _activity_inproc
        with _span_mu:
            _activity_starts += 1
            _activity_inproc += 1

    def __exit__(self, *exc):
        global _activity_inproc
        with _span_mu:
            _activity_inproc -= 1


def set_span_process(on: bool) -> None:
    """Run the full memtest (``run_burnin`` level ``full``) in a child process."""
    global _SPAN_PROCESS
    _SPAN_PROCESS = bool(on)


def _wait_span_children(dev: Optional[int] = None) -> None:
    """Wait for the span children (of ``dev`` only, when given) to exit."""
    with _span_mu:
        children = [c for c in _span_children if dev is None or c[0] == dev]
    for _, proc in children:
        try:  # a release takes seconds; a child stuck far longer than that is killed
            proc.wait(timeout=SPAN_RELEASE_TIMEOUT_S)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
    with _span_mu:
        for c in children:
            if c in _span_children:
                _span_children.remove(c)


def memtest_span_process(dev: int, nbytes: int = 0, headroom: int = 4 << 30, passes: int = 1,
                         timeout: float = 900.0, release_arena: bool = True, chunk: int = 0) -> Dict[str, float]:
    """:func:`memtest_span` in a ``gpu-burnin --memtest-span`` child: returns as soon as the
    child reports its verdict; the child releases the span afterwards (joined by
    :func:`wait_frees`).  This process's burn-in arena is freed first, so its HBM is tested."""
    if release_arena:
        release_scratch(dev)
    _lib().tkp_wait_frees()
    _wait_span_children(dev)  # this device's previous span is released before this one allocates
    try:  # built from this tree's sources (a stale build would ignore --memtest-span)
        exe = _burnin_exe()
    except native.NativeUnavailable as exc:
        return _span_in_process(dev, nbytes, headroom, passes, f"gpu-burnin unusable: {exc}")
    argv = [exe, "--memtest-span", "--device", str(int(dev)), "--span-bytes", str(int(nbytes)),
            "--span-headroom", str(int(headroom)), "--span-passes", str(int(passes)),
            "--span-chunk", str(int(chunk or SPAN_CHILD_CHUNK))]
    try:
        doc, process_ms = _child_verdict(argv, dev, timeout, "memtest_span")
    except _ChildUnstartable as exc:
        return _span_in_process(dev, nbytes, headroom, passes, str(exc))
    if not doc.get("ok"):
        raise ProbeError(f"memtest_span: {doc.get('error', 'failed')}")
    try:
        return {"errors": int(doc["errors"]), "verify_gbps": float(doc["verify_gbps"]), "bytes": int(doc["bytes"]),
                "hbm_bytes": int(doc["hbm_bytes"]), "alloc_ms": float(doc["alloc_ms"]),
                "test_ms": float(doc["test_ms"]), "free_ms": 0.0, "process_ms": process_ms}
    except (KeyError, TypeError, ValueError) as exc:
        # not a --memtest-span verdict (a whole burn-in's report, say): no verdict at all
        raise ProbeError(f"memtest_span: {exe} gave no memtest-span verdict ({type(exc).__name__}: {exc}): "
                         f"{json.dumps(doc)[:200]!r}") from None


class _ChildUnstartable(native.NativeUnavailable):
    """The ``gpu-burnin`` child could not be started (nothing ran on the GPU)."""


# Called (on a thread of its own) before a child releases the HBM it tested; None: release
# at once.  The node agent waits here for its RCCL communicator inits (node/agent.py): the
# driver clears a release of ~300 GB for seconds, and an init loading RCCL's device code
# meanwhile waited behind that clearing (1.8 s -> 3.5 s, profiles/round5/README.md).
_RELEASE_HOLD: Optional[Callable[[], None]] = None
RELEASE_HOLD_MAX_MS = 30000  # the child releases by itself after this long


def set_release_hold(fn: Optional[Callable[[], None]]) -> None:
    """``fn`` returns when a burn-in child may release what it holds (see ``_RELEASE_HOLD``)."""
    global _RELEASE_HOLD
    _RELEASE_HOLD = fn


def _release_after_hold(proc: Any, hold: Callable[[], None]) -> None:
    try:
        hold()
    except Exception:  # noqa: BLE001 - the child must be released whatever the hold did
        pass
    finally:
        try:
            proc.stdin.close()  # EOF: the child frees and exits
        except OSError:
            pass


def _child_verdict(argv: List[str], dev: int, timeout: float, what: str,
                   hold: bool = True) -> Tuple[Dict[str, Any], float]:
    """Start a ``gpu-burnin`` child for ``dev`` and return its JSON verdict (the first JSON
    line it prints) and the ms until then.  The child is registered with the device's span
    children: it releases what it holds after the verdict -- once the release hold says so
    (:func:`set_release_hold`) -- and the next span on the device (and :func:`wait_frees`)
    waits for it to exit."""
    t0 = time.perf_counter()
    hold = _RELEASE_HOLD if hold else None  # a child holding no HBM has nothing to release
    if hold is not None:
        argv = list(argv) + ["--hold-stdin", "--hold-max-ms", str(RELEASE_HOLD_MAX_MS)]
    try:
        proc = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True,
                                stdin=subprocess.PIPE if hold is not None else subprocess.DEVNULL,
                                start_new_session=True)
    except OSError as exc:
        raise _ChildUnstartable(f"cannot start {argv[0]}: {exc}") from exc
    with _span_mu:
        global _activity_starts
        _span_children.append((dev, proc))
        _activity_starts += 1
    # the verdict is the one JSON line (a library may print others); read on a thread, so a
    # line already buffered behind an earlier one is not waited for
    got: "queue.Queue[str]" = queue.Queue()

    def read_verdict() -> None:
        verdict = ""
        for text in proc.stdout:  # read to the end: a child writing after its verdict never blocks on the pipe
            if text.startswith("{") and not verdict:
                verdict = text
                got.put(text)
        if not verdict:
            got.put("")
        proc.stdout.close()

    threading.Thread(target=read_verdict, name=f"tk-span-{dev}", daemon=True).start()
    try:
        line = got.get(timeout=timeout)
    except queue.Empty:
        proc.kill()
        raise ProbeError(f"{what}: {os.path.basename(argv[0])} {argv[1]} gave no verdict within {timeout:.0f} s") \
            from None
    if not line:
        proc.wait(timeout=SPAN_RELEASE_TIMEOUT_S)
        raise ProbeError(f"{what}: {os.path.basename(argv[0])} {argv[1]} exited {proc.returncode} without a verdict")
    try:
        doc = json.loads(line)
    except ValueError as exc:
        proc.kill()
        raise ProbeError(f"{what}: unreadable verdict {line[:200]!r}") from exc
    if not isinstance(doc, dict):
        proc.kill()
        raise ProbeError(f"{what}: unreadable verdict {line[:200]!r}")
    ms = round((time.perf_counter() - t0) * 1e3, 1)
    if hold is not None:
        threading.Thread(target=_release_after_hold, args=(proc, hold), name=f"tk-release-{dev}",
                         daemon=True).start()
    return doc, ms


def _span_in_process(dev: int, nbytes: int, headroom: int, passes: int, why: str) -> Dict[str, float]:
    """The span memtest in this process (``gpu-burnin`` cannot run here): the same test,
    released on this process's background thread; ``span_fallback`` says why."""
    out: Dict[str, Any] = dict(memtest_span(dev, nbytes, headroom=headroom, passes=passes))
    out["span_fallback"] = why
    return out


def _span(dev: int, nbytes: int, passes: int) -> Dict[str, float]:
    if _SPAN_PROCESS:
        return memtest_span_process(dev, nbytes, passes=passes)
    return memtest_span(dev, nbytes, passes=passes)


def memtest_selfcheck(dev: int, nbytes: int, corrupt: int) -> int:
    out = (ctypes.c_double * 1)()
    _check(_lib().tkp_memtest_selfcheck(dev, nbytes, corrupt, out), "memtest_selfcheck")
    return int(out[0])


def p2p_bandwidth(src: int, dst: int, nbytes: int = 256 << 20, iters: int = 5) -> Dict[str, float]:
    out = (ctypes.c_double * 2)()
    _check(_lib().tkp_p2p_bandwidth(src, dst, nbytes, iters, out), "p2p_bandwidth")
    return {"gbps": out[0], "peer_access": bool(out[1])}


# MI355X: 7 xGMI links per GPU of ~153.6 GB/s (both directions together), so ~76.8 GB/s per
# direction.  The link check fails a pair below half of that, whatever the node's median.
XGMI_LINK_ONE_WAY_GBPS = 76.8
DEFAULT_MIN_LINK_GBPS = 38.0
LINK_METHODS = {"sdma-copy": 0, "kernel-read": 1}


def link_matrix_process(devices: Sequence[int], nbytes: int = 64 << 20, iters: int = 3,
                        method: str = "kernel-read", timeout: float = 600.0) -> Dict[str, Any]:
    """:func:`link_matrix` measured by a ``gpu-burnin --p2p-child`` process (same result):
    a node agent's own HIP runtime may be busy loading RCCL's device code for the cluster
    gate, and its kernel launches wait behind that load (``_burnin_child``).  Raises
    ``NativeUnavailable`` (``_ChildUnstartable``) when the child cannot run."""
    if method not in LINK_METHODS:
        raise ValueError(f"link method must be one of {sorted(LINK_METHODS)}")
    devs = [int(d) for d in devices]
    argv = [_burnin_exe(), "--p2p-child", "--devices", ",".join(str(d) for d in devs), "--bytes", str(int(nbytes)),
            "--iters", str(int(iters)), "--p2p-method", method]
    doc, _ = _child_verdict(argv, devs[0] if devs else 0, timeout, "link_matrix", hold=False)
    if not doc.get("ok"):
        raise ProbeError(f"link_matrix: {doc.get('error', 'no verdict')}")
    if "pairs" not in doc:
        raise ProbeError(f"link_matrix: unreadable verdict {json.dumps(doc)[:200]}")
    return {k: doc.get(k) for k in ("pairs", "peer_access", "errors", "bytes", "method", "data_errors")}


def link_matrix(devices: Sequence[int], nbytes: int = 64 << 20, iters: int = 3,
                method: str = "kernel-read") -> Dict[str, Any]:
    """Peer bandwidth of every ordered GPU pair: ``{"pairs": {"i-j": GB/s}, "peer_access":
    {"i-j": bool}, "errors": [...], "method": ...}``.  ``kernel-read`` (default): a kernel on
    the receiving GPU reads the sender's memory over xGMI, the way RCCL and workloads use the
    fabric; ``sdma-copy``: ``hipMemcpyPeerAsync`` on the copy engines.  ``tkp_link_matrix_mode``
    measures the pairs in rounds of a round-robin pairing: transfers run concurrently only on
    disjoint pairs, so each number is still one xGMI link's, not a share of a busy fabric
    (8 GPUs: 14 timed slots instead of 56).  A pair that fails is recorded as an error, not
    raised: the caller decides (``node/labels.py:link_labels``).  ``data_errors``: what
    arrived was checked against the sender's pattern after each pair's last transfer
    (mismatching 32-bit words per pair): a link that corrupts data at full speed."""
    devs = list(devices)
    n = len(devs)
    pairs: Dict[str, float] = {}
    access: Dict[str, bool] = {}
    errors: List[str] = []
    if method not in LINK_METHODS:
        raise ValueError(f"link method must be one of {sorted(LINK_METHODS)}")
    data_errors: Dict[str, int] = {}
    if n < 2:
        return {"pairs": pairs, "peer_access": access, "errors": errors, "bytes": nbytes, "method": method,
                "data_errors": data_errors}
    gbps = (ctypes.c_double * (n * n))()
    acc = (ctypes.c_int * (n * n))()
    errs = (ctypes.c_double * (n * n))()
    _check(_lib().tkp_link_matrix_check((ctypes.c_int * n)(*devs), n, nbytes, iters, LINK_METHODS[method], gbps, acc,
                                        errs), "link_matrix")
    for a, i in enumerate(devs):
        for b, j in enumerate(devs):
            if a == b:
                continue
            v = gbps[a * n + b]
            access[f"{i}-{j}"] = bool(acc[a * n + b]) or i == j
            if v < 0:
                errors.append(f"{i}->{j}: peer {'read' if method == 'kernel-read' else 'copy'} failed")
                continue
            pairs[f"{i}-{j}"] = round(v, 1)
            if errs[a * n + b] > 0:
                data_errors[f"{i}-{j}"] = int(errs[a * n + b])
    return {"pairs": pairs, "peer_access": access, "errors": errors, "bytes": nbytes, "method": method,
            "data_errors": data_errors}


# --- burn-in policy ------------------------------------------------------------------
REMEASURE = 2  # extra runs of a throughput gate that read below its floor
LEVELS = {
    # level: (hbm bytes, hbm iters, mfma iters (x 8 accumulator chains per wave), memtest bytes, memtest passes)
    # memtest bytes 0 = every free byte of HBM but 4 GiB (memtest_span), sized from
    # hipMemGetInfo when it runs; quick tests 1 GiB (0.35 % of 288 GiB).  full is the
    # default of a node joining a cluster (models/baremetal.py); the node labels say which
    # (node/labels.py:burnin_labels)
    "quick": (1 << 30, 3, 2000, 1 << 30, 1),
    # hbm: best of 3 timed passes per stream kind over 16 GiB, as `gpu-burnin --all` (the
    # SSH / Terraform path) has always run it; 10 passes added ~90 ms for the same number
    "full": (16 << 30, 3, 20000, 0, 3),
}


@dataclass
class Thresholds:
    min_read_frac: float = 0.60
    min_bf16_frac: float = 0.55
    min_fp8_frac: float = 0.55
    # the checksum-verified GEMMs (ops/gemm.py): a fraction of the dense bf16 / fp8 peak
    min_gemm_frac: float = 0.30
    min_gemm_fp8_frac: float = 0.30
    require_gfx950: bool = True
    min_cus: int = MI355X_CUS
    # a compute partition's share of the chip (node/partition.py): scales every throughput
    # floor and the CU minimum; mem_share: its share of the HBM pool it allocates from
    # (sizes the full memtest when partitions of one pool are tested concurrently)
    share: float = 1.0
    mem_share: float = 1.0

    @classmethod
    def for_partition(cls, compute: str = "spx", memory: str = "nps1") -> "Thresholds":
        from ..node.partition import compute_share, memory_share, normalize

        c, m = normalize(compute, memory)
        return cls(min_cus=int(MI355X_CUS * compute_share(c)), share=compute_share(c), mem_share=memory_share(c, m))


@dataclass
class BurninResult:
    device: DeviceInfo
    level: str
    hbm: Dict[str, float] = field(default_factory=dict)
    mfma: Dict[str, Dict[str, float]] = field(default_factory=dict)
    gemm: Dict[str, Any] = field(default_factory=dict)
    gemm_fp8: Dict[str, Any] = field(default_factory=dict)
    memtest: Dict[str, float] = field(default_factory=dict)
    failures: List[str] = field(default_factory=list)
    remeasured: List[str] = field(default_factory=list)  # throughput gates read low and measured again
    phase_ms: Dict[str, float] = field(default_factory=dict)  # wall time of each screen, as run

    @property
    def ok(self) -> bool:
        return not self.failures

    def to_json(self) -> Dict:
        d = asdict(self)
        d["ok"] = self.ok
        return d


@contextlib.contextmanager
def _phase(res: "BurninResult", name: str, dev: int):
    """A burn-in screen: a trace span, and its wall time in ``res.phase_ms``."""
    t0 = time.perf_counter()
    with span(f"burnin.{name}", dev=dev):
        try:
            yield
        finally:
            res.phase_ms[name] = round(res.phase_ms.get(name, 0.0) + (time.perf_counter() - t0) * 1e3, 1)


# --- the burn-in in a child process (node agents) --------------------------------------------
# A node agent's HIP runtime is also where the cluster gate's RCCL communicator starts, and
# starting one loads RCCL's code objects under the runtime's locks: the screens' kernel
# launches in the same process waited behind it, 1.5 s at quick and up to 4 s at full
# (profiles/round5/README.md).  An agent therefore runs each GPU's burn-in in a
# ``gpu-burnin --burnin-child`` process of its own (set_burnin_process): the same
# measurements with the parameters and floors of LEVELS / Thresholds, judged here by the
# same rules (_judge).
_BURNIN_PROCESS = False


def set_burnin_process(on: bool) -> None:
    """Run :func:`run_burnin` in ``gpu-burnin --burnin-child`` processes (node agents)."""
    global _BURNIN_PROCESS
    _BURNIN_PROCESS = bool(on)


def _floors(th: Thresholds) -> Dict[str, float]:
    return {"read": th.min_read_frac * MI355X_HBM_ACHIEVABLE_GBPS * th.share,
            "bf16": th.min_bf16_frac * MI355X_BF16_DENSE_TFLOPS * th.share,
            "fp8": th.min_fp8_frac * MI355X_FP8_DENSE_TFLOPS * th.share,
            "gemm_bf16": th.min_gemm_frac * MI355X_BF16_DENSE_TFLOPS * th.share,
            "gemm_fp8": th.min_gemm_fp8_frac * MI355X_FP8_DENSE_TFLOPS * th.share}


def _judge(res: BurninResult, th: Thresholds, first_bad: Dict[str, Optional[Dict[str, Any]]]) -> BurninResult:
    """The burn-in's verdict from its measurements (in-process or from a child), appended
    to ``res.failures``: arch and CUs, each throughput against its floor, any GEMM run
    with a checksum mismatch (``first_bad``: the first such run per dtype), memtest words."""
    info, fl = res.device, _floors(th)
    if th.require_gfx950 and not info.is_gfx950:
        res.failures.append(f"arch {info.arch} is not gfx950")
    if info.compute_units < th.min_cus:
        res.failures.append(f"{info.compute_units} CUs < {th.min_cus}")
    if res.hbm["read_gbps"] < fl["read"]:
        res.failures.append(f"HBM read {res.hbm['read_gbps']:.0f} GB/s below "
                            f"{th.min_read_frac:.0%} of {MI355X_HBM_ACHIEVABLE_GBPS:.0f}")
    if res.mfma["bf16"]["tflops"] < fl["bf16"]:
        res.failures.append(f"bf16 MFMA {res.mfma['bf16']['tflops']:.0f} TF below "
                            f"{th.min_bf16_frac:.0%} of dense peak")
    if res.mfma["fp8"]["tflops"] < fl["fp8"]:
        res.failures.append(f"fp8 MFMA {res.mfma['fp8']['tflops']:.0f} TF below "
                            f"{th.min_fp8_frac:.0%} of dense peak")
    for dtype, g, frac in (("bf16", res.gemm, th.min_gemm_frac), ("fp8", res.gemm_fp8, th.min_gemm_fp8_frac)):
        name = "GEMM" if dtype == "bf16" else "fp8 GEMM"
        bad = first_bad.get(dtype)
        if bad is not None:  # a mismatch in ANY run fails the GPU
            res.failures.append(f"{name} checksum mismatch: {int(bad['bad_rows'])} rows / "
                                f"{int(bad['bad_columns'])} columns (first at row {int(bad['first_bad_row'])}, "
                                f"column {int(bad['first_bad_column'])})")
        if g["tflops"] < fl[f"gemm_{dtype}"]:
            res.failures.append(f"{name} {g['tflops']:.0f} TF below {frac:.0%} of dense {dtype} peak")
    if res.memtest["errors"]:
        res.failures.append(f"memtest: {res.memtest['errors']} mismatching words")
    return res


# HBM a full span leaves free.  A node agent's cluster-gate communicator allocates its
# buffers (per channel and peer, plus RCCL's device code on every GPU) while a child holds its
# span -- the release waits for the init -- so a node of several GPUs leaves more
# (set_span_headroom; node/agent.py: 4 GiB + 512 MiB per further GPU of the node).
SPAN_HEADROOM = 4 << 30


def set_span_headroom(nbytes: int) -> None:
    global SPAN_HEADROOM
    SPAN_HEADROOM = max(1 << 30, int(nbytes))


def _burnin_child(dev: int, level: str, th: Thresholds, timeout: float = 900.0) -> BurninResult:
    """:func:`run_burnin` in a ``gpu-burnin --burnin-child`` process (see above): the span
    memtest's memory is released by the child after its verdict (joined by :func:`wait_frees`)."""
    from . import gemm

    hbm_bytes, hbm_iters, mfma_iters, mt_bytes, mt_passes = LEVELS[level]
    m, n, k, reps = gemm.SCREEN_SIZES[level]
    fl = _floors(th)
    exe = _burnin_exe()
    _lib().tkp_wait_frees()
    _wait_span_children(dev)  # this device's previous span is released before this one allocates
    argv = [exe, "--burnin-child", "--device", str(int(dev)), "--hbm-bytes", str(hbm_bytes),
            "--hbm-iters", str(hbm_iters), "--mfma-iters", str(mfma_iters), "--gemm", f"{m},{n},{k},{reps}",
            "--memtest-bytes", str(mt_bytes), "--memtest-passes", str(mt_passes),
            "--span-headroom", str(int(SPAN_HEADROOM)), "--span-chunk", str(SPAN_CHILD_CHUNK),
            "--min-read-gbps", f"{fl['read']:.3f}", "--min-bf16-tflops", f"{fl['bf16']:.3f}",
            "--min-fp8-tflops", f"{fl['fp8']:.3f}", "--min-gemm-tflops", f"{fl['gemm_bf16']:.3f}",
            "--min-gemm-fp8-tflops", f"{fl['gemm_fp8']:.3f}"]
    doc, process_ms = _child_verdict(argv, dev, timeout, "burn-in")
    if not doc.get("ok"):
        raise ProbeError(f"burn-in (gpu-burnin --burnin-child): {doc.get('error', 'failed')}")
    try:
        i = doc["info"]
        info = DeviceInfo(index=dev, name=str(i["name"]), arch=str(i["arch"]), compute_units=int(i["compute_units"]),
                          wavefront_size=int(i["wavefront_size"]), clock_mhz=int(i["clock_khz"]) / 1000.0,
                          total_mem_gib=int(i["total_mem"]) / 2 ** 30, free_mem_gib=int(i["free_mem"]) / 2 ** 30,
                          l2_bytes=int(i["l2_bytes"]),
                          pci_bus_id=f"{int(i['pci_domain']):04x}:{int(i['pci_bus']):02x}:{int(i['pci_device']):02x}.0")
        res = BurninResult(info, level, hbm={k2: float(v) for k2, v in doc["hbm"].items()},
                           mfma={"bf16": dict(doc["bf16"]), "fp8": dict(doc["fp8"])},
                           gemm=dict(doc["gemm"], m=m, n=n, k=k, dtype="bf16"),
                           gemm_fp8=dict(doc["gemm_fp8"], m=m, n=n, k=k, dtype="fp8"),
                           memtest=dict(doc["memtest"], free_ms=0.0, process_ms=process_ms),
                           remeasured=list(doc.get("remeasured") or []),
                           phase_ms=dict(doc.get("phase_ms") or {}))
        for g in (res.gemm, res.gemm_fp8):
            g["ok"] = not (g["bad_columns"] or g["bad_rows"])
        res.memtest["errors"] = int(res.memtest["errors"])
        res.phase_ms["process"] = process_ms
        return _judge(res, th, {"bf16": doc.get("gemm_first_bad"), "fp8": doc.get("gemm_fp8_first_bad")})
    except (KeyError, TypeError, ValueError) as exc:
        raise ProbeError(f"burn-in: {exe} gave no burn-in verdict ({type(exc).__name__}: {exc})") from None


def run_burnin(dev: int, level: str = "quick", thresholds: Optional[Thresholds] = None) -> BurninResult:
    th = thresholds or Thresholds()
    # partitions of one HBM pool (mem_share < 1) burn in in-process: they share the pool
    if level != "off" and _BURNIN_PROCESS and th.mem_share >= 1.0:
        try:
            return _burnin_child(dev, level, th)
        except native.NativeUnavailable:
            pass  # no usable gpu-burnin here: the same burn-in in this process
    with _InProcess():
        return _run_burnin_here(dev, level, th)


def _run_burnin_here(dev: int, level: str, th: "Thresholds") -> BurninResult:
    """:func:`run_burnin` in this process."""
    info = device_info(dev)
    res = BurninResult(info, level)
    if level == "off":
        return res
    hbm_bytes, hbm_iters, mfma_iters, mt_bytes, mt_passes = LEVELS[level]
    # Throughput gates are re-measured (best of up to REMEASURE + 1 runs) before they fail
    # a node: a short kernel that overlapped other GPU work on the node (a previous
    # communicator's teardown, another process) reads low once; a slow GPU reads low every
    # time.  Correctness results (checksums, memtest words) are never retried away.
    def best(measure, value, floor, what):
        r = measure()
        for _ in range(REMEASURE):
            if value(r) >= floor:
                break
            again = measure()
            res.remeasured.append(what)
            if value(again) > value(r):
                r = again
        return r

    fl = _floors(th)
    with _phase(res, "hbm", dev):
        res.hbm = best(lambda: hbm_bandwidth(dev, hbm_bytes, hbm_iters), lambda r: r["read_gbps"], fl["read"], "hbm")
    with _phase(res, "mfma_bf16", dev):
        res.mfma["bf16"] = best(lambda: mfma_peak(dev, "bf16", mfma_iters), lambda r: r["tflops"], fl["bf16"],
                                "mfma_bf16")
    with _phase(res, "mfma_fp8", dev):
        res.mfma["fp8"] = best(lambda: mfma_peak(dev, "fp8", mfma_iters // 2), lambda r: r["tflops"], fl["fp8"],
                               "mfma_fp8")
    from . import gemm

    m, n, k, reps = gemm.SCREEN_SIZES[level]
    first_bad: Dict[str, Optional[Dict[str, Any]]] = {}
    for dtype in ("bf16", "fp8"):
        runs = []

        def screen_once(dtype=dtype, runs=runs):
            g = gemm.screen(dev, m, n, k, reps, dtype=dtype)
            runs.append(g)
            return g

        with _phase(res, f"gemm_{dtype}", dev):
            g = best(screen_once, lambda r: r.tflops, fl[f"gemm_{dtype}"], f"gemm_{dtype}")
        if dtype == "bf16":
            res.gemm = g.to_json()
        else:
            res.gemm_fp8 = g.to_json()
        bad = next((r for r in runs if not r.ok), None)  # a mismatch in ANY run fails the GPU
        first_bad[dtype] = bad.to_json() if bad is not None else None
    with _phase(res, "memtest", dev):
        if mt_bytes:
            res.memtest = memtest(dev, mt_bytes, mt_passes)
            res.memtest.update(bytes=mt_bytes, hbm_bytes=int(info.total_mem_gib * (1 << 30)))
        elif th.mem_share < 1.0:
            # concurrent partitions share one pool: each holds its share of what is free
            # (the arena's buffers are freed first: they are memtested, not left beside it)
            release_scratch(dev)
            headroom = max(512 << 20, int((4 << 30) * th.mem_share))
            span_bytes = max(1 << 30, int(free_bytes(dev) * th.mem_share) - headroom)
            res.memtest = _span(dev, span_bytes, mt_passes)
        else:
            res.memtest = _span(dev, 0, mt_passes)
    return _judge(res, th, first_bad)


def prealloc_scratch(dev: int, level: str = "quick") -> int:
    """Allocate the burn-in arena of ``level`` on ``dev`` now (turns the cache on).

    A long-lived node agent calls this at startup, so a bring-up's burn-in streams
    and memtests through resident buffers instead of a hipMalloc/hipFree of GiBs
    per run; measured on MI355X, those big allocations intermittently stall for
    0.1-0.8 s when they follow recent frees.  Returns the bytes held."""
    if level not in LEVELS:
        return 0
    hbm_bytes, _, _, mt_bytes, _ = LEVELS[level]
    mt_bytes = mt_bytes or (1 << 30)  # the span memtest allocates its own chunks
    lib = _lib()
    lib.tkp_set_scratch_cache(1)
    rc = lib.tkp_prealloc_scratch(dev, ctypes.c_size_t(hbm_bytes), ctypes.c_size_t(mt_bytes))
    _check(rc, f"prealloc_scratch(dev {dev})")
    return max(hbm_bytes, mt_bytes) + hbm_bytes  # the memtest shares the first stream buffer


def set_scratch_cache(on: bool) -> None:
    """Keep the burn-in's multi-GiB buffers allocated between runs (long-lived agents)."""
    _lib().tkp_set_scratch_cache(1 if on else 0)


def release_scratch(dev: Optional[int] = None) -> int:
    """Free cached burn-in buffers (of ``dev`` only, when given); returns the bytes released."""
    if dev is not None:
        return int(_lib().tkp_release_scratch_dev(dev))
    return int(_lib().tkp_release_scratch())
