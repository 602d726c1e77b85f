#!/usr/bin/env python3
"""Where a long-lived process's host memory goes per gate: RSS (after ``malloc_trim``) and
malloc's in-use bytes around N repetitions of (a) a HIP stream + two events created and
destroyed, (b) a one-rank gate communicator (``ops/rccl.GateComm``) initialised, swept and
torn down.  One JSON line per phase.

    python scripts/leak_probe.py [--n 50]
"""

import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _MallInfo2(ctypes.Structure):
    _fields_ = [(n, ctypes.c_size_t) for n in ("arena", "ordblks", "smblks", "hblks", "hblkhd", "usmblks",
                                               "fsmblks", "uordblks", "fordblks", "keepcost")]


_libc = ctypes.CDLL(None)
_libc.mallinfo2.restype = _MallInfo2


def held() -> dict:
    _libc.malloc_trim(0)
    mi = _libc.mallinfo2()
    with open("/proc/self/statm", encoding="ascii") as fh:
        rss = int(fh.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")
    return {"rss_mib": round(rss / 2 ** 20, 2), "malloc_mib": round((mi.uordblks + mi.hblkhd) / 2 ** 20, 2)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50)
    args = ap.parse_args()
    from triton_kubernetes_amd.ops import native, rccl

    native.runtime_dir()
    rccl.unique_id()  # loads libtk_rccl.so and, through it, the runtime's libamdhip64.so.7
    hip = ctypes.CDLL("libamdhip64.so.7")  # the copy already loaded (same soname)
    s, e0, e1 = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()

    def streams():
        for _ in range(args.n):
            assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
            assert hip.hipEventCreate(ctypes.byref(e0)) == 0 and hip.hipEventCreate(ctypes.byref(e1)) == 0
            hip.hipEventDestroy(e0)
            hip.hipEventDestroy(e1)
            hip.hipStreamDestroy(s)

    def gates():
        for _ in range(args.n):
            g = rccl.GateComm(rccl.unique_id(), 1, 0, [0], blocking=False, prealloc_bytes=4 << 20)
            assert g.sweep([1 << 20, 4 << 20], iters=2, warmup=1, async_teardown=False).ok
        rccl.drain()

    hip.hipSetDevice(0)
    streams()  # warm-up of each phase: first-use costs are not growth
    gates()
    for name, fn in (("stream+2 events", streams), ("one-rank gate", gates)):
        before = held()
        fn()
        after = held()
        print(json.dumps({"phase": name, "n": args.n, "before": before, "after": after,
                          "rss_kib_per_rep": round((after["rss_mib"] - before["rss_mib"]) * 1024 / args.n, 1),
                          "malloc_kib_per_rep": round((after["malloc_mib"] - before["malloc_mib"]) * 1024 / args.n, 1)}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
