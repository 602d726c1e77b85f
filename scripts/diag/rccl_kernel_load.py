#!/usr/bin/env python3
"""Diagnostic (not product code): what does loading RCCL's kernels cost, kernel by kernel?

In a fresh process: hipFuncGetAttributes on every kernel handle librccl exports (the
calls RCCL's own ``kernels`` init phase makes), timed one by one, then a 1-rank
communicator init.  If the per-kernel loads add up to the ~1.7 s of a first init and the
init afterwards is fast, an agent can pay the load at start-up through public API.
"""

import ctypes
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main() -> None:
    lib_path = "/opt/rocm/lib/librccl.so.1"
    syms = []
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True, text=True, check=True).stdout
    for line in out.splitlines():
        parts = line.split()
        if len(parts) == 3 and parts[1] == "D" and ("Kernel" in parts[2]):
            syms.append(parts[2])
    t0 = time.perf_counter()
    rccl = ctypes.CDLL(lib_path, mode=ctypes.RTLD_GLOBAL)
    hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    hip.hipSetDevice(0)
    hip.hipFree(None)
    t_init = (time.perf_counter() - t0) * 1e3
    attr = ctypes.create_string_buffer(1024)
    times = []
    for s in syms:
        fn = ctypes.c_void_p.in_dll(rccl, s)
        addr = ctypes.addressof(fn)
        t = time.perf_counter()
        rc = hip.hipFuncGetAttributes(attr, ctypes.c_void_p(addr))
        times.append((s, round((time.perf_counter() - t) * 1e3, 2), rc))
    total = sum(t for _, t, _ in times)
    from triton_kubernetes_amd.ops import rccl as tk

    t = time.perf_counter()
    g = tk.GateComm(tk.unique_id(), 1, 0, [0], blocking=True)
    init_ms = (time.perf_counter() - t) * 1e3
    res = g.sweep([1 << 20], iters=2, warmup=1, async_teardown=True)
    tk.drain()
    slow = sorted(times, key=lambda x: -x[1])[:12]
    print(json.dumps({"hip_init_ms": round(t_init, 1), "kernels": len(syms), "load_total_ms": round(total, 1),
                      "slowest": slow, "rc_nonzero": [x for x in times if x[2]][:5],
                      "init_after_ms": round(init_ms, 1), "sweep_ok": res.ok}), flush=True)


if __name__ == "__main__":
    main()
