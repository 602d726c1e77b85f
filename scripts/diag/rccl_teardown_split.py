#!/usr/bin/env python3
"""Diagnostic (not product code): where a gate communicator's ~0.5 s teardown goes.

Each variant runs in a fresh child process: a 1-rank communicator (blocking init), one
verified sweep with a synchronous teardown, three times; the child prints the teardown's
split (sweep-buffer frees vs ``ncclCommDestroy``/``ncclCommAbort``, from
``tkr_last_teardown_ms``).  One JSON line per variant.
"""

import ctypes
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

VARIANTS = {
    "destroy": {},
    "abort": {"TK_TEARDOWN_ABORT": "1"},
    "destroy_2": {},
}


def child() -> None:
    from triton_kubernetes_amd.ops import rccl

    lib = rccl._lib()
    lib.tkr_last_teardown_ms.restype = ctypes.c_double
    lib.tkr_last_teardown_ms.argtypes = [ctypes.c_int]
    if os.environ.get("TK_TEARDOWN_ABORT") == "1":
        lib.tkr_set_teardown_abort(1)
    runs = []
    for _ in range(3):
        g = rccl.GateComm(rccl.unique_id(), 1, 0, [0], blocking=True)
        t = time.perf_counter()
        r = g.sweep([1 << 20, 64 << 20], iters=3, warmup=1, async_teardown=False)
        runs.append({"ok": r.ok, "sweep_call_ms": round((time.perf_counter() - t) * 1e3, 1),
                     "teardown_ms": r.phase_ms.get("teardown"),
                     "free_ms": round(lib.tkr_last_teardown_ms(0), 2),
                     "comm_ms": round(lib.tkr_last_teardown_ms(1), 2)})
    print(json.dumps({"runs": runs}), flush=True)


def parent() -> None:
    for name in sys.argv[1:] or list(VARIANTS):
        env = dict(os.environ, **VARIANTS[name])
        proc = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True,
                              text=True, timeout=240, check=False)
        line = next((ln for ln in proc.stdout.splitlines() if ln.startswith("{")), "{}")
        doc = {"variant": name, "rc": proc.returncode, **json.loads(line)}
        if proc.returncode:
            doc["stderr"] = proc.stderr[-1500:]
        print(json.dumps(doc), flush=True)
        if proc.returncode not in (0, 1):
            break


if __name__ == "__main__":
    child() if "--child" in sys.argv else parent()
