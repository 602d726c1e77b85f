#!/usr/bin/env python3
"""Diagnostic (not product code): a fresh process's first quick burn-in vs its second.

A cold agent's burn-in step reads ~130 ms where a resident agent's reads ~18 ms
(profiles/round2/rccl_slim_ab.md).  Each variant runs in a fresh child that does what the
agent does at start (native libraries, HIP init, burn-in arena), then times
``run_burnin(0, "quick")`` twice, per burn-in span (hbm, mfma, gemm, memtest).  With
``TK_BURNIN_GATE=1`` a 1-rank RCCL communicator init runs on its own thread during the first
burn-in, as the pipelined gate does in a real create.
"""

import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

VARIANTS = {
    "alone": {},
    "with_gate": {"TK_BURNIN_GATE": "1"},
    "alone_2": {},
    "with_gate_2": {"TK_BURNIN_GATE": "1"},
}


def child() -> None:
    t0 = time.perf_counter()
    from triton_kubernetes_amd.ops import probe, rccl
    from triton_kubernetes_amd.utils.trace import TRACER

    rccl._lib()
    probe._lib()
    probe.device_count()
    probe.prealloc_scratch(0, "quick")
    start_ms = round((time.perf_counter() - t0) * 1e3, 1)
    gate = None
    if os.environ.get("TK_BURNIN_GATE") == "1":
        gate = rccl.GateComm(rccl.unique_id(), 1, 0, [0], blocking=False)
    out = {"start_ms": start_ms, "runs": []}
    for _ in range(2):
        TRACER.reset()
        t = time.perf_counter()
        res = probe.run_burnin(0, "quick")
        total = round((time.perf_counter() - t) * 1e3, 1)
        spans = {s["name"]: round(s["duration"] * 1e3, 1) for s in TRACER.report()["spans"]}
        out["runs"].append({"ok": res.ok, "total_ms": total, "spans": spans, "remeasured": res.remeasured})
    if gate is not None:
        r = gate.sweep([1 << 20], iters=2, warmup=1, async_teardown=False)
        out["gate"] = {"ok": r.ok, "init_total_ms": r.phase_ms.get("init_total")}
    print(json.dumps(out), flush=True)


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
