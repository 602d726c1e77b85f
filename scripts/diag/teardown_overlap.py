#!/usr/bin/env python3
"""Diagnostic (not product code): does a communicator teardown disturb a burn-in next to it?

A resident agent drains the previous create's RCCL teardown (~0.48 s, all of it inside
``ncclCommDestroy``: profiles/round2/rccl_teardown_split.jsonl) before its next burn-in, so
no throughput gate is timed next to it.  This measures whether that wait is needed: in one
warm process, 6 rounds of {gate init + sweep with async teardown, then at once a quick
burn-in}, alternating "overlap" (burn-in while the teardown runs) and "drained" (burn-in
after ``rccl.drain()``).  Per round: burn-in gate readings and any re-measured gates.
"""

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main() -> None:
    from triton_kubernetes_amd.ops import probe, rccl

    probe.prealloc_scratch(0, "quick")
    probe.run_burnin(0, "quick")  # warm: code objects, queues, arena
    for i in range(6):
        mode = "overlap" if i % 2 == 0 else "drained"
        g = rccl.GateComm(rccl.unique_id(), 1, 0, [0], blocking=True)
        r = g.sweep([1 << 20, 64 << 20], iters=3, warmup=1, async_teardown=True)
        t = time.perf_counter()
        if mode == "drained":
            rccl.drain()
        wait_ms = round((time.perf_counter() - t) * 1e3, 1)
        t = time.perf_counter()
        b = probe.run_burnin(0, "quick")
        print(json.dumps({"round": i, "mode": mode, "gate_ok": r.ok, "drain_wait_ms": wait_ms,
                          "burnin_ms": round((time.perf_counter() - t) * 1e3, 1), "ok": b.ok,
                          "failures": b.failures, "remeasured": b.remeasured,
                          "hbm_read_gbps": round(b.hbm.get("read_gbps", 0.0)),
                          "mfma_bf16_tf": round(b.mfma["bf16"]["tflops"]), "mfma_fp8_tf": round(b.mfma["fp8"]["tflops"]),
                          "gemm_bf16_tf": round(b.gemm.get("tflops", 0.0)),
                          "gemm_fp8_tf": round(b.gemm_fp8.get("tflops", 0.0))}), flush=True)
    rccl.drain()


if __name__ == "__main__":
    main()
