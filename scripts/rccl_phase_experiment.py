#!/usr/bin/env python3
"""RCCL gate phase breakdown (init / alloc / sweep / teardown), sync vs async teardown."""
import json
import sys
import time
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triton_kubernetes_amd.ops import rccl  # noqa: E402

for mode in (False, True):
    rccl.set_async_teardown(mode)
    for i in range(4):
        t0 = time.perf_counter()
        r = rccl.sweep_rank(0, 1, rccl.unique_id(), 0, [1 << 20, 64 << 20], iters=5, warmup=2)
        print(json.dumps({"async_teardown": mode, "run": i, "total_ms": round((time.perf_counter() - t0) * 1e3, 1),
                          "phases": r.phase_ms, "ok": r.ok}), flush=True)
print(json.dumps({"drained": rccl.drain()}))
