"""One fresh process: the agent's first RCCL communicator (1 rank, libtk_rccl via ctypes on
/opt/rocm's runtime), timed.  For profiling the init (scripts/prof_rccl_init.sh)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
t0 = time.perf_counter()
from triton_kubernetes_amd.ops import rccl  # noqa: E402

uid = rccl.unique_id()
t1 = time.perf_counter()
g = rccl.GateComm(uid, 1, 0, [0], blocking=True)
t2 = time.perf_counter()
res = g.sweep([1 << 20], iters=3, warmup=1)
print(json.dumps({"uid_ms": round((t1 - t0) * 1e3, 1), "init_ms": round((t2 - t1) * 1e3, 1), "ok": res.ok}),
      flush=True)
