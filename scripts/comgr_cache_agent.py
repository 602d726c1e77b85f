"""GPU box: the agent's first RCCL communicator init (libtk_rccl through ctypes, /opt/rocm's
HIP runtime, as the node agent loads it) in fresh processes, with comgr's cache off, cold and
warm.  One JSON line per process."""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, os, sys, time
t0 = time.perf_counter()
sys.path.insert(0, os.environ["TK_ROOT"])
from triton_kubernetes_amd.ops import native, rccl
t1 = time.perf_counter()
uid = rccl.unique_id()
t2 = time.perf_counter()
g = rccl.GateComm(uid, 1, 0, [0], blocking=True)
t3 = time.perf_counter()
res = g.sweep([1 << 20], iters=3, warmup=1)
t4 = time.perf_counter()
print(json.dumps({"import_ms": round((t1 - t0) * 1e3, 1), "uid_ms": round((t2 - t1) * 1e3, 1),
                  "init_ms": round((t3 - t2) * 1e3, 1), "sweep_ms": round((t4 - t3) * 1e3, 1), "ok": res.ok}))
sys.stdout.flush()
rccl.exit_now(0)
"""
cache = tempfile.mkdtemp(prefix="tk-comgr-agent-")
for tag, env in [("off", {"AMD_COMGR_CACHE": "0"}), ("cold", {"AMD_COMGR_CACHE": "1", "AMD_COMGR_CACHE_DIR": cache}),
                 ("warm", {"AMD_COMGR_CACHE": "1", "AMD_COMGR_CACHE_DIR": cache}),
                 ("warm2", {"AMD_COMGR_CACHE": "1", "AMD_COMGR_CACHE_DIR": cache}), ("off2", {"AMD_COMGR_CACHE": "0"})]:
    t0 = time.monotonic()
    out = subprocess.run(["timeout", "-k", "10", "120", sys.executable, "-c", CHILD], capture_output=True, text=True,
                         env=dict(os.environ, TK_ROOT=ROOT, TK_HIP_RUNTIME="system", **env))
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    print(json.dumps({"tag": tag, "rc": out.returncode, "wall_ms": round((time.monotonic() - t0) * 1e3, 1),
                      "child": json.loads(lines[-1]) if lines else out.stderr[-400:]}), flush=True)
