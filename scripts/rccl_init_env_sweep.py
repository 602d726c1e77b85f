#!/usr/bin/env python3
"""RCCL warm communicator-init cost (1 rank, torch's RCCL, as in bench.py) under env variants.

The sampler (scripts/rccl_init_sampler.py) put ~15 of the ~43 ms of a warm init in a large
host memcpy on RCCL's init thread and most of the rest in waits; these variants probe
the knobs that size init-time host/device structures.  Each variant is a fresh process:
six blocking inits (+64 MiB prealloc, as the agent's gate does), each followed by a 1 MiB
sweep and a synchronous teardown; the median of inits 2-6 is reported.  JSON lines.
"""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, statistics, sys, time
sys.path.insert(0, %r)
import torch
torch.zeros(1, device="cuda:0"); torch.cuda.synchronize()
from triton_kubernetes_amd.ops import rccl
ms = []
for i in range(6):
    uid = rccl.unique_id()
    t0 = time.perf_counter()
    g = rccl.GateComm(uid, 1, 0, [0], blocking=True, prealloc_bytes=64 << 20)
    ms.append((time.perf_counter() - t0) * 1e3)
    r = g.sweep([1 << 20], iters=2, warmup=1, async_teardown=False)
    assert r.ok
print(json.dumps({"init_ms": [round(x, 1) for x in ms], "median_warm_ms": round(statistics.median(ms[1:]), 1),
                  "teardown_ms": r.phase_ms.get("teardown")}))
"""

VARIANTS = {
    "baseline": {},
    "work_fifo_64k": {"NCCL_WORK_FIFO_BYTES": str(64 << 10)},
    "work_fifo_depth_1k": {"NCCL_WORK_FIFO_DEPTH": "1024"},
    "buffsize_1m": {"NCCL_BUFFSIZE": str(1 << 20)},
    "max_nchannels_1": {"NCCL_MAX_NCHANNELS": "1"},
    "runtime_connect_0": {"NCCL_RUNTIME_CONNECT": "0"},
    "runtime_connect_1": {"NCCL_RUNTIME_CONNECT": "1"},
    "proto_simple_ring": {"NCCL_PROTO": "Simple", "NCCL_ALGO": "Ring"},
    "cumem_0": {"NCCL_CUMEM_ENABLE": "0"},
    "dmabuf_0": {"NCCL_DMABUF_ENABLE": "0"},
    "no_register": {"NCCL_LOCAL_REGISTER": "0", "NCCL_GRAPH_REGISTER": "0"},
    "proxy_shm_small": {"NCCL_PROXY_APPEND_BATCH_SIZE": "4", "NCCL_CREATE_THREAD_CONTEXT": "0"},
    "msccl_off": {"RCCL_MSCCL_ENABLE": "0", "RCCL_MSCCLPP_ENABLE": "0"},
    "rccl_kernel_trace_off": {"RCCL_KERNEL_COLL_TRACE_ENABLE": "0", "NCCL_COLLNET_ENABLE": "0", "NCCL_NVLS_ENABLE": "0"},
    # glibc keeps the init's ~100 MiB topology-XML buffers in the heap instead of fresh mmaps
    # (a fresh mapping page-faults on first touch; a reused heap chunk does not)
    "malloc_heap": {"MALLOC_MMAP_THRESHOLD_": str(1 << 30), "MALLOC_TRIM_THRESHOLD_": str(4 << 30)},
    "malloc_heap_tunables": {"GLIBC_TUNABLES": f"glibc.malloc.mmap_threshold={1 << 30}:glibc.malloc.trim_threshold={4 << 30}"},
}


def main() -> int:
    names = sys.argv[1:] or list(VARIANTS)
    for name in names:
        e = dict(os.environ)
        e.update(VARIANTS[name])
        proc = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=e, capture_output=True, text=True, timeout=240)
        lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
        rec = {"variant": name, "env": VARIANTS[name], "rc": proc.returncode}
        if lines:
            rec.update(json.loads(lines[-1]))
        else:
            rec["stderr"] = proc.stderr[-500:]
        print(json.dumps(rec), flush=True)
        if proc.returncode not in (0, 1):
            return proc.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
