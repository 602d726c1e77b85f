#!/usr/bin/env python3
"""Where does a warm RCCL communicator init (~45 ms, 1 rank) spend its time?

Samples every thread of this process with ``scripts/native/tk_sampler.so`` while
``GateComm(blocking=True)`` runs, for several warm inits, then aggregates: per thread,
the leaf frame and the first HIP/HSA API frame of each sample.  Prints a JSON summary;
raw samples go to gpurun_out/sampler/.
"""

import collections
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import torch

    torch.zeros(1, device="cuda:0")
    torch.cuda.synchronize()
    from triton_kubernetes_amd.ops import rccl

    lib = ctypes.CDLL(os.path.join(HERE, "native", "tk_sampler.so"))
    lib.tks_start.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.tks_stop.argtypes = [ctypes.c_char_p]
    out_dir = os.path.join(os.path.dirname(HERE), "gpurun_out", "sampler")
    os.makedirs(out_dir, exist_ok=True)
    interval = int(os.environ.get("TKS_INTERVAL_US", "250"))
    runs = []
    for i in range(7):
        uid = rccl.unique_id()
        sample = i >= 2  # two warm-up inits first
        path = os.path.join(out_dir, f"init{i}.txt")
        if sample:
            assert lib.tks_start(0, interval) == 0
        t0 = time.perf_counter()
        g = rccl.GateComm(uid, 1, 0, [0], blocking=True)
        init_ms = (time.perf_counter() - t0) * 1e3
        n = lib.tks_stop(path.encode()) if sample else 0
        g.sweep([1 << 20], iters=2, warmup=1, async_teardown=False)
        runs.append({"i": i, "init_ms": round(init_ms, 2), "samples": n})

    # aggregate sampled runs
    leaf = collections.Counter()
    api = collections.Counter()
    per_tid = collections.Counter()
    for i in range(2, 7):
        for line in open(os.path.join(out_dir, f"init{i}.txt")):
            tid, _, stack = line.strip().partition(" ")
            frames = stack.split(";") if stack else []
            if not frames:
                continue
            # skip idle threads: leaf in a wait with no RCCL frame on the stack
            rcclish = any("rccl" in f for f in frames)
            per_tid[(tid, rcclish)] += 1
            if not rcclish:
                continue
            leaf[frames[0].split("+")[0]] += 1
            first_api = next((f.split("+")[0] for f in frames
                              if f.startswith(("libamdhip64", "libhsa-runtime64", "libc.so", "libpthread"))
                              and "!?" not in f), "none")
            outer = next((f.split("+")[0] for f in reversed(frames) if f.startswith("libamdhip64")), "")
            api[first_api + (" <= " + outer if outer and outer != first_api else "")] += 1
    summary = {"runs": runs, "interval_us": interval,
               "rccl_thread_samples": sum(leaf.values()),
               "threads": {f"{k[0]}{'*' if k[1] else ''}": v for k, v in per_tid.most_common(20)},
               "leaf": leaf.most_common(30), "api": api.most_common(30)}
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
