#!/usr/bin/env python3
"""Which threads of a process stall while an RCCL communicator is created / destroyed?

Diagnosis for the occasional 100-200 ms bring-up stalls seen in ``bench.py`` while a
previous gate's communicator teardown runs in the background.  Three monitor threads
record their worst scheduling gaps:

* ``py``    — pure Python, ``time.sleep(0.5 ms)`` loop (GIL / scheduler stalls);
* ``mmap``  — allocates and touches a fresh 4 MiB buffer each iteration (glibc mmaps it:
              stalls here mean the process's mmap lock is held);
* ``gpu``   — a tiny torch kernel + synchronize on cuda:0 (GPU queue stalls / evictions).

Meanwhile the RCCL work (blocking init -> verified sweep -> destroy, 1 rank) runs either
in this process (``--where self``) or in a child process (``--where child``), with
pauses in between so each window is separable.  Prints one JSON document.
"""

import argparse
import json
import os
import subprocess
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def rccl_cycles(n: int, pause: float, sizes):
    from triton_kubernetes_amd.ops import rccl

    out = []
    for _ in range(n):
        uid = rccl.unique_id()
        t0 = time.time()
        g = rccl.GateComm(uid, 1, 0, [0], blocking=True)
        t1 = time.time()
        res = g.sweep(sizes, iters=3, warmup=1, async_teardown=False)
        t2 = time.time()
        out.append({"init": [t0, t1], "sweep_teardown": [t1, t2], "phases": res.phase_ms, "ok": res.ok})
        time.sleep(pause)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--where", choices=["self", "child", "worker"], default="self")
    ap.add_argument("--cycles", type=int, default=5)
    ap.add_argument("--pause", type=float, default=0.3)
    ap.add_argument("--threshold-ms", type=float, default=8.0)
    args = ap.parse_args()
    sizes = [1 << 20, 4 << 20]

    if args.where == "worker":  # child side
        print(json.dumps(rccl_cycles(args.cycles, args.pause, sizes)))
        return 0

    import torch

    x = torch.zeros(1024, device="cuda:0")
    torch.cuda.synchronize()
    stop = threading.Event()
    gaps = {"py": [], "mmap": [], "gpu": []}
    thr = args.threshold_ms / 1e3

    def mon(name, body):
        last = time.time()
        while not stop.is_set():
            body()
            now = time.time()
            if now - last > thr:
                gaps[name].append([last, round((now - last) * 1e3, 2)])
            last = now

    def py_body():
        time.sleep(0.0005)

    def mmap_body():
        b = bytearray(4 << 20)
        b[:: 4096] = b"\x01" * len(b[:: 4096])
        time.sleep(0.0005)

    def gpu_body():
        x.add_(1.0)
        torch.cuda.synchronize()
        time.sleep(0.0005)

    ts = [threading.Thread(target=mon, args=(n, f), daemon=True)
          for n, f in (("py", py_body), ("mmap", mmap_body), ("gpu", gpu_body))]
    for t in ts:
        t.start()
    time.sleep(0.5)
    t_start = time.time()
    if args.where == "self":
        cycles = rccl_cycles(args.cycles, args.pause, sizes)
    else:
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--where", "worker", "--cycles",
                            str(args.cycles), "--pause", str(args.pause)], capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            print(p.stderr[-3000:], file=sys.stderr)
            return p.returncode
        cycles = json.loads(p.stdout.strip().splitlines()[-1])
    time.sleep(0.3)
    stop.set()
    for t in ts:
        t.join()

    def where(ts_):
        for i, c in enumerate(cycles):
            if c["init"][0] <= ts_ <= c["init"][1]:
                return f"init{i}"
            if c["sweep_teardown"][0] <= ts_ <= c["sweep_teardown"][1]:
                return f"sweep_teardown{i}"
        return "idle"

    report = {"where": args.where, "t_start": t_start,
              "cycles": [{"init_ms": round((c["init"][1] - c["init"][0]) * 1e3, 1),
                          "sweep_teardown_ms": round((c["sweep_teardown"][1] - c["sweep_teardown"][0]) * 1e3, 1),
                          "phases": c["phases"]} for c in cycles],
              "gaps": {k: [{"at_ms": round((g[0] - t_start) * 1e3, 1), "ms": g[1], "during": where(g[0])}
                           for g in v] for k, v in gaps.items()}}
    print(json.dumps(report))
    return 0


if __name__ == "__main__":
    sys.exit(main())
