#!/usr/bin/env python3
"""The cluster gate communicator's device footprint on this box.

A full burn-in's span leaves ``probe.SPAN_HEADROOM`` free per GPU while the gate's
communicator initialises; this measures what that init takes (``tk_rccl_probe.hip``: this
process's VRAM -- or, inside a PID namespace, the device's used memory -- around the grouped
init, then around the preallocated sweep buffers), for the sizes the readiness gate uses.  One JSON line per case; run in a fresh process each (RCCL's
device code loads once per process and counts in the first init only).

    python scripts/gate_footprint.py [--prealloc-mib 64] [--repeat 3] [--ndev N]

``--ndev N``: one grouped communicator over devices 0..N-1 in this process, the node agent's
shape -- on an 8-GPU node, the per-peer part of the footprint this one-GPU pool cannot show.
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--prealloc-mib", type=int, default=64)
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--ndev", type=int, default=1, help="GPUs of the communicator (devices 0..N-1)")
    args = ap.parse_args()
    from triton_kubernetes_amd.ops import native, probe, rccl

    free0 = probe.free_bytes(0)
    for i in range(args.repeat):
        t0 = time.perf_counter()
        devs = list(range(args.ndev))
        g = rccl.GateComm(rccl.unique_id(), len(devs), 0, devs, blocking=False,
                          prealloc_bytes=args.prealloc_mib << 20)
        res = g.sweep([1 << 20, args.prealloc_mib << 20], iters=3, warmup=1, async_teardown=False)
        print(json.dumps({"case": i, "first_in_process": i == 0, "ok": res.ok, "world": res.world,
                          "prealloc_mib": args.prealloc_mib, "init_total_ms": res.phase_ms.get("init_total"),
                          "footprint_mib": res.phase_ms.get("footprint_mib"),
                          "footprint_total_mib": res.phase_ms.get("footprint_total_mib"),
                          "footprint_kind": res.phase_ms.get("footprint_kind"),
                          "free_gib_before_any": round(free0 / 2 ** 30, 2),
                          "free_gib_after": round(probe.free_bytes(0) / 2 ** 30, 2),
                          "wall_ms": round((time.perf_counter() - t0) * 1e3, 1),
                          "runtime": native.runtime_dir(), "preload": rccl.preload_report()}), flush=True)
    rccl.drain()
    return 0


if __name__ == "__main__":
    sys.exit(main())
