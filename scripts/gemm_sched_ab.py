#!/usr/bin/env python3
"""A/B of the bf16 GEMM main loops (``ops/gemm.py:SCHEDULES``) in one process: bitwise
agreement of their fp32 outputs, then kernel time of each (fp32 C, which every loop
writes), interleaved over rounds (median; the clock drifts under sustained load).  One JSON
line per size.  ``profiles/round6/gemm_four_wave_ab.jsonl`` is this script's output for a
four-wave (4 x 128x128, one wave per SIMD) loop that was measured and dropped.

    python scripts/gemm_sched_ab.py [--sizes 4096,8192] [--schedules staggered,single-barrier]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from triton_kubernetes_amd.ops import gemm  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,8192")
    ap.add_argument("--schedules", default="staggered,single-barrier")
    ap.add_argument("--rounds", type=int, default=7)
    args = ap.parse_args()
    scheds = args.schedules.split(",")
    g = torch.Generator(device="cuda").manual_seed(1)
    for m, n, k in ((256, 256, 64), (256, 512, 128), (768, 512, 192), (1024, 1024, 2048)):
        a = torch.randn((m, k), device="cuda", generator=g).to(torch.bfloat16)
        b = torch.randn((n, k), device="cuda", generator=g).to(torch.bfloat16)
        outs = {}
        for sc in scheds:
            gemm.set_schedule(sc)
            outs[sc] = gemm.gemm_bt(a, b)
        ref = outs[scheds[0]]
        for sc in scheds[1:]:
            print(json.dumps({"shape": [m, n, k], "schedule": sc, "bitwise_equal_to": scheds[0],
                              "equal": torch.equal(outs[sc], ref),
                              "max_diff": (outs[sc] - ref).abs().max().item()}), flush=True)
    for size in (int(x) for x in args.sizes.split(",")):
        a = torch.randn(size, size, device="cuda").to(torch.bfloat16)
        b = torch.randn(size, size, device="cuda").to(torch.bfloat16)
        out = torch.empty(size, size, device="cuda", dtype=torch.float32)
        reps = 20 if size <= 4096 else 5
        times = {sc: [] for sc in scheds}
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(args.rounds + 1):
            for sc in scheds:
                gemm.set_schedule(sc)
                torch.cuda.synchronize()
                start.record()
                for _ in range(reps):
                    gemm.gemm_bt(a, b, out)
                end.record()
                torch.cuda.synchronize()
                if r:  # round 0 warms up
                    times[sc].append(start.elapsed_time(end) / reps)
        med = {sc: sorted(v)[len(v) // 2] for sc, v in times.items()}
        print(json.dumps({"size": size, "tflops": {sc: round(2.0 * size ** 3 / t / 1e9, 1) for sc, t in med.items()},
                          "ms": {sc: round(t, 4) for sc, t in med.items()}, "rounds": args.rounds}), flush=True)
    gemm.set_schedule("staggered")
    return 0


if __name__ == "__main__":
    sys.exit(main())
