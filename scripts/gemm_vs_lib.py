#!/usr/bin/env python3
"""The burn-in's hand-written GEMM (ops/csrc/tk_gemm_screen.hip) against the vendor library
on the same GPU: ``torch.mm`` (hipBLASLt) for bf16, ``torch._scaled_mm`` for fp8 e4m3 with
unit scales.  One JSON line per (dtype, size): TFLOP/s of each and their ratio.

Both write bf16 C (``ours_tflops``; ``ours_fp32_tflops``: the same kernel writing fp32,
twice the output bytes).  Every launch is queued back to back on torch's stream (no host
synchronisation between launches, as for the library), so the event time is kernel time.
Run on the GPU box: ``python scripts/gemm_vs_lib.py > gpurun_out/gemm_vs_lib.jsonl``, under
``rocprofv3 --kernel-trace`` for per-kernel durations.
"""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from triton_kubernetes_amd.ops import gemm  # noqa: E402


ROUNDS = 7


def timed(fn, reps: int) -> float:
    """Mean ms of ``fn`` over ``reps`` back-to-back launches."""
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    start.record()
    for _ in range(reps):
        fn()
    end.record()
    torch.cuda.synchronize()
    return start.elapsed_time(end) / reps


def compare(arms: dict, reps: int) -> dict:
    """Median ms per arm over ``ROUNDS`` rounds that run every arm in turn: the chip's
    clock drifts under a sustained GEMM load (DVFS), so arms timed one after the other
    would be compared at different clocks."""
    for fn in arms.values():  # warm-up: code objects, library heuristics, clocks
        timed(fn, 3)
    times = {name: [] for name in arms}
    for _ in range(ROUNDS):
        for name, fn in arms.items():
            times[name].append(timed(fn, reps))
    return {name: sorted(v)[len(v) // 2] for name, v in times.items()}


def main() -> int:
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    fp8 = getattr(torch, "float8_e4m3fn", None)
    for size in (4096, 8192):
        m = n = k = size
        flop = 2.0 * m * n * k
        reps = 20 if size <= 4096 else 5
        tf = lambda ms: round(flop / ms / 1e9, 1)  # noqa: E731
        a = torch.randn(m, k, device=dev).to(torch.bfloat16)
        b = torch.randn(n, k, device=dev).to(torch.bfloat16)
        out = torch.empty(m, n, device=dev, dtype=torch.float32)
        out16 = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        t = compare({"ours": lambda: gemm.gemm_bt(a, b, out16), "lib": lambda: torch.mm(a, b.t()),
                     "ours_fp32": lambda: gemm.gemm_bt(a, b, out)}, reps)
        err = (gemm.gemm_bt(a, b, out) - (a.float() @ b.float().t())).abs().max().item()
        print(json.dumps({"dtype": "bf16", "m": m, "n": n, "k": k, "ours_tflops": tf(t["ours"]),
                          "ours_fp32_tflops": tf(t["ours_fp32"]), "lib_tflops": tf(t["lib"]),
                          "ours_over_lib": round(t["lib"] / t["ours"], 3), "max_abs_err_vs_fp32": err,
                          "lib": "torch.mm (hipBLASLt)", "rounds": ROUNDS}), flush=True)
        if fp8 is not None:
            a8, b8 = (a * 0.5).to(fp8), (b * 0.5).to(fp8)
            one = torch.ones((), device=dev, dtype=torch.float32)
            arms = {"ours": lambda: gemm.gemm_bt(a8, b8, out16), "ours_fp32": lambda: gemm.gemm_bt(a8, b8, out)}
            row = {"dtype": "fp8_e4m3", "m": m, "n": n, "k": k}
            try:
                torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
                arms["lib"] = lambda: torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
            except (RuntimeError, TypeError) as exc:  # not every build has an e4m3fn kernel for this GPU
                row.update(lib_tflops=None, lib_error=str(exc)[:200])
            t = compare(arms, reps)
            row.update(ours_tflops=tf(t["ours"]), ours_fp32_tflops=tf(t["ours_fp32"]), rounds=ROUNDS)
            if "lib" in t:
                row.update(lib_tflops=tf(t["lib"]), ours_over_lib=round(t["lib"] / t["ours"], 3),
                           lib="torch._scaled_mm")
            print(json.dumps(row), flush=True)
        del a, b, out, out16
        torch.cuda.empty_cache()
    for size in (8192,):
        r = gemm.screen(0, size, size, size, reps=5)
        print(json.dumps({"screen": "bf16", "m": size, "tflops_with_checksums": round(r.tflops, 1), "ok": r.ok}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
