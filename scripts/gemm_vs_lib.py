#!/usr/bin/env python3
"""The burn-in's hand-written GEMM (ops/csrc/tk_gemm_screen.hip) against the vendor library
on the same GPU: ``torch.mm`` (hipBLASLt) for bf16, ``torch._scaled_mm`` for fp8 e4m3 with
unit scales.  One JSON line per (dtype, size): TFLOP/s of each and their ratio.

The library writes bf16 (fp8: bf16) output, ours fp32; at these sizes the output is
<1 % of the traffic, so the comparison is of the main loops.  Run on the GPU box:
``python scripts/gemm_vs_lib.py > gpurun_out/gemm_vs_lib.jsonl``.
"""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from triton_kubernetes_amd.ops import gemm  # noqa: E402


def timed(fn, reps: int) -> float:
    """Mean ms of ``fn`` over ``reps`` launches (after 3 untimed)."""
    for _ in range(3):
        fn()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    start.record()
    for _ in range(reps):
        fn()
    end.record()
    torch.cuda.synchronize()
    return start.elapsed_time(end) / reps


def main() -> int:
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    fp8 = getattr(torch, "float8_e4m3fn", None)
    for size in (4096, 8192):
        m = n = k = size
        flop = 2.0 * m * n * k
        reps = 50 if size <= 4096 else 20
        a = torch.randn(m, k, device=dev).to(torch.bfloat16)
        b = torch.randn(n, k, device=dev).to(torch.bfloat16)
        out = torch.empty(m, n, device=dev, dtype=torch.float32)
        ours = timed(lambda: gemm.gemm_bt(a, b, out), reps)
        lib = timed(lambda: torch.mm(a, b.t()), reps)
        err = (gemm.gemm_bt(a, b, out) - (a.float() @ b.float().t())).abs().max().item()
        print(json.dumps({"dtype": "bf16", "m": m, "n": n, "k": k, "ours_tflops": round(flop / ours / 1e9, 1),
                          "lib_tflops": round(flop / lib / 1e9, 1), "ours_over_lib": round(lib / ours, 3),
                          "max_abs_err_vs_fp32": err, "lib": "torch.mm (hipBLASLt)"}), flush=True)
        if fp8 is not None:
            a8, b8 = (a * 0.5).to(fp8), (b * 0.5).to(fp8)
            row = {"dtype": "fp8_e4m3", "m": m, "n": n, "k": k}
            ours8 = timed(lambda: gemm.gemm_bt(a8, b8, out), reps)
            row["ours_tflops"] = round(flop / ours8 / 1e9, 1)
            one = torch.ones((), device=dev, dtype=torch.float32)
            try:
                lib8 = timed(lambda: torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one,
                                                      out_dtype=torch.bfloat16), reps)
                row.update(lib_tflops=round(flop / lib8 / 1e9, 1), ours_over_lib=round(lib8 / ours8, 3),
                           lib="torch._scaled_mm")
            except (RuntimeError, TypeError) as exc:  # not every build has an e4m3fn kernel for this GPU
                row.update(lib_tflops=None, lib_error=str(exc)[:200])
            print(json.dumps(row), flush=True)
        del a, b, out
        torch.cuda.empty_cache()
    for size in (8192,):
        r = gemm.screen(0, size, size, size, reps=5)
        print(json.dumps({"screen": "bf16", "m": size, "tflops_with_checksums": round(r.tflops, 1), "ok": r.ok}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
