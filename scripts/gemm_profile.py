#!/usr/bin/env python3
"""One 8192^3 GEMM screen (for rocprofv3 counter passes over k_gemm_bt or, with TKG_SCHED=1,
k_gemm8).  TK_GEMM_DTYPE=fp8 screens fp8 e4m3 operands instead of bf16."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triton_kubernetes_amd.ops import gemm  # noqa: E402

r = gemm.screen(0, 8192, 8192, 8192, reps=2, dtype=os.environ.get("TK_GEMM_DTYPE", "bf16"))
print(r.to_json())
