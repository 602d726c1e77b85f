#!/usr/bin/env python3
"""A/B the two GEMM screen schedules in ONE process (tkg_set_schedule: 0 = one barrier per
K-step, 1 = 8-phase staggered): exactness vs a torch fp32 reference on edge shapes, then
interleaved screens (best TFLOP/s of 3 rounds x 5 timed reps, ABFT must pass)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402  (torch's HIP runtime first)

from triton_kubernetes_amd.ops import gemm  # noqa: E402

lib = gemm._lib()
lib.tkg_set_schedule.argtypes = [ctypes.c_int]
out = {"exact": {}, "tflops": {}}
torch.manual_seed(0)
for m, n, k in ((256, 256, 64), (256, 512, 128), (512, 256, 192), (768, 1024, 320), (2048, 1536, 4096)):
    a = torch.randn(m, k, device="cuda").to(torch.bfloat16)
    b = torch.randn(n, k, device="cuda").to(torch.bfloat16)
    ref = a.float() @ b.float().T
    for sched in (0, 1):
        assert lib.tkg_set_schedule(sched) == sched
        c = gemm.gemm_bt(a, b)
        err = ((c - ref).abs() / (ref.abs() + 1.0)).max().item()
        out["exact"][f"s{sched}@{m}x{n}x{k}"] = err
        assert err < 1e-3, (sched, m, n, k, err)
for size in (4096, 8192):
    best = {0: 0.0, 1: 0.0}
    for _ in range(3):
        for sched in (0, 1):
            lib.tkg_set_schedule(sched)
            r = gemm.screen(0, size, size, size, reps=5)
            assert r.ok, r
            best[sched] = max(best[sched], r.tflops)
    for sched in (0, 1):
        out["tflops"][f"s{sched}@{size}"] = round(best[sched], 1)
# the screen must still catch a corrupted element with the 8-phase schedule
lib.tkg_set_schedule(1)
bad = gemm.screen(0, 4096, 4096, 4096, reps=1, inject=1234 * 4096 + 3071)
out["inject_8phase"] = {"ok": bad.ok, "row": bad.first_bad_row, "col": bad.first_bad_column}
assert not bad.ok and bad.first_bad_row == 1234 and bad.first_bad_column == 3071
print(json.dumps(out))
