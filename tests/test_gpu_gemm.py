"""GEMM SDC screen (csrc/tk_gemm_screen.hip) on the MI355X: numerics of the LDS-tiled
MFMA GEMM against a plain PyTorch fp32 reference, the checksum screen's pass on a healthy
GPU, and its detection of an injected fault."""

import json

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (512, 768, 1024), (1024, 256, 4096)])
def test_gemm_matches_fp32_reference(m, n, k):
    import torch

    from triton_kubernetes_amd.ops import gemm

    g = torch.Generator(device="cuda").manual_seed(m + n + k)
    a = (torch.rand((m, k), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand((n, k), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    got = gemm.gemm_bt(a, b)
    ref = a.float() @ b.float().T
    torch.cuda.synchronize()
    err = (got - ref).abs().max().item()
    assert err <= 1e-3 * max(1.0, ref.abs().max().item()), err


def test_gemm_exact_on_integer_data_asymmetric():
    """Exact small integers (bf16-exact, fp32-exact sums) with an asymmetric B: any
    row/column mix-up in fragments, swizzle or epilogue shows as a nonzero difference."""
    import torch

    from triton_kubernetes_amd.ops import gemm

    m, n, k = 512, 256, 128
    a = (torch.arange(m * k, device="cuda").reshape(m, k) % 7 - 3).to(torch.bfloat16)
    b = ((torch.arange(n * k, device="cuda").reshape(n, k) * 3 + torch.arange(n, device="cuda")[:, None]) % 5 - 2
         ).to(torch.bfloat16)
    got = gemm.gemm_bt(a, b)
    ref = a.float() @ b.float().T
    assert torch.equal(got, ref)


def test_gemm_rejects_untiled_shapes():
    import torch

    from triton_kubernetes_amd.ops import gemm

    a = torch.zeros((300, 64), device="cuda", dtype=torch.bfloat16)
    b = torch.zeros((256, 64), device="cuda", dtype=torch.bfloat16)
    with pytest.raises(gemm.GemmError):
        gemm.gemm_bt(a, b)


def test_screen_passes_and_catches_injected_fault():
    from triton_kubernetes_amd.ops import gemm

    ok = gemm.screen(0, 4096, 4096, 4096, reps=3)
    print(json.dumps(ok.to_json()))
    assert ok.ok and ok.max_norm_error < 0.5, ok
    assert ok.tflops > 500, ok
    row, col = 1234, 3071
    bad = gemm.screen(0, 4096, 4096, 4096, reps=1, inject=row * 4096 + col)
    print(json.dumps(bad.to_json()))
    assert not bad.ok
    assert (bad.bad_rows, bad.bad_columns) == (1, 1)
    assert (bad.first_bad_row, bad.first_bad_column) == (row, col)


def test_screen_full_size_throughput():
    from triton_kubernetes_amd.ops import gemm

    r = gemm.screen(0, 8192, 8192, 8192, reps=5)
    print(json.dumps(r.to_json()))
    assert r.ok, r
    assert r.tflops > 1000, r  # 1.44-1.54 PF measured with the staggered schedule


def test_schedules_agree_bitwise():
    """The staggered 2-phase loop and the single-barrier loop feed every accumulator the same
    MFMAs in the same K order, so their fp32 outputs are identical, bit for bit; the tail
    shapes (one and two K-tiles) exercise the vmcnt(0) paths."""
    import torch

    from triton_kubernetes_amd.ops import gemm

    g = torch.Generator(device="cuda").manual_seed(7)
    try:
        for m, n, k in ((256, 256, 64), (256, 512, 128), (768, 512, 192), (1024, 1024, 2048)):
            a = torch.randn((m, k), device="cuda", generator=g).to(torch.bfloat16)
            b = torch.randn((n, k), device="cuda", generator=g).to(torch.bfloat16)
            assert gemm.set_schedule("single-barrier") == "single-barrier"
            ref = gemm.gemm_bt(a, b)
            assert gemm.set_schedule("staggered") == "staggered"
            got = gemm.gemm_bt(a, b)
            assert torch.equal(got, ref), (m, n, k, (got - ref).abs().max().item())
    finally:
        gemm.set_schedule("staggered")


# --- fp8 e4m3 (block-scaled 16x16x128 MFMA, unit scales) ------------------------------------------


@pytest.mark.parametrize("m,n,k", [(256, 256, 128), (512, 768, 1024), (1024, 256, 4096)])
def test_fp8_gemm_matches_fp32_reference(m, n, k):
    import torch

    from triton_kubernetes_amd.ops import gemm

    g = torch.Generator(device="cuda").manual_seed(m * 3 + n + k)
    a = (torch.rand((m, k), device="cuda", generator=g) * 4 - 2).to(torch.float8_e4m3fn)
    b = (torch.rand((n, k), device="cuda", generator=g) * 4 - 2).to(torch.float8_e4m3fn)
    got = gemm.gemm_bt(a, b)
    ref = a.float() @ b.float().T
    torch.cuda.synchronize()
    err = (got - ref).abs().max().item()
    assert err <= 1e-4 * max(1.0, (a.float().abs() @ b.float().abs().T).max().item()), err


def test_fp8_gemm_exact_on_integer_data_asymmetric():
    """Small integers are exact in e4m3 and their sums exact in fp32: any fragment, k-order
    or epilogue mix-up of the fp8 path shows as a nonzero difference."""
    import torch

    from triton_kubernetes_amd.ops import gemm

    m, n, k = 512, 256, 256
    a = (torch.arange(m * k, device="cuda").reshape(m, k) % 7 - 3).to(torch.float8_e4m3fn)
    b = ((torch.arange(n * k, device="cuda").reshape(n, k) * 3 + torch.arange(n, device="cuda")[:, None]) % 5 - 2
         ).to(torch.float8_e4m3fn)
    got = gemm.gemm_bt(a, b)
    ref = a.float() @ b.float().T
    torch.cuda.synchronize()
    assert torch.equal(got, ref), (got - ref).abs().max().item()


def test_fp8_screen_passes_catches_fault_and_runs_at_rate():
    from triton_kubernetes_amd.ops import gemm

    with pytest.raises(gemm.GemmError):
        gemm.screen(0, 256, 256, 64, dtype="fp8")  # K must be a multiple of 128 for fp8
    ok = gemm.screen(0, 8192, 8192, 8192, reps=5, dtype="fp8")
    print(json.dumps(ok.to_json()))
    assert ok.ok and ok.max_norm_error < 0.5 and ok.dtype == "fp8", ok
    assert ok.tflops > 2000, ok
    row, col = 777, 4095
    bad = gemm.screen(0, 4096, 4096, 4096, reps=1, inject=row * 4096 + col, dtype="fp8")
    assert not bad.ok and (bad.first_bad_row, bad.first_bad_column) == (row, col), bad


# --- bf16 output (the vendor GEMM's output type), stream-ordered ----------------------------------


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
@pytest.mark.parametrize("m,n,k", [(256, 256, 128), (768, 512, 256), (1024, 1280, 2048)])
def test_bf16_output_is_the_fp32_result_rounded_once(dtype, m, n, k):
    """The bf16 epilogue (lane exchange, swizzled LDS image, 16-byte stores) against the fp32
    output of the same kernel rounded to bf16 by torch: identical, element for element, so
    any row, column or lane-pair mix-up of the transposition shows.  Asymmetric integer
    data (exact in fp32) and random data both."""
    import torch

    from triton_kubernetes_amd.ops import gemm

    el = torch.bfloat16 if dtype == "bf16" else torch.float8_e4m3fn
    ia = (torch.arange(m * k, device="cuda").reshape(m, k) % 7 - 3).to(el)
    ib = ((torch.arange(n * k, device="cuda").reshape(n, k) * 3 + torch.arange(n, device="cuda")[:, None]) % 5 - 2
          ).to(el)
    g = torch.Generator(device="cuda").manual_seed(m + 2 * n + k)
    ra = (torch.rand((m, k), device="cuda", generator=g) * 2 - 1).to(el)
    rb = (torch.rand((n, k), device="cuda", generator=g) * 2 - 1).to(el)
    for a, b in ((ia, ib), (ra, rb)):
        full = gemm.gemm_bt(a, b)
        got = gemm.gemm_bt(a, b, out_dtype=torch.bfloat16)
        assert got.dtype == torch.bfloat16 and got.shape == (m, n)
        assert torch.equal(got, full.to(torch.bfloat16)), (got.float() - full).abs().max().item()
    ref = ia.float() @ ib.float().T
    assert torch.equal(gemm.gemm_bt(ia, ib, out_dtype=torch.bfloat16), ref.to(torch.bfloat16))


def test_gemm_runs_on_torchs_current_stream():
    """Queued on the caller's stream like a torch op: a GEMM on a side stream, whose inputs a
    kernel on that same stream just wrote, sees them; nothing blocks the host."""
    import torch

    from triton_kubernetes_amd.ops import gemm

    m = n = 512
    k = 1024
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        a = torch.full((m, k), 0.5, device="cuda", dtype=torch.bfloat16)
        b = torch.full((n, k), 0.25, device="cuda", dtype=torch.bfloat16)
        a.mul_(2.0)  # queued on s just before the GEMM
        out = gemm.gemm_bt(a, b, out_dtype=torch.bfloat16)
    s.synchronize()
    assert torch.equal(out, torch.full((m, n), 0.25 * k, device="cuda", dtype=torch.bfloat16))


def test_bf16_output_refuses_what_it_cannot_write():
    import torch

    from triton_kubernetes_amd.ops import gemm

    a = torch.zeros((256, 64), device="cuda", dtype=torch.bfloat16)
    with pytest.raises(gemm.GemmError):
        gemm.gemm_bt(a, a, out_dtype=torch.float16)
    with pytest.raises(gemm.GemmError):  # 2-byte offset: not 16-byte aligned
        gemm.gemm_bt(a, a, out=torch.empty(256 * 256 + 1, device="cuda", dtype=torch.bfloat16)[1:].view(256, 256))
    try:
        gemm.set_schedule("single-barrier")
        with pytest.raises(gemm.GemmError):
            gemm.gemm_bt(a, a, out_dtype=torch.bfloat16)
    finally:
        gemm.set_schedule("staggered")
