"""Python front-end of the MI355X GEMM silent-data-corruption screen (``csrc/tk_gemm_screen.hip``).

``screen(dev)`` runs an LDS-tiled bf16 MFMA GEMM on random operands and checks it with
row/column checksums (algorithm-based fault tolerance); the burn-in fails a GPU whose
GEMM disagrees with the independently computed checksums.  ``gemm_bt`` exposes the same
kernel with a full C output (fp32, or bf16 as the vendor GEMM writes), stream-ordered on
torch's current stream, for numerics tests against a PyTorch reference and for the
comparison with hipBLASLt (``scripts/gemm_vs_lib.py``).
"""

import ctypes
from dataclasses import asdict, dataclass
from typing import Any, Dict

from .native import load

TILE_M = TILE_N = 256
TILE_K = 64  # bf16 elements per K-tile (128 bytes of a row)
TILE_K_FP8 = 128  # fp8 e4m3 elements per K-tile

# level -> (M, N, K, timed reps)
# quick: a 4096^3 GEMM is ~60-100 us, so best of 5 (each rep is one timed launch)
SCREEN_SIZES = {"quick": (4096, 4096, 4096, 5), "full": (8192, 8192, 8192, 5)}


class GemmError(RuntimeError):
    pass


def _lib():
    lib = load("libtk_gemm.so")
    lib.tkg_last_error.restype = ctypes.c_char_p
    lib.tkg_screen.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_longlong, ctypes.POINTER(ctypes.c_double)]
    lib.tkg_screen_fp8.argtypes = lib.tkg_screen.argtypes
    lib.tkg_set_schedule.argtypes = [ctypes.c_int]
    lib.tkg_gemm.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return lib


SCHEDULES = {"staggered": 1, "single-barrier": 0}


def set_schedule(name: str) -> str:
    """Select the GEMM main loop: ``staggered`` (default: two wave groups one barrier apart,
    two phases per K-tile) or ``single-barrier`` (one barrier per K-step, kept for A/B).
    Returns the schedule in effect."""
    if name not in SCHEDULES:
        raise GemmError(f"unknown schedule '{name}' ({' | '.join(SCHEDULES)})")
    got = _lib().tkg_set_schedule(SCHEDULES[name])
    return next(k for k, v in SCHEDULES.items() if v == got)


def check_shape(m: int, n: int, k: int, dtype: str = "bf16") -> None:
    tk = TILE_K_FP8 if dtype == "fp8" else TILE_K
    if m <= 0 or n <= 0 or k <= 0 or m % TILE_M or n % TILE_N or k % tk:
        raise GemmError(f"shape {m}x{n}x{k}: M and N must be multiples of {TILE_M}, K of {tk}")


def gemm_bt(a, b, out=None, out_dtype=None):
    """``out = a @ b.T`` for CUDA tensors ``a [M,K]``, ``b [N,K]`` (contiguous), both bf16 or
    both fp8 e4m3 (``torch.float8_e4m3fn``: the block-scaled MFMA with unit scales).  ``out``
    (or ``out_dtype``) is fp32 (default) or bf16.  The kernel is queued on torch's current
    stream of ``a``'s device, like a torch op: nothing waits for it here."""
    import torch

    from .native import require_torch_first

    require_torch_first()
    fp8 = getattr(torch, "float8_e4m3fn", None)
    if a.dtype != b.dtype or a.dtype not in (torch.bfloat16, fp8) or not (a.is_cuda and b.is_cuda):
        raise GemmError("gemm_bt wants two bf16 or two float8_e4m3fn CUDA tensors")
    if not (a.is_contiguous() and b.is_contiguous()) or a.shape[1] != b.shape[1] or a.device != b.device:
        raise GemmError("gemm_bt wants contiguous a [M,K] and b [N,K] on one device")
    m, k = a.shape
    n = b.shape[0]
    dtype = "fp8" if a.dtype == fp8 else "bf16"
    check_shape(m, n, k, dtype)
    want = out.dtype if out is not None else (out_dtype or torch.float32)
    if want not in (torch.float32, torch.bfloat16):
        raise GemmError("out must be fp32 or bf16")
    if out is None:
        out = torch.empty((m, n), dtype=want, device=a.device)
    elif out.shape != (m, n) or not out.is_contiguous() or out.device != a.device:
        raise GemmError("out must be a contiguous [M,N] tensor on a's device")
    dev = a.device.index if a.device.index is not None else torch.cuda.current_device()
    stream = torch.cuda.current_stream(a.device).cuda_stream
    rc = _lib().tkg_gemm(dev, 1 if dtype == "fp8" else 2, a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k,
                         1 if want == torch.bfloat16 else 0, stream)
    if rc != 0:
        raise GemmError(_lib().tkg_last_error().decode())
    return out


@dataclass
class ScreenResult:
    m: int
    n: int
    k: int
    tflops: float
    ms: float
    bad_columns: int
    bad_rows: int
    first_bad_column: int
    first_bad_row: int
    max_norm_error: float  # |checksum error| / tolerance, worst over all rows and columns
    dtype: str = "bf16"

    @property
    def ok(self) -> bool:
        return self.bad_columns == 0 and self.bad_rows == 0

    def to_json(self) -> Dict[str, Any]:
        d = asdict(self)
        d["ok"] = self.ok
        return d


def screen(dev: int, m: int = 4096, n: int = 4096, k: int = 4096, reps: int = 2, inject: int = -1,
           dtype: str = "bf16") -> ScreenResult:
    """Run the checksum-verified GEMM on random ``dtype`` (bf16 | fp8) operands; ``inject``
    (row*N + col) corrupts one C element to prove the screen catches it."""
    if dtype not in ("bf16", "fp8"):
        raise GemmError(f"unknown dtype '{dtype}' (bf16 | fp8)")
    check_shape(m, n, k, dtype)
    out = (ctypes.c_double * 7)()
    fn = _lib().tkg_screen_fp8 if dtype == "fp8" else _lib().tkg_screen
    rc = fn(dev, m, n, k, reps, inject, out)
    if rc != 0:
        raise GemmError(_lib().tkg_last_error().decode())
    return ScreenResult(m, n, k, out[0], out[1], int(out[2]), int(out[3]), int(out[4]), int(out[5]), out[6], dtype)
