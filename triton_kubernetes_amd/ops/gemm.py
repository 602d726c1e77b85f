"""Python front-end of the MI355X GEMM silent-data-corruption screen (``csrc/tk_gemm_screen.hip``).

``screen(dev)`` runs an LDS-tiled bf16 MFMA GEMM on random operands and checks it with
row/column checksums (algorithm-based fault tolerance); the burn-in fails a GPU whose
GEMM disagrees with the independently computed checksums.  ``gemm_bt`` exposes the same
kernel with a full fp32 C output for numerics tests against a PyTorch reference.
"""

import ctypes
from dataclasses import asdict, dataclass
from typing import Any, Dict

from .native import load

TILE_M = TILE_N = 256
TILE_K = 64

# level -> (M, N, K, timed reps)
SCREEN_SIZES = {"quick": (4096, 4096, 4096, 2), "full": (8192, 8192, 8192, 5)}


class GemmError(RuntimeError):
    pass


def _lib():
    lib = load("libtk_gemm.so")
    lib.tkg_last_error.restype = ctypes.c_char_p
    lib.tkg_gemm_bt.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.tkg_screen.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_longlong, ctypes.POINTER(ctypes.c_double)]
    lib.tkg_set_schedule.argtypes = [ctypes.c_int]
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


def check_shape(m: int, n: int, k: int) -> None:
    if m <= 0 or n <= 0 or k <= 0 or m % TILE_M or n % TILE_N or k % TILE_K:
        raise GemmError(f"shape {m}x{n}x{k}: M and N must be multiples of {TILE_M}, K of {TILE_K}")


def gemm_bt(a, b, out=None):
    """``out = a @ b.T`` in fp32 for bf16 CUDA tensors ``a [M,K]``, ``b [N,K]`` (contiguous)."""
    import torch

    from .native import require_torch_first

    require_torch_first()
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or not (a.is_cuda and b.is_cuda):
        raise GemmError("gemm_bt wants bf16 CUDA tensors")
    if not (a.is_contiguous() and b.is_contiguous()) or a.shape[1] != b.shape[1]:
        raise GemmError("gemm_bt wants contiguous a [M,K] and b [N,K]")
    m, k = a.shape
    n = b.shape[0]
    check_shape(m, n, k)
    if out is None:
        out = torch.empty((m, n), dtype=torch.float32, device=a.device)
    elif out.shape != (m, n) or out.dtype != torch.float32 or not out.is_contiguous():
        raise GemmError("out must be a contiguous fp32 [M,N] tensor")
    rc = _lib().tkg_gemm_bt(a.device.index or 0, a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k)
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

    @property
    def ok(self) -> bool:
        return self.bad_columns == 0 and self.bad_rows == 0

    def to_json(self) -> Dict[str, Any]:
        d = asdict(self)
        d["ok"] = self.ok
        return d


def screen(dev: int, m: int = 4096, n: int = 4096, k: int = 4096, reps: int = 2, inject: int = -1) -> ScreenResult:
    """Run the checksum-verified GEMM; ``inject`` (row*N + col) corrupts one C element to
    prove the screen catches it."""
    check_shape(m, n, k)
    out = (ctypes.c_double * 7)()
    rc = _lib().tkg_screen(dev, m, n, k, reps, inject, out)
    if rc != 0:
        raise GemmError(_lib().tkg_last_error().decode())
    return ScreenResult(m, n, k, out[0], out[1], int(out[2]), int(out[3]), int(out[4]), int(out[5]), out[6])
