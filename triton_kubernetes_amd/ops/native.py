"""Loading of the in-tree native libraries (``ops/lib``, built by ``ops/build.py``).

Libraries are loaded with ``ctypes`` from this package's ``lib/`` directory —
never from site-packages or a JIT cache — so the round-end check sees exactly
which ``.so`` files ran.  On a machine with a GPU a missing library is an error
(:class:`NativeUnavailable`), never a silent fallback.
"""

import ctypes
import os
import threading
from typing import Dict

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")

_lock = threading.Lock()
_cache: Dict[str, ctypes.CDLL] = {}
# Whether the first HIP library was loaded before torch: torch bundles its own
# libamdhip64 / librccl under the same sonames as /opt/rocm's, and the one loaded first
# serves the whole process; torch imported afterwards would run on the other build.
_HIP_LIBS = {"libtk_gpu_probe.so", "libtk_gemm.so", "libtk_rccl.so"}
_hip_before_torch = None


class NativeUnavailable(RuntimeError):
    pass


def lib_path(name: str) -> str:
    return os.path.join(LIB_DIR, name)


def load(name: str, autobuild: bool = True) -> ctypes.CDLL:
    with _lock:
        if name in _cache:
            return _cache[name]
        path = lib_path(name)
        if not os.path.exists(path) and autobuild:
            from .build import build

            try:
                build(only=[name])
            except Exception as exc:  # pragma: no cover - build env specific
                raise NativeUnavailable(f"{name} is not built and building it failed: {exc}") from exc
        if not os.path.exists(path):
            raise NativeUnavailable(f"native library {path} is missing; run `python -m "
                                    "triton_kubernetes_amd.ops.build`")
        global _hip_before_torch
        if name in _HIP_LIBS and _hip_before_torch is None:
            import sys

            _hip_before_torch = "torch" not in sys.modules
        try:
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        except OSError as exc:
            raise NativeUnavailable(f"cannot load {path}: {exc}") from exc
        _cache[name] = lib
        return lib


def gpu_present() -> bool:
    """True when the host exposes an AMD GPU (KFD device node or visible devices)."""
    if os.environ.get("TK_FORCE_NO_GPU"):
        return False
    return os.path.exists("/dev/kfd")


def executable(name: str) -> str:
    path = lib_path(name)
    if not os.path.exists(path):
        from .build import build

        build(only=[name])
    return path


def require_torch_first() -> None:
    """Raise unless torch was imported before this process loaded a native HIP library
    (callers that hand torch tensors to native code: both must share one HIP runtime)."""
    import sys

    if _hip_before_torch and "torch" in sys.modules:
        raise NativeUnavailable("torch was imported after the native HIP libraries were loaded; import torch "
                                "first so both use torch's HIP runtime")
