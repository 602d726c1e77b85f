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


_runtime_dir = None
SYSTEM_LIB_DIR = "/opt/rocm/lib"
_RUNTIME_LIBS = ("libhsa-runtime64.so", "libamd_comgr.so", "libamdhip64.so", "librccl.so")


def _torch_lib_dir() -> str:
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return ""
    d = os.path.join(list(spec.submodule_search_locations)[0], "lib")
    return d if os.path.exists(os.path.join(d, "librccl.so")) and os.path.exists(os.path.join(d, "libamdhip64.so")) \
        else ""


def select_runtime() -> str:
    """The HIP runtime + RCCL directory this process will use (``TK_HIP_RUNTIME``), without
    loading anything: ``"system"`` or a directory.

    * ``system`` (default): ``/opt/rocm`` -- the libraries' RUNPATH, the ROCm the in-tree
      ``.so`` files are compiled against;
    * ``torch``: the builds bundled with an installed PyTorch-ROCm wheel (its ``lib/``,
      found without importing torch), required;
    * ``slim``: opt-in single-target copy of ``/opt/rocm``'s RCCL (``ops/rccl_slim.py``),
      prepared and verified now if the node has no verified copy yet;
    * a path: a directory holding ``libamdhip64.so`` / ``librccl.so``.

    A process that imports torch before loading a native library runs on torch's runtime
    whatever this says (one HIP runtime per process)."""
    sel = os.environ.get("TK_HIP_RUNTIME", "system") or "system"
    if sel == "system":
        return "system"
    if sel == "torch":
        d = _torch_lib_dir()
        if not d:
            raise NativeUnavailable("TK_HIP_RUNTIME=torch but no PyTorch-ROCm runtime is installed")
        return d
    if sel == "slim":
        from . import rccl_slim

        if not os.path.exists(os.path.join(SYSTEM_LIB_DIR, "librccl.so")):
            raise NativeUnavailable("TK_HIP_RUNTIME=slim but no RCCL is installed")
        slim = rccl_slim.cached(SYSTEM_LIB_DIR)
        if slim:
            return slim
        try:
            return str(rccl_slim.prepare(SYSTEM_LIB_DIR)["dir"])
        except (rccl_slim.SlimError, OSError) as exc:
            raise NativeUnavailable(f"TK_HIP_RUNTIME=slim: {exc}") from exc
    return sel


def runtime_dir() -> str:
    """Load the selected runtime (:func:`select_runtime`) before the first native HIP
    library: non-system runtimes are ``dlopen``ed with ``RTLD_GLOBAL``, so the
    ``libamdhip64.so.7`` / ``librccl.so.1`` dependencies of ``ops/lib`` bind to them (same
    sonames).  A process that already imported torch runs on torch's runtime regardless."""
    global _runtime_dir
    if _runtime_dir is not None:
        return _runtime_dir
    import sys

    if "torch" in sys.modules:
        _runtime_dir = "torch (imported)"
        return _runtime_dir
    d = select_runtime()
    if d != "system":
        for so in _RUNTIME_LIBS:
            path = os.path.join(d, so)
            if os.path.exists(path):
                ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            elif so in ("libamdhip64.so", "librccl.so"):
                raise NativeUnavailable(f"HIP runtime {d}: {path} missing")
    _runtime_dir = d
    return d


def lib_path(name: str) -> str:
    """The in-tree library ``name``; ``TK_RCCL_LIB`` names another ``libtk_rccl.so`` (the ABI
    stub ``libtk_rccl_stub.so`` for a dry run of the cluster gate without GPUs)."""
    if name == "libtk_rccl.so" and os.environ.get("TK_RCCL_LIB"):
        return os.environ["TK_RCCL_LIB"]
    return os.path.join(LIB_DIR, name)


def load(name: str, autobuild: bool = True) -> ctypes.CDLL:
    with _lock:
        if name in _cache:
            return _cache[name]
        path = lib_path(name)
        if not os.path.exists(path) and autobuild and os.path.dirname(path) == LIB_DIR:
            from .build import build

            try:
                build(only=[name])
            except Exception as exc:  # pragma: no cover - build env specific
                raise NativeUnavailable(f"{name} is not built and building it failed: {exc}") from exc
        if not os.path.exists(path):
            raise NativeUnavailable(f"native library {path} is missing; run `python -m "
                                    "triton_kubernetes_amd.ops.build`")
        global _hip_before_torch
        if name in _HIP_LIBS and _hip_before_torch is None and os.path.dirname(path) == LIB_DIR:
            import sys

            _hip_before_torch = "torch" not in sys.modules
            runtime_dir()
        try:
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        except OSError as exc:
            raise NativeUnavailable(f"cannot load {path}: {exc}") from exc
        _cache[name] = lib
        return lib


def executable(name: str) -> str:
    """The in-tree tool ``name``, built from this tree's sources (``ops/build.py`` stamps):
    a missing or stale tool is rebuilt when a compiler is there, else NativeUnavailable --
    never a run of a binary that predates its sources (a stale ``gpu-burnin`` ignores the
    flags it does not know and runs something else)."""
    from .build import build, current

    path = lib_path(name)
    if not current(name):
        try:
            build(only=[name])
        except Exception as exc:  # pragma: no cover - build env specific
            raise NativeUnavailable(f"{name} is {'stale' if os.path.exists(path) else 'not built'} and "
                                    f"building it failed: {exc}") from exc
        if not current(name):
            raise NativeUnavailable(f"{path} does not match its sources and could not be rebuilt")
    return path


def require_torch_first() -> None:
    """Raise unless torch was imported before this process loaded a native HIP library
    (callers that hand torch tensors to native code: both must share one HIP runtime)."""
    import sys

    if _hip_before_torch and "torch" in sys.modules:
        raise NativeUnavailable("torch was imported after the native HIP libraries were loaded; import torch "
                                "first so both use torch's HIP runtime")
