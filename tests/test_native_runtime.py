"""HIP runtime selection for the native libraries (``TK_HIP_RUNTIME``, ops/native.py)."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code, **env):
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT, timeout=120,
                          env=dict(os.environ, **env))


def test_system_runtime():
    p = _run("from triton_kubernetes_amd.ops import native; print(native.runtime_dir())", TK_HIP_RUNTIME="system")
    assert p.returncode == 0 and p.stdout.strip() == "system", p.stderr


def test_missing_runtime_dir_fails_loudly(tmp_path):
    code = ("from triton_kubernetes_amd.ops import native\n"
            "try:\n    native.runtime_dir()\nexcept native.NativeUnavailable as e:\n    print('refused', e)\n")
    p = _run(code, TK_HIP_RUNTIME=str(tmp_path))
    assert p.returncode == 0 and p.stdout.startswith("refused") and "libamdhip64.so missing" in p.stdout


def test_default_runtime_is_the_system_rocm(tmp_path):
    """no bench-tuned runtime by default -- /opt/rocm's HIP and RCCL, the ROCm
    the in-tree libraries are compiled against, even with a prepared slim cache present."""
    env = dict(os.environ, TK_RCCL_SLIM_DIR=str(tmp_path))
    env.pop("TK_HIP_RUNTIME", None)
    p = subprocess.run([sys.executable, "-c", "from triton_kubernetes_amd.ops import native; print(native.select_runtime())"],
                       capture_output=True, text=True, cwd=ROOT, timeout=120, env=env)
    assert p.returncode == 0 and p.stdout.strip() == "system", p.stdout + p.stderr


def test_node_tools_link_the_installed_rccl():
    """rccl-ready and libtk_rccl resolve librccl through a RUNPATH of /opt/rocm only (no
    DT_RPATH into a patched copy); the opt-in copy is reached only through the wrapper."""
    from triton_kubernetes_amd.ops import build, native

    build.build(only=["rccl-ready", "libtk_rccl.so"])
    for name in ("rccl-ready", "libtk_rccl.so"):
        out = subprocess.run(["readelf", "-d", native.lib_path(name)], capture_output=True, text=True).stdout
        assert "(RPATH)" not in out, name
        runpath = next(ln for ln in out.splitlines() if "(RUNPATH)" in ln)
        assert "/opt/rocm" in runpath and "rccl-slim" not in runpath, runpath


def test_torch_runtime_preloads_the_bundled_libraries():
    code = ("from triton_kubernetes_amd.ops import native\n"
            "d = native.runtime_dir()\n"
            "maps = open('/proc/self/maps').read()\n"
            "print(d.endswith('torch/lib'), (d + '/libamdhip64.so') in maps, (d + '/librccl.so') in maps,\n"
            "      'import torch' and __import__('sys').modules.get('torch') is None)\n")
    p = _run(code, TK_HIP_RUNTIME="torch")
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ["True", "True", "True", "True"]  # loaded without importing torch
