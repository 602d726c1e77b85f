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


def test_auto_prefers_the_pytorch_rocm_runtime(tmp_path):
    # (an empty single-target cache: tests/test_rccl_slim.py covers the prepared case)
    p = _run("from triton_kubernetes_amd.ops import native; print(native.select_runtime())", TK_HIP_RUNTIME="auto",
             TK_RCCL_SLIM_DIR=str(tmp_path))
    assert p.returncode == 0 and p.stdout.strip().endswith("torch/lib"), p.stdout + p.stderr


def test_torch_runtime_preloads_the_bundled_libraries():
    code = ("from triton_kubernetes_amd.ops import native\n"
            "d = native.runtime_dir()\n"
            "maps = open('/proc/self/maps').read()\n"
            "print(d.endswith('torch/lib'), (d + '/libamdhip64.so') in maps, (d + '/librccl.so') in maps,\n"
            "      'import torch' and __import__('sys').modules.get('torch') is None)\n")
    p = _run(code, TK_HIP_RUNTIME="torch")
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ["True", "True", "True", "True"]  # loaded without importing torch
