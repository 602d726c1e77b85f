import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# One HIP runtime per process: torch ships its own libamdhip64 / librccl (same sonames as
# /opt/rocm's).  Whichever loads first serves both, so torch goes first — as in bench.py —
# before any test dlopens the native libraries; a torch imported after them would run on
# the other runtime build (seen as heap corruption at interpreter exit).
try:
    import torch  # noqa: F401,E402
except ImportError:  # pragma: no cover - torch is part of the image
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: multi-second tests")


def gpu_available() -> bool:
    return os.path.exists("/dev/kfd") and not os.environ.get("TK_FORCE_NO_GPU")


@pytest.fixture
def tk_home(tmp_path, monkeypatch):
    """Isolated ~/.triton-kubernetes for local-backend tests."""
    home = tmp_path / "home"
    home.mkdir()
    monkeypatch.setenv("HOME", str(home))
    monkeypatch.delenv("TRITON_KUBERNETES_HOME", raising=False)
    return home
