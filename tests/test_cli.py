"""CLI surface (reference cmd/*.go): argument errors, exit codes, version, config."""

import io
import os
import subprocess
import sys

import pytest

from triton_kubernetes_amd.cli.main import run, version_text

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(argv, **kw):
    out = io.StringIO()
    code = run(argv, out=out, **kw)
    return code, out.getvalue()


@pytest.mark.parametrize("cmd,name", [("create", "create"), ("destroy", "destory"), ("get", "get")])
def test_requires_one_argument(cmd, name):
    assert _run([cmd]) == (255, f'"triton-kubernetes {name}" requires one argument\n')
    assert _run([cmd, "manager", "cluster"])[0] == 255


@pytest.mark.parametrize("cmd,bad", [("create", "x"), ("destroy", "everything"), ("get", "node")])
def test_invalid_argument(cmd, bad):
    name = "destory" if cmd == "destroy" else cmd
    assert _run([cmd, bad]) == (255, f'invalid argument "{bad}" for "triton-kubernetes {name}"\n')


def test_version_output():
    assert _run(["version"]) == (0, version_text())
    assert version_text("") == "no version set for this build... triton-kubernetes v0.8.2 (local)\n"
    assert version_text("abc123") == "triton-kubernetes v0.8.2 (abc123)\n"


def test_non_interactive_missing_backend_exits_1(tk_home):
    code, out = _run(["--non-interactive", "get", "manager"])
    assert code == 1
    assert out.splitlines()[0] == "Running in non interactive mode"
    assert out.splitlines()[-1] == "backend_provider must be provided"


def test_config_file_and_env(tk_home, tmp_path, monkeypatch):
    cfg = tmp_path / "c.yaml"
    cfg.write_text("backend_provider: local\n")
    code, out = _run(["--config", str(cfg), "--non-interactive", "get", "manager"])
    assert f"Using config file: {cfg}" in out
    assert "get manager called" in out
    assert code == 1 and out.rstrip().endswith("No cluster managers.")
    monkeypatch.setenv("BACKEND_PROVIDER", "floppy")
    code, out = _run(["--non-interactive", "get", "manager"])
    assert code == 1 and "Unsupported backend provider 'floppy'" in out


def test_default_config_discovered_in_home(tk_home):
    (tk_home / ".triton-kubernetes.yaml").write_text("backend_provider: local\n")
    code, out = _run(["--non-interactive", "get", "cluster"])
    assert "Using config file:" in out and code == 1


def test_flags_after_subcommand(tk_home):
    code, out = _run(["get", "--non-interactive", "manager"])
    assert "Running in non interactive mode" in out


def test_entry_points_subprocess(tk_home):
    env = dict(os.environ, HOME=str(tk_home), PYTHONPATH=ROOT)
    for argv in ([sys.executable, "-m", "triton_kubernetes_amd", "version"],
                 [os.path.join(ROOT, "bin", "triton-kubernetes"), "version"]):
        proc = subprocess.run(argv, capture_output=True, text=True, env=env, timeout=60)
        assert proc.returncode == 0, proc.stderr
        assert "triton-kubernetes v0.8.2" in proc.stdout
    proc = subprocess.run([sys.executable, "-m", "triton_kubernetes_amd", "destroy"], capture_output=True,
                          text=True, env=env, timeout=60)
    assert proc.returncode == 255 and "requires one argument" in proc.stdout


def test_help_lists_commands():
    code, out = _run([])
    assert code == 0
    for word in ("create", "destroy", "get", "version", "wait", "gpu", "agent", "image", "backup", "restore",
                 "userdata"):
        assert word in out
