"""Shared test helpers: contexts, fake terraform on PATH, SSH key fixtures."""

import io
import json
import os
import shutil
import stat
import subprocess
import sys
from typing import Any, Dict, List, Optional

from triton_kubernetes_amd.config import Context, ScriptedPrompter, Settings

HERE = os.path.dirname(os.path.abspath(__file__))
FAKE_TF = os.path.join(HERE, "fixtures", "fake_terraform.py")


def make_ctx(values: Optional[Dict[str, Any]] = None, answers: Optional[List[Any]] = None,
             non_interactive: bool = True, cloud=None, env: Optional[Dict[str, str]] = None) -> Context:
    vals = dict(values or {})
    if non_interactive:
        vals.setdefault("non-interactive", True)
    prompter = ScriptedPrompter(answers or []) if answers is not None or not non_interactive else None
    ctx = Context(settings=Settings(vals, env=env or {}), prompter=prompter, out=io.StringIO(), cloud=cloud)
    return ctx


def output(ctx: Context) -> str:
    return ctx.out.getvalue()


def install_fake_terraform(tmp_path, monkeypatch, version: str = "1.5.7", fail: str = "") -> str:
    bindir = tmp_path / "bin"
    bindir.mkdir(exist_ok=True)
    exe = bindir / "terraform"
    exe.write_text(f"#!/bin/sh\nexec {sys.executable} {FAKE_TF} \"$@\"\n")
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)
    log = tmp_path / "tf.log"
    monkeypatch.setenv("PATH", f"{bindir}{os.pathsep}{os.environ.get('PATH', '')}")
    monkeypatch.setenv("FAKE_TF_LOG", str(log))
    monkeypatch.setenv("FAKE_TF_VERSION", version)
    if fail:
        monkeypatch.setenv("FAKE_TF_FAIL", fail)
    else:
        monkeypatch.delenv("FAKE_TF_FAIL", raising=False)
    return str(log)


def tf_calls(log_path: str) -> List[Dict[str, Any]]:
    if not os.path.exists(log_path):
        return []
    with open(log_path, "r", encoding="utf-8") as fh:
        return [json.loads(line) for line in fh if line.strip()]


def make_ssh_key(path, kind: str = "rsa") -> str:
    args = ["ssh-keygen", "-q", "-t", kind, "-N", "", "-f", str(path)]
    if kind == "rsa":
        args[4:4] = ["-b", "2048", "-m", "PEM"]
    subprocess.run(args, check=True, capture_output=True)
    return str(path)


def have(binary: str) -> bool:
    return shutil.which(binary) is not None


def assert_blocks_match_modules(st) -> None:
    """Every module block of a rendered document points at a module directory that exists
    (the packaged tree by default), every key it sets is a variable declared there, every
    required variable is set, and every value passes the variable's type and ``validation``
    conditions — read from the module's own .tf files with the HCL parser and evaluator,
    not from the generator's data."""
    import os

    from triton_kubernetes_amd.terraform import catalog, hcl

    for key, block in (st.doc.get("module") or {}).items():
        info = catalog.module_from_source(block["source"])
        assert info is not None, f"{key}: unknown module source {block['source']}"
        local = catalog.local_module_dir(block["source"])
        mod_dir = local if local is not None else info.local_dir
        assert os.path.isfile(os.path.join(mod_dir, "main.tf")), f"{key}: {block['source']} has no main.tf"
        rep = hcl.check_module(mod_dir)
        assert not rep.errors, rep.errors
        extra = set(block) - {"source"} - rep.variables
        assert not extra, f"{key} -> {info.name}: keys not declared as module variables: {sorted(extra)}"
        missing = rep.required - set(block)
        assert not missing, f"{key} -> {info.name}: required variables not set: {sorted(missing)}"
        # what `terraform plan` would reject: types and the modules' own validation blocks
        problems = hcl.check_inputs(mod_dir, block)
        assert not problems, f"{key} -> {info.name}: {problems}"
        # ... and every expression of the module evaluated for these inputs (terraform/plan.py)
        from triton_kubernetes_amd.terraform.plan import plan_module

        planned = plan_module(mod_dir, block, check_files=False)
        assert planned.ok, f"{key} -> {info.name}: {planned.errors}"