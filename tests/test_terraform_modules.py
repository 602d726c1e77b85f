"""Generated Terraform module library (T1–T17 + MI355X modules).

* the committed ``terraform/modules`` tree is exactly what the generator emits;
* every ``var.X`` a module uses is declared, and every key the providers write
  into a module block is a variable of that module;
* every shell template renders (templatefile directives expanded with dummy
  values) to syntactically valid bash.
"""

import json
import os
import re
import subprocess

import pytest

from triton_kubernetes_amd.terraform import catalog, generate, scripts

MODULES = generate.modules()
BY_NAME = {m.name: m for m in MODULES}


def _declared(mod):
    return {v.name for v in mod.variables}


def test_catalog_and_generator_agree():
    assert sorted(BY_NAME) == sorted(m.name for m in catalog._MODULES)
    assert len(catalog.REFERENCE_MODULES) == 17


@pytest.mark.parametrize("mod", MODULES, ids=lambda m: m.name)
def test_committed_tree_in_sync(mod):
    root = os.path.join(catalog.MODULES_DIR, mod.name)
    want = generate.rendered_files(mod)
    on_disk = set()
    for dirpath, _, files in os.walk(root):
        for f in files:
            on_disk.add(os.path.relpath(os.path.join(dirpath, f), root))
    assert on_disk == set(want), "run: python -m triton_kubernetes_amd.terraform.generate"
    for rel, content in want.items():
        with open(os.path.join(root, rel), encoding="utf-8") as fh:
            assert fh.read() == content, f"{mod.name}/{rel} is stale"


@pytest.mark.parametrize("mod", MODULES, ids=lambda m: m.name)
def test_var_references_declared(mod):
    text = generate.render_main(mod) + generate.render_outputs(mod)
    used = set(re.findall(r"\bvar\.([A-Za-z_][A-Za-z0-9_]*)", text))
    missing = used - _declared(mod)
    assert not missing, f"{mod.name}: undeclared variables {sorted(missing)}"


@pytest.mark.parametrize("mod", MODULES, ids=lambda m: m.name)
def test_outputs_match_catalog(mod):
    info = next(m for m in catalog._MODULES if m.name == mod.name)
    assert {o[0] for o in mod.outputs} >= set(info.outputs)


def _render_template(text: str, values=None) -> str:
    """Minimal templatefile(): keeps every %{ if } branch, substitutes ${x}, unescapes $${."""
    values = values or {}
    out = []
    for line in text.splitlines():
        if re.match(r"^\s*%\{.*\}\s*$", line):
            continue
        out.append(line)
    body = "\n".join(out) + "\n"
    body = body.replace("$${", "\x00")
    body = re.sub(r"\$\{([A-Za-z_][A-Za-z0-9_]*)\}", lambda m: str(values.get(m.group(1), "x")), body)
    return body.replace("\x00", "${")


TEMPLATES = {name: getattr(scripts, name) for name in dir(scripts)
             if name.isupper() and isinstance(getattr(scripts, name), str)}


@pytest.mark.parametrize("name", sorted(TEMPLATES))
def test_scripts_are_valid_bash(name):
    text = TEMPLATES[name]
    if name in ("INSTALL_DOCKER", "INSTALL_RANCHER_SERVER", "SETUP_RANCHER", "INSTALL_RANCHER_AGENT",
                "INSTALL_MI355X_NODE"):
        text = _render_template(text, {"gpu_count": 8, "rccl_min_busbw": 0, "extra_agent_args": ""})
    proc = subprocess.run(["bash", "-n"], input=text, capture_output=True, text=True, check=False)
    assert proc.returncode == 0, f"{name}: {proc.stderr}"


def test_generated_module_files_are_valid_bash():
    for mod in MODULES:
        for rel, content in generate.rendered_files(mod).items():
            if not (rel.endswith(".sh") or rel.endswith(".sh.tftpl")):
                continue
            text = _render_template(content, {"gpu_count": 8}) if rel.endswith(".tftpl") else content
            proc = subprocess.run(["bash", "-n"], input=text, capture_output=True, text=True, check=False)
            assert proc.returncode == 0, f"{mod.name}/{rel}: {proc.stderr}"


def test_mi355x_template_uses_labeller_flag_the_binary_implements():
    src = open(os.path.join(generate.CSRC, "tk_topo.cpp"), encoding="utf-8").read()
    assert '"--labels"' in src
    assert "amdgpu-topo-labeller --labels" in scripts.INSTALL_MI355X_NODE
