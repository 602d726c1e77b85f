"""Generated Terraform module library (T1–T17 + MI355X modules).

* the committed ``terraform/modules`` tree is exactly what the generator emits;
* every ``var.X`` a module uses is declared, and every key the providers write
  into a module block is a variable of that module;
* every shell template renders (templatefile directives expanded with dummy
  values) to syntactically valid bash.
"""

import os
import re
import subprocess

import pytest

from triton_kubernetes_amd.terraform import catalog, generate, hcl, scripts

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


def _hcl_structure_errors(text: str) -> list:
    """Lexical sanity of generated HCL: balanced {}/[]/() outside strings and comments,
    terminated strings and ${...}/%{...} templates, closed heredocs."""
    errs, stack = [], []
    i, n, line = 0, len(text), 1
    pairs = {"}": "{", "]": "[", ")": "("}
    while i < n:
        c = text[i]
        if c == "\n":
            line += 1
        if c == "#" or text.startswith("//", i):
            j = text.find("\n", i)
            i = n if j < 0 else j
            continue
        if text.startswith("/*", i):
            j = text.find("*/", i + 2)
            if j < 0:
                errs.append(f"line {line}: unterminated /* comment")
                break
            line += text.count("\n", i, j)
            i = j + 2
            continue
        if text.startswith("<<", i):
            m = re.match(r"<<-?([A-Za-z_]+)\n", text[i:])
            if m:
                end = re.search(r"^\s*" + m.group(1) + r"\s*$", text[i + m.end():], re.M)
                if not end:
                    errs.append(f"line {line}: heredoc {m.group(1)} not closed")
                    break
                seg = text[i:i + m.end() + end.end()]
                line += seg.count("\n")
                i += len(seg)
                continue
        if c == '"':
            j, depth = i + 1, 0
            while j < n:
                if text[j] == "\\":
                    j += 2
                    continue
                if text.startswith("${", j) or text.startswith("%{", j):
                    depth += 1
                    j += 2
                    continue
                if text[j] == "}" and depth:
                    depth -= 1
                elif text[j] == '"' and not depth:
                    break
                elif text[j] == "\n" and not depth:
                    errs.append(f"line {line}: newline in string")
                    break
                j += 1
            if j >= n:
                errs.append(f"line {line}: unterminated string")
                break
            line += text.count("\n", i, j)
            i = j + 1
            continue
        if c in "{[(":
            stack.append((c, line))
        elif c in "}])":
            if not stack or stack[-1][0] != pairs[c]:
                errs.append(f"line {line}: unbalanced {c!r}")
                break
            stack.pop()
        i += 1
    errs += [f"line {ln}: {ch!r} never closed" for ch, ln in stack]
    return errs


@pytest.mark.parametrize("mod", MODULES, ids=lambda m: m.name)
def test_hcl_is_lexically_well_formed(mod):
    for rel in ("main.tf", "variables.tf", "outputs.tf", "versions.tf"):
        text = generate.rendered_files(mod)[rel]
        assert not _hcl_structure_errors(text), (mod.name, rel, _hcl_structure_errors(text))
    assert _hcl_structure_errors('a = { b = "x"') == ["line 1: '{' never closed"]
    assert _hcl_structure_errors('a = "${var.x}" }')[0].startswith("line 1: unbalanced")


@pytest.mark.parametrize("module", ["bare-metal-mi355x-rancher-k8s-host", "bare-metal-rancher-k8s-host"])
@pytest.mark.parametrize("key,bad", [
    ("rancher_api_url", "https://r'; curl x | sh; '"), ("rancher_api_url", "ftp://r"),
    ("rancher_cluster_registration_token", "t' $(id) '"), ("rancher_cluster_ca_checksum", "c;id"),
    ("hostname", "h'x"), ("hostname", "-h"), ("rancher_registry_password", "p'w"),
    ("rancher_agent_image", "rancher/agent; id"), ("docker_install_sha256", "zz"),
])
def test_host_modules_refuse_values_that_would_break_out_of_the_script(module, key, bad):
    """The host scripts put these values inside single quotes or on a command line; the
    modules' validations refuse quotes and shell syntax, as the node agent does for its own
    steps (node/agent_steps.py)."""
    mod = os.path.join(catalog.MODULES_DIR, module)
    base = {"hostname": "gpu-1.example", "rancher_api_url": "https://rancher.example:8443",
            "rancher_cluster_registration_token": "abc123xyz", "rancher_cluster_ca_checksum": "0a" * 32,
            "rancher_host_labels": {"worker": "true"}, "host": "10.0.0.9"}
    assert not [p for p in hcl.check_inputs(mod, base) if "must be" in p or "must not" in p]
    problems = hcl.check_inputs(mod, dict(base, **{key: bad}))
    assert any(key in p for p in problems), (key, bad, problems)
