"""HCL2 parser + static module checker (terraform/hcl.py) over all 19 shipped modules.

No terraform binary exists in CI, so the modules are parsed here: syntax (blocks,
strings, heredocs, ``%{}`` directives), references (var/local/data/resource), and
``templatefile`` vars against the placeholders of the template they render.  Each
check must also fail on a deliberately broken fixture.
"""

import os
import shutil

import pytest

from triton_kubernetes_amd.terraform import catalog, hcl

MODULE_NAMES = sorted(os.listdir(catalog.MODULES_DIR))


def test_all_nineteen_modules_present():
    assert len(MODULE_NAMES) == 19 and set(MODULE_NAMES) == set(catalog.CATALOG)


@pytest.mark.parametrize("name", MODULE_NAMES)
def test_module_parses_and_cross_checks(name):
    rep = hcl.check_module(os.path.join(catalog.MODULES_DIR, name))
    assert not rep.errors, "\n".join(rep.errors)
    assert set(rep.files) == {"main.tf", "variables.tf", "outputs.tf", "versions.tf"}
    info = catalog.CATALOG[name]
    assert set(info.outputs) <= rep.outputs


@pytest.mark.parametrize("name", MODULE_NAMES)
def test_templates_parse(name):
    files = os.path.join(catalog.MODULES_DIR, name, "files")
    for dirpath, _, fnames in os.walk(files):
        for fn in fnames:
            if fn.endswith(".tftpl"):
                with open(os.path.join(dirpath, fn), encoding="utf-8") as fh:
                    hcl.parse_template(fh.read(), fn)


def test_templatefile_calls_found_and_matched():
    rep = hcl.check_module(os.path.join(catalog.MODULES_DIR, "bare-metal-rancher"))
    calls = [n for n in hcl.walk(rep.files["main.tf"]) if n.kind == "call" and n.value == "templatefile"]
    assert [hcl._module_relative_path(c.children[0]) for c in calls] == [
        "files/install_docker.sh.tftpl", "files/install_rancher_server.sh.tftpl", "files/setup_rancher.sh.tftpl"]


GOOD = [
    'a = { k = 1, k2 = 2 }',
    'a = [for k, v in m : v if k != "x"]',
    'a = {for k, v in m : k => v...}',
    'x = a.b[0].c[*].d',
    'x = !a && b || c ? 1 : -2',
    'x = f(a...)',
    'x = <<-EOT\n  %{for x in y~}\n  ${x}\n  %{endfor~}\n  EOT\n',
    'x = "$${lit} %%{lit}"',
    'resource "a" "b" {\n  dynamic "d" {\n    for_each = var.x\n    content { v = d.value }\n  }\n}\n',
    'x = (\n  1 +\n  2\n)',
]
BAD = [
    'a = {',
    'x = 1 +',
    'resource "a" "b" {\n c = "x\n}',
    'a = <<EOT\nhello\n',
    'a = "${var.x"',
    'a = "%{ if x }y"',
    'a = "%{ endif }"',
    'a = [for x in y : ]',
    'b {\n c = d e\n}',
    'a = f(1,,2)',
    'a = { k = 1 k2 = 2 }',
    'a = "\\q"',
    'block "x" {\n a = 1\n',
]


@pytest.mark.parametrize("src", GOOD)
def test_parser_accepts(src):
    hcl.parse(src)


@pytest.mark.parametrize("src", BAD)
def test_parser_rejects(src):
    with pytest.raises(hcl.HCLSyntaxError):
        hcl.parse(src)


def _broken_copy(tmp_path, edit):
    src = os.path.join(catalog.MODULES_DIR, "bare-metal-rancher")
    dst = tmp_path / "bare-metal-rancher"
    shutil.copytree(src, dst, symlinks=True)
    edit(dst)
    return hcl.check_module(str(dst))


def _replace(path, old, new):
    text = path.read_text()
    assert old in text, old
    path.write_text(text.replace(old, new, 1))


@pytest.mark.parametrize("case,edit,expect", [
    ("syntax", lambda d: _replace(d / "main.tf", "triggers_replace = [local.rancher_master_id]",
                                  "triggers_replace = [local.rancher_master_id"), "expected"),
    ("templatefile missing var", lambda d: _replace(d / "main.tf", "      bootstrap_password   = local.bootstrap_password\n",
                                                    ""), "does not pass ['bootstrap_password']"),
    ("templatefile unused var", lambda d: _replace(d / "main.tf", "      bootstrap_password   = local.bootstrap_password\n",
                                                   "      bootstrap_password   = local.bootstrap_password\n"
                                                   "      extra_thing          = 1\n"), "passes unused ['extra_thing']"),
    ("undeclared var", lambda d: _replace(d / "main.tf", "var.ssh_user", "var.ssh_usr"), "undeclared variable var.ssh_usr"),
    ("undefined local", lambda d: _replace(d / "main.tf", "local.rancher_master_ip\n", "local.rancher_master_ipp\n"),
     "undefined local.rancher_master_ipp"),
    ("undefined resource", lambda d: _replace(d / "main.tf", "[terraform_data.install_docker]",
                                              "[terraform_data.install_dockr]"),
     "undefined resource terraform_data.install_dockr"),
    ("template directive", lambda d: _replace(d / "files" / "install_docker.sh.tftpl", "%{ endif ~}\n", "", ),
     "is never closed"),
    ("template missing file", lambda d: os.remove(d / "files" / "setup_rancher.sh.tftpl"), "missing file"),
    # list()/map() were removed in Terraform 0.15; a typo'd function does not plan either
    ("removed function", lambda d: _replace(d / "main.tf", "[terraform_data.install_docker]",
                                                                  "list(terraform_data.install_docker)"),
     "unknown function list()"),
    ("provider not required", lambda d: _replace(d / "versions.tf", "    external = {", "    externall = {"),
     "external needs provider 'external'"),
])
def test_checker_catches_broken_fixture(tmp_path, case, edit, expect):
    rep = _broken_copy(tmp_path, edit)
    assert any(expect in e for e in rep.errors), (case, rep.errors)


def test_template_names_respect_for_bindings():
    parts = hcl.parse_template("%{ for x in items ~}${x}-${suffix}%{ endfor ~}${other.attr}")
    assert hcl.template_names(parts) == {"items", "suffix", "other"}


def test_check_inputs_evaluates_the_modules_validations():
    import os

    from triton_kubernetes_amd.terraform.catalog import MODULES_DIR

    mod = os.path.join(MODULES_DIR, "bare-metal-rancher-k8s")
    base = {"name": "c", "rancher_api_url": "${module.cluster-manager.rancher_url}",
            "rancher_access_key": "${module.cluster-manager.rancher_access_key}",
            "rancher_secret_key": "${module.cluster-manager.rancher_secret_key}",
            "k8s_version": "v1.28.10-rancher1-1", "k8s_network_provider": "calico"}
    assert hcl.check_inputs(mod, base) == []
    bad = hcl.check_inputs(mod, dict(base, k8s_version="v1.9.5-rancher1-1", k8s_network_provider="weird", extra=1))
    assert any(e.startswith("k8s_version: k8s_version must be an RKE2 (") for e in bad), bad
    assert any(e.startswith("k8s_network_provider:") for e in bad) and "unsupported argument 'extra'" in bad
    assert "missing required argument 'name'" in hcl.check_inputs(mod, {k: v for k, v in base.items() if k != "name"})
    mgr = os.path.join(MODULES_DIR, "bare-metal-rancher")
    pw = {"name": "m", "host": "10.0.0.1", "rancher_admin_password": "short"}
    assert any("at least 12 characters" in e for e in hcl.check_inputs(mgr, pw))
    assert any("at least 12 characters" in e for e in hcl.check_inputs(mgr, dict(pw, rancher_admin_password="quote'pw123456")))
    assert not [e for e in hcl.check_inputs(mgr, dict(pw, rancher_admin_password="long-enough-pw-1")) if "password" in e]
    host = os.path.join(MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host")
    errs = hcl.check_inputs(host, {"rancher_host_labels": {"worker": "true", "etcd": "true"}, "gpu_burnin": "max",
                                   "gpu_count": "eight"})
    assert any(e.startswith("rancher_host_labels:") for e in errs) and any(e.startswith("gpu_burnin:") for e in errs)
    assert any("gpu_count: 'eight' is not a number" == e for e in errs), errs


@pytest.mark.parametrize("src,want", [
    ('[for k, v in m : "${k}=${v}"]', ["a=1", "b=2"]),
    ('[for v in l : upper(v) if v != "y"]', ["X", "Z"]),
    ('[for i, v in l : i]', [0, 1, 2]),
    ('{for k, v in m : v => k}', {"1": "a", "2": "b"}),
    ('alltrue([for v in l : length(v) == 1])', True),
    ('anytrue([for v in l : v == "q"])', False),
    ('length(regexall("^W$", "W\\n"))', 0),  # RE2: "$" is the end of the text
])
def test_expression_evaluator_for_expressions_and_list_predicates(src, want):
    """for-expressions (lists, maps in key order, object form, if filters), alltrue/anytrue,
    and RE2's end-of-text "$": what the modules' variable validations use."""
    body = hcl.parse(f"x = {src}\n")
    expr = body.attr("x").expr
    assert hcl.eval_expr(expr, {"m": {"b": "2", "a": "1"}, "l": ["x", "y", "z"]}) == want


def test_regexall_translates_only_bare_dollars():
    """``$`` inside a character class or after an escaped backslash keeps its
    RE2 meaning (``[$]`` a literal; ``\\\\$`` a backslash at the end)."""
    from triton_kubernetes_amd.terraform import hcl as h

    assert h.re2_pattern("^a$") == "^a\\Z"
    assert h.re2_pattern("[$]x") == "[$]x"
    assert h.re2_pattern("[^]$]+$") == "[^]$]+\\Z"
    assert h.re2_pattern("\\\\$") == "\\\\\\Z"
    assert h.re2_pattern("a\\$b") == "a\\$b"
    regexall = h._FUNCS["regexall"]
    assert regexall("[$]", "cost: $5") == ["$"]
    assert regexall("\\\\$", "ends with \\") == ["\\"]
    assert regexall("^ab$", "ab\n") == []  # RE2: no match before a final newline
    assert regexall("^ab$", "ab") == ["ab"]


def test_module_report_parses_once_under_concurrent_first_calls(tmp_path, monkeypatch):
    """A cluster's host modules start their applies together; their input checks share one
    parse of the module (the others wait for it) instead of each parsing it again."""
    import threading
    import time

    src = os.path.join(catalog.MODULES_DIR, "bare-metal-rancher-k8s-host")
    mod = tmp_path / "bare-metal-rancher-k8s-host"
    shutil.copytree(src, mod)
    calls = []
    real = hcl.check_module

    def slow_check(d):
        calls.append(d)
        time.sleep(0.05)
        return real(d)

    monkeypatch.setattr(hcl, "check_module", slow_check)
    reports = []
    threads = [threading.Thread(target=lambda: reports.append(hcl.module_report(str(mod)))) for _ in range(16)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert len(calls) == 1 and len(reports) == 16 and all(r is reports[0] for r in reports)
