import os
"""Static plan of the Terraform modules (``terraform/plan.py``): every expression of a module
evaluated for concrete module-block inputs, the way ``terraform plan`` would, with
apply-time values unknown.  Broken copies of real modules show what it catches that the
syntax/reference checker (``hcl.check_module``) cannot."""

import shutil
import subprocess

import pytest

from triton_kubernetes_amd.terraform import catalog, hcl
from triton_kubernetes_amd.terraform.plan import UNKNOWN, _Scope, evaluate, plan_module

HOST = "bare-metal-mi355x-rancher-k8s-host"
HOST_INPUTS = {
    "hostname": "gpu-1", "host": "10.0.0.5", "rancher_api_url": "https://rancher.example",
    "rancher_cluster_registration_token": "tok123", "rancher_cluster_ca_checksum": "ab" * 32,
    "rancher_host_labels": {"worker": "true"}, "gpu_count": "8", "gpu_burnin": "full",
    "rccl_env": {"NCCL_IB_HCA": "=mlx5_0:1", "NCCL_SOCKET_IFNAME": "eth0"},
}


def _dir(name):
    return catalog.CATALOG[name].local_dir


@pytest.mark.parametrize("name", sorted(catalog.CATALOG))
def test_every_module_plans_with_apply_time_inputs(name):
    """Required inputs as ``${module...}`` interpolations (unknown until apply): every
    expression still evaluates; counts stay known at plan time."""
    rep = hcl.check_module(_dir(name))
    planned = plan_module(_dir(name), {v: "${module.up.out}" for v in rep.required}, check_files=False)
    assert planned.ok, planned.errors
    assert planned.instances and all(n >= 0 for n in planned.instances.values())


def test_mi355x_host_renders_its_install_script():
    planned = plan_module(_dir(HOST), HOST_INPUTS, check_files=False)
    assert planned.ok, planned.errors
    assert planned.locals["rancher_node_role"] == "worker"
    assert planned.locals["rccl_env_file"] == 'NCCL_IB_HCA="=mlx5_0:1"\nNCCL_SOCKET_IFNAME="eth0"'
    (script,) = planned.rendered["install_mi355x_node.sh.tftpl"]
    assert "tok123" in script and "gpu-1" in script and "--level 'full'" in script
    proc = subprocess.run(["bash", "-n"], input=script, capture_output=True, text=True, check=False)
    assert proc.returncode == 0, proc.stderr
    assert "--min-link-frac 0.5 " in script  # the module default
    tuned = plan_module(_dir(HOST), dict(HOST_INPUTS, gpu_link_min_frac="0.7"), check_files=False)
    assert "--min-link-frac 0.7 " in tuned.rendered["install_mi355x_node.sh.tftpl"][0]
    # a control node becomes Rancher's "controlplane" role
    ctl = plan_module(_dir(HOST), dict(HOST_INPUTS, rancher_host_labels={"control": "true"}), check_files=False)
    assert ctl.locals["rancher_node_role"] == "controlplane"


@pytest.mark.parametrize("name", ["bare-metal-rancher", "aws-rancher", "triton-rancher", "gcp-rancher",
                                  "azure-rancher"])
def test_module_bootstrap_password_is_the_given_random_one(name):
    """The first-login password is the one the CLI keeps in the state backend (rendered
    into rancher_bootstrap_password): no function of the admin password."""
    rep = hcl.check_module(_dir(name))
    inputs = {v: "${module.up.out}" for v in rep.required}
    inputs.update(name="mgr-1", rancher_admin_password="s3cret-passw0rd", rancher_bootstrap_password="Rnd-0123")
    planned = plan_module(_dir(name), inputs, check_files=False)
    assert planned.ok, planned.errors
    assert planned.locals["bootstrap_password"] == "Rnd-0123"
    main = open(os.path.join(_dir(name), "main.tf")).read()
    assert "sha256(" not in main and "rancher_admin_password" not in main.split("data \"external\"")[0]


def test_missing_ssh_key_is_an_error_only_when_files_are_checked(tmp_path):
    inputs = dict(HOST_INPUTS, key_path=str(tmp_path / "absent"))
    assert plan_module(_dir(HOST), inputs, check_files=False).ok
    strict = plan_module(_dir(HOST), inputs, check_files=True)
    assert any("no such file" in e and "absent" in e for e in strict.errors)
    key = tmp_path / "id"
    key.write_text("KEY")
    assert plan_module(_dir(HOST), dict(inputs, key_path=str(key)), check_files=True).ok


def test_input_conversion_errors():
    bad = plan_module(_dir(HOST), dict(HOST_INPUTS, gpu_count="eight"), check_files=False)
    assert any("'eight' is not a number" in e for e in bad.errors)
    bad = plan_module(_dir(HOST), dict(HOST_INPUTS, rccl_env=["x"]), check_files=False)
    assert any("is not a map" in e for e in bad.errors)


def _broken(tmp_path, name, rel, old, new):
    dst = tmp_path / name
    shutil.copytree(_dir(name), dst, symlinks=True)
    path = dst / rel
    text = path.read_text()
    assert old in text, old
    path.write_text(text.replace(old, new, 1))
    return str(dst)


@pytest.mark.parametrize("name,rel,old,new,expect", [
    # a counted data source read without an instance key
    ("triton-rancher", "main.tf", "data.triton_network.networks[*].id", "data.triton_network.networks.id",
     "an instance key is required"),
    # count must be known at plan time
    ("aws-rancher", "main.tf", 'count      = var.aws_public_key_path != "" ? 1 : 0',
     'count      = aws_vpc.default.id != "" ? 1 : 0', "known only after apply"),
    # index past the end of a known list
    (HOST, "main.tf", "keys(var.rancher_host_labels)[0]", "keys(var.rancher_host_labels)[1]",
     "index 1 out of range"),
    # a list interpolated into the rendered install script
    (HOST, "main.tf", "gpu_burnin                         = var.gpu_burnin",
     "gpu_burnin                         = [var.gpu_burnin]", "cannot interpolate a list"),
    # wrong arity
    (HOST, "main.tf", "lookup({ spx = 1, dpx = 2, qpx = 4, cpx = 8 }, var.gpu_compute_partition, 1)",
     "lookup({ spx = 1, dpx = 2, qpx = 4, cpx = 8 })", "lookup() takes"),
    # locals that depend on each other
    (HOST, "main.tf", 'local.rancher_node_role_raw == "control"', 'local.rancher_node_role == "control"',
     "cycle among locals"),
])
def test_plan_catches_what_the_syntax_checker_cannot(tmp_path, name, rel, old, new, expect):
    mod = _broken(tmp_path, name, rel, old, new)
    assert not hcl.check_module(mod).errors  # still parses, every reference resolves
    inputs = HOST_INPUTS if name == HOST else dict(
        {v: "${module.up.out}" for v in hcl.check_module(mod).required},
        aws_public_key_path="~/.ssh/id_rsa.pub", triton_network_names=["a", "b"])
    inputs = {k: v for k, v in inputs.items() if k in hcl.check_module(mod).variables}
    planned = plan_module(mod, inputs, check_files=False)
    assert any(expect in e for e in planned.errors), planned.errors


def test_file_provisioner_source_must_exist(tmp_path):
    dst = tmp_path / HOST
    shutil.copytree(_dir(HOST), dst, symlinks=True)
    shutil.rmtree(dst / "files" / "src")
    planned = plan_module(str(dst), HOST_INPUTS, check_files=False)
    assert any("file provisioner source" in e and "files/src" in e for e in planned.errors), planned.errors


def _ev(src, **extra):
    class _P:
        def root(self, name):
            raise AssertionError(name)

    node = hcl.parse(f"x = {src}\n").attributes[0].expr
    return evaluate(node, _Scope(_P(), extra))


def test_expression_semantics():
    # unknown propagates through operators, functions and templates
    assert _ev("a + 1", a=UNKNOWN) is UNKNOWN
    assert _ev('"x-${a}"', a=UNKNOWN) is UNKNOWN
    assert _ev("length(a)", a=UNKNOWN) is UNKNOWN
    # the unselected branch's errors do not count; an unknown condition evaluates both
    assert _ev('c ? 1 : tonumber("x")', c=True) == 1
    with pytest.raises(ValueError):
        _ev('c ? 1 : tonumber("x")', c=UNKNOWN)
    # splat over a list of objects, for expressions with a filter, grouping
    assert _ev("xs[*].n", xs=[{"n": 1}, {"n": 2}]) == [1, 2]
    assert _ev("[for k, v in m : k if v > 1]", m={"a": 1, "b": 2}) == ["b"]
    assert _ev("{for s in xs : substr(s, 0, 1) => s...}", xs=["ab", "ac", "b"]) == {"a": ["ab", "ac"], "b": ["b"]}
    assert _ev('try(tonumber("x"), 7)') == 7 and _ev('can(tonumber("x"))') is False
    assert _ev('lookup(m, "k", "d")', m={}) == "d"
    with pytest.raises(ValueError, match="not in the map"):
        _ev('lookup(m, "k")', m={})
    assert _ev('replace("a-b-c", "/-([a-z])/", "_$1")') == "a_b_c"
    with pytest.raises(ValueError, match="unknown function"):
        _ev("frobnicate(1)")
