"""Host tuning checks at MI355X bring-up (``node/hosttune.py``): NUMA auto-balancing and
the IOMMU mode, from fixture /proc and /sys trees, on the agent and shell paths alike."""

import os
import subprocess

import pytest

from triton_kubernetes_amd.errors import ConfigError
from triton_kubernetes_amd.node import hosttune
from triton_kubernetes_amd.node.agent import NodeAgent
from triton_kubernetes_amd.node.labels import synthetic_topology
from triton_kubernetes_amd.node.plan import BURNIN_LABEL_FILE, build_host_plan


def host(root, numa="0", cmdline="BOOT_IMAGE=/vmlinuz root=/dev/sda1 iommu=pt", iommu_units=True):
    os.makedirs(os.path.join(root, "proc/sys/kernel"), exist_ok=True)
    if numa is not None:
        with open(os.path.join(root, "proc/sys/kernel/numa_balancing"), "w") as fh:
            fh.write(numa + "\n")
    with open(os.path.join(root, "proc/cmdline"), "w") as fh:
        fh.write(cmdline + "\n")
    if iommu_units:
        os.makedirs(os.path.join(root, "sys/class/iommu/ivhd0"), exist_ok=True)
    return root


CASES = [  # (numa, cmdline, iommu units) -> facts
    (("0", "ro iommu=pt", True), {"numa_balancing": "off", "iommu": "pt"}),
    (("1", "ro amd_iommu=pt", True), {"numa_balancing": "on", "iommu": "pt"}),
    (("0", "ro quiet", True), {"numa_balancing": "off", "iommu": "translated"}),
    (("0", "ro amd_iommu=off", True), {"numa_balancing": "off", "iommu": "off"}),
    ((None, "ro", False), {"numa_balancing": "unknown", "iommu": "off"}),
]


@pytest.mark.parametrize("args,want", CASES)
def test_facts_and_shell_twin(tmp_path, args, want):
    root = host(str(tmp_path / "h"), *args)
    f = hosttune.facts(root)
    assert f == want
    assert hosttune.labels(f) == {"amd.com/host.numa-balancing": want["numa_balancing"],
                                  "amd.com/host.iommu": want["iommu"]}
    # the shell check over the same tree: same labels, warnings, enforce exits 1
    for policy in ("warn", "enforce"):
        labels = tmp_path / policy / "etc" / "labels"  # its directory does not exist yet
        body = hosttune.shell_check(policy, str(labels)).replace("sudo ", "")
        for path in ("/proc/sys/kernel/numa_balancing", "/proc/cmdline", "/sys/class/iommu"):
            body = body.replace(path, root + path)
        p = subprocess.run(["bash", "-c", "set -euo pipefail\nf() {\n" + body + "\n}\nf"], capture_output=True,
                           text=True)
        got = dict(ln.split("=", 1) for ln in labels.read_text().splitlines())
        assert got == hosttune.labels(f), p.stderr
        bad = hosttune.problems(f)
        assert p.returncode == (1 if bad and policy == "enforce" else 0), p.stderr
        assert ("host tuning:" in p.stderr) == bool(bad)
    assert hosttune.shell_check("off", "x") == ""


def test_policy():
    assert hosttune.policy_of({}) == "warn"
    with pytest.raises(ConfigError, match="gpu_host_tuning must be one of warn, enforce, off"):
        hosttune.policy_of({"gpu_host_tuning": "strict"})


@pytest.mark.parametrize("policy", ["warn", "enforce", "off"])
def test_agent_preflight(tmp_path, policy):
    root = host(str(tmp_path / "node"), numa="1", cmdline="ro quiet")  # untuned: both problems
    agent = NodeAgent(name="n", mode="sim", devices=list(range(8)), token="t" * 24, root=root,
                      topology_override=synthetic_topology(8), burnin_override=lambda d, lvl: {"ok": True})
    try:
        cfg = {"hostname": "g", "rancher_host_labels": {"worker": "true"}, "gpu_count": 8,
               "gpu_host_tuning": policy}
        plan = build_host_plan(cfg, "http://127.0.0.1:9", "t", "s", mi355x=True)
        plan.steps = [s for s in plan.steps if s.action != "agent"]
        res = agent.run_plan(plan)
    finally:
        agent.stop()
    pre = next(s for s in res["steps"] if s["name"] == "gpu_preflight")
    if policy == "enforce":
        assert not res["ok"] and "host tuning: kernel.numa_balancing is on" in res["error"]
        return
    assert res["ok"], res
    if policy == "off":
        assert "host" not in pre["detail"] and "amd.com/host.iommu" not in res["labels"]
        return
    assert pre["detail"]["host"]["iommu"] == "translated" and len(pre["detail"]["host"]["warnings"]) == 2
    assert res["labels"]["amd.com/host.numa-balancing"] == "on"


def test_burnin_keeps_the_host_labels():
    """The shell preflight writes the host labels into the extra-labels file; the burn-in
    step appends to it instead of replacing it."""
    cfg = {"hostname": "g", "rancher_host_labels": {"worker": "true"}, "gpu_count": 8}
    plan = build_host_plan(cfg, "https://r", "t", "s", mi355x=True)
    pre = next(s for s in plan.steps if s.name == "gpu_preflight")
    burn = next(s for s in plan.steps if s.name == "gpu_burnin")
    assert f"sudo tee -a {BURNIN_LABEL_FILE} >/dev/null" in pre.shell and pre.params["host_tuning"] == "warn"
    assert f"sudo tee -a {BURNIN_LABEL_FILE} < /tmp/tk-burnin-labels" in burn.shell
    assert "install -m 0644 /tmp/tk-burnin-labels" not in burn.shell


def test_terraform_host_script_renders_the_tuning_policy():
    from triton_kubernetes_amd.terraform import plan as tfplan
    from triton_kubernetes_amd.terraform.catalog import MODULES_DIR

    mod = os.path.join(MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host")
    result = {}
    for policy in ("warn", "enforce", "off"):
        res = tfplan.plan_module(mod, {"hostname": "g", "host": "10.0.0.9", "rancher_api_url": "https://r",
                                       "rancher_cluster_registration_token": "t", "rancher_cluster_ca_checksum": "c",
                                       "rancher_host_labels": {"worker": "true"}, "gpu_host_tuning": policy},
                                 check_files=False)
        assert not res.errors, res.errors
        script = "\n".join(str(x) for x in _strings(res))
        result[policy] = script
    assert "amd.com/host.numa-balancing" in result["warn"] and "|| true" in result["warn"]
    assert "[ $_tk_bad = 0 ] || exit 1" in result["enforce"]
    assert "amd.com/host.numa-balancing" not in result["off"]


def _strings(res):
    """Every rendered string of a planned module (the remote-exec inline scripts among them)."""
    out = []

    def walk(v):
        if isinstance(v, str):
            out.append(v)
        elif isinstance(v, dict):
            for x in v.values():
                walk(x)
        elif isinstance(v, (list, tuple)):
            for x in v:
                walk(x)

    walk(getattr(res, "resources", None) or getattr(res, "values", None) or res.__dict__)
    return out


def test_gpu_policy_variables_are_validated():
    """The MI355X host module's GPU policy variables carry validation blocks: the HCL input
    check and the planner refuse what Terraform would ("Invalid value for variable")."""
    import os

    from triton_kubernetes_amd.terraform import hcl
    from triton_kubernetes_amd.terraform.catalog import MODULES_DIR
    from triton_kubernetes_amd.terraform.plan import plan_module

    mod = os.path.join(MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host")
    base = {"hostname": "g", "rancher_api_url": "https://r", "rancher_cluster_registration_token": "t",
            "rancher_cluster_ca_checksum": "c", "rancher_host_labels": {"worker": "true"}, "host": "10.0.0.9"}
    good = dict(base, gpu_health="taint", gpu_host_tuning="enforce", gpu_max_uncorrectable_ecc="2",
                gpu_max_retired_pages="auto", gpu_metrics_textfile="/var/lib/node_exporter/textfile")
    assert not [p for p in hcl.check_inputs(mod, good) if "gpu_" in p]
    assert not [e for e in plan_module(mod, good, check_files=False).errors if "Invalid value" in e]
    for key, bad in (("gpu_health", "warn"), ("gpu_host_tuning", "strict"), ("gpu_max_uncorrectable_ecc", "-1"),
                     ("gpu_max_retired_pages", "lots"), ("gpu_metrics_textfile", "relative/dir"),
                     ("gpu_metrics_textfile", "/var/../etc")):
        problems = hcl.check_inputs(mod, dict(good, **{key: bad}))
        assert any(key in p for p in problems), (key, bad, problems)
        errors = plan_module(mod, dict(good, **{key: bad}), check_files=False).errors
        assert any(f"Invalid value for variable '{key}'" in e for e in errors), (key, bad, errors)
