"""End-to-end MI355X bring-up on the real GPU (``pytest -m gpu``).

A bare-metal ``create cluster`` through the DirectExecutor whose worker agent
runs the native GPU steps for real: amd_smi topology labels, the default (full)
burn-in (HBM/MFMA/GEMM screens and a memtest of every free byte of HBM), then the
readiness waiter's RCCL gate.
"""

import json
import tempfile

import pytest

pytestmark = pytest.mark.gpu


def test_real_gpu_bringup(tmp_path):
    from triton_kubernetes_amd.backend import LocalBackend
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.parallel.transport import AgentTransport
    from triton_kubernetes_amd.rancher.fake import FakeRancher
    from triton_kubernetes_amd.workflows import new_cluster, new_manager

    from helpers import make_ctx, output

    token = "gpu-e2e-token-1234"
    fake = FakeRancher.for_manager("mgr", "tk-admin-pw-0123").start()
    cp = NodeAgent(name="cp", mode="sim", token=token, root=tempfile.mkdtemp())
    w = NodeAgent(name="w0", mode="sim", devices=[0], token=token, root=tempfile.mkdtemp())
    cp_url, w_url = cp.serve(), w.serve()
    backend = LocalBackend(str(tmp_path / "state"))
    base = {"executor": "direct", "agent_token": token}
    try:
        new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr", rancher_admin_password="tk-admin-pw-0123",
                                  rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="u", bastion_host="", key_path="k")), backend)
        # the default distribution: an RKE2 custom cluster (nodes register as rancher-system-agent)
        ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="gpu",
                            k8s_version="v1.31", k8s_network_provider="canal", gpu_addons=True,
                            wait=True, rccl_gate=True, nodes=[
                                {"rancher_host_label": "control", "node_count": 1, "hostname": "cp", "ssh_user": "u",
                                 "bastion_host": "", "key_path": "k", "hosts": ["agent+" + cp_url]},
                                {"rancher_host_label": "etcd", "node_count": 1, "hostname": "etcd", "ssh_user": "u",
                                 "bastion_host": "", "key_path": "k", "hosts": ["agent+" + cp_url]},
                                {"rancher_host_label": "worker", "node_count": 1, "hostname": "mi355x",
                                 "ssh_user": "u", "bastion_host": "", "key_path": "k", "hosts": ["agent+" + w_url],
                                 "gpu": "mi355x", "gpu_count": 1},
                            ]))
        ctx.extras["agent_transport"] = AgentTransport(token=token)
        new_cluster(ctx, backend)
        assert "rccl_gate" in output(ctx)
        labels = w.last_labels
        print(json.dumps(labels, indent=1))
        assert labels["amd.com/gpu.present"] == "true"
        assert labels["amd.com/gpu.target"] == "gfx950"
        assert labels["amd.com/gpu.product-name"].startswith("MI355")
        hist = w.history[-1]
        burn = [s for s in hist["steps"] if s["name"] == "gpu_burnin"][0]
        assert burn["ok"] and burn["detail"]["0"]["ok"], burn
        # the product default is the full burn-in: every free byte of HBM memtested, and the
        # node's labels say so (>= 300 GB of the 288 GiB card when the GPU is one SPX/NPS1 device)
        rep = ctx.extras["last_readiness"]
        # the labels the node joined with (the topology labels above plus the burn-in's)
        (joined,) = [d["labels"] for d in rep.nodes.values() if d["labels"].get("amd.com/gpu.present") == "true"]
        assert joined["amd.com/gpu.burnin"] == "passed" and joined["amd.com/gpu.burnin-level"] == "full", joined
        tested_gib = int(joined["amd.com/gpu.burnin-hbm-tested-gib"])
        if (labels.get("amd.com/gpu.compute-partition", "spx").lower(),
                labels.get("amd.com/gpu.memory-partition", "nps1").lower()) == ("spx", "nps1"):
            assert tested_gib * (1 << 30) >= 300e9, labels
        else:
            assert tested_gib >= 16, labels
        # the gate's verdict: one RCCL all-reduce sweep over the node's GPU, passed
        assert rep.rccl and rep.rccl["ok"] is True and rep.rccl.get("world", 1) == 1, rep.rccl
        assert "rccl_gate" in rep.phases
        print(json.dumps({"burnin_ms": burn.get("ms"), "hbm_tested_gib": tested_gib, "rccl": rep.rccl}, default=str))
        assert {n["agentKind"] for n in fake.state.nodes.values()} == {"system-agent"}
        assert "fleet-default/gpu" in fake.state.v2_clusters
    finally:
        w.stop()
        cp.stop()
        fake.stop()


# a curl that serves an empty /cacerts (a publicly trusted server) and an installer that
# records its arguments
CURL_STUB = """while [ $# -gt 0 ]; do case $1 in -o) out=$2; shift;; http*) url=$1;; esac; shift; done
case $url in */cacerts) : > "$out";; *) printf '#!/bin/sh\\necho "system-agent-install $*" >> {log}\\n' > "$out";; esac"""


def _stub(bindir, name, body):
    p = bindir / name
    p.write_text("#!/bin/bash\n" + body + "\n")
    p.chmod(0o755)


@pytest.mark.parametrize("rccl_slim,dist,burnin", [("off", "rke2", "quick"), ("on", "rke1", "quick"),
                                                    ("off", "rke2", "full")])
def test_rendered_shell_bootstrap_runs_on_mi355x(tmp_path, rccl_slim, dist, burnin):
    """The SSH path's rendered bash bootstrap, run for real on the box: the native tools
    (gpu-burnin, amdgpu-topo-labeller incl. --rccl-env, rccl-ready) copied from ops/lib,
    /etc relocated under tmp_path, and only sudo/docker/curl/systemctl/hostnamectl/usermod/lsmod
    stubbed (no root, no container runtime, no Rancher on the box; the stub curl serves an
    installer that records its arguments).  ``rccl_slim=on``: the opt-in step verifies the
    single-target copy on the GPU before installing rccl-ready-slim.  RKE2 joins through the
    system-agent installer, RKE1 through docker run rancher-agent."""
    import os
    import shutil
    import subprocess

    from triton_kubernetes_amd.node.plan import TOOLS_DIR, build_host_plan, parse_step_markers
    from triton_kubernetes_amd.ops.native import LIB_DIR, SYSTEM_LIB_DIR
    from triton_kubernetes_amd.parallel.rccl_env import parse_env_file

    tools = tmp_path / "tools"
    tools.mkdir()
    for exe in ("amdgpu-topo-labeller", "gpu-burnin", "rccl-ready"):
        shutil.copy2(os.path.join(LIB_DIR, exe), tools / exe)
    bindir = tmp_path / "bin"
    bindir.mkdir()
    log = tmp_path / "calls.log"
    _stub(bindir, "sudo", 'exec "$@"')
    for name in ("docker", "systemctl", "hostnamectl", "usermod"):
        _stub(bindir, name, f'echo "{name} $*" >> {log}')
    _stub(bindir, "curl", CURL_STUB.format(log=log))
    _stub(bindir, "lsmod", "echo 'Module Size Used by'; test -c /dev/kfd && echo 'amdgpu 1 0'")
    etc = tmp_path / "etc"
    (etc / "docker").mkdir(parents=True)
    cfg = {"hostname": "gpu-1", "rancher_host_labels": {"worker": "true"}, "gpu_count": 1, "gpu_burnin": burnin,
           "rccl_env": {"NCCL_DEBUG": "WARN"}, "rccl_slim": rccl_slim, "k8s_distribution": dist}
    plan = build_host_plan(cfg, "https://rancher.example", "regtok", "cafe", mi355x=True)
    script = (plan.render_shell().replace("/etc/", f"{etc}/").replace(TOOLS_DIR, str(tools))
              .replace("/var/lib/triton-kubernetes", str(tmp_path / "var")))
    env = dict(os.environ, PATH=f"{bindir}:{os.environ.get('PATH', '/usr/bin:/bin')}")
    proc = subprocess.run(["bash", "-s"], input=script, capture_output=True, text=True, env=env, timeout=300)
    assert proc.returncode == 0, proc.stderr[-3000:]
    steps = parse_step_markers(proc.stdout)
    print("\n".join(ln for ln in proc.stdout.splitlines() if "tk-step" in ln))
    assert all(steps.get(n, {}).get("status") == "ok" for n in plan.step_names()), steps
    burn = json.loads((etc / "triton-kubernetes/gpu-burnin.json").read_text())
    assert burn["ok"] and burn["gpus"] and all(g["ok"] for g in burn["gpus"]), burn
    assert burn["level"] == burnin
    if burnin == "full":  # every free byte but the headroom, on the SSH path too
        assert all(g["memtest_bytes"] >= 0.9 * g["hbm_bytes"] for g in burn["gpus"]), burn
    labels = dict(ln.split("=", 1) for ln in (etc / "triton-kubernetes/gpu-labels").read_text().splitlines())
    assert labels["amd.com/gpu.count"] == "1" and labels["amd.com/gpu.target"] == "gfx950"
    rccl = parse_env_file((etc / "rccl/rccl.env").read_text())
    assert rccl["NCCL_DEBUG"] == "WARN"
    if int(labels.get("amd.com/rdma.count", "0")) > 0:  # the box's RDMA ports land in the env
        assert rccl["NCCL_IB_HCA"].startswith("=")
    # default: the installed RCCL; opt-in: the verified copy through the wrapper
    if rccl_slim == "off":
        assert not (tools / "rccl-ready-slim").exists()
        tool, want = tools / "rccl-ready", os.path.join(SYSTEM_LIB_DIR, "librccl.so")
    else:
        assert (tools / "rccl-ready-slim").exists(), proc.stderr[-2000:]
        env_vals = dict(ln.split("=", 1) for ln in (tools / "rccl-slim.env").read_text().splitlines())
        tool, want = tools / "rccl-ready-slim", os.path.join(env_vals["TK_RCCL_SLIM_DIR"], "librccl.so")
    ready = subprocess.run(["timeout", "-k", "5", "120", str(tool), "--ngpus", "1", "--iters", "3", "--max-mib", "8",
                            "--expect-rccl", want], capture_output=True, text=True)
    assert ready.returncode == 0, ready.stdout[-2000:] + ready.stderr[-2000:]
    doc = json.loads([ln for ln in ready.stdout.splitlines() if ln.startswith("{")][-1])
    assert doc["ok"] and doc["rccl_mapped"], doc
    calls = log.read_text()
    assert "hostnamectl set-hostname gpu-1" in calls
    if dist == "rke2":
        assert "system-agent-install --server https://rancher.example" in calls and "docker" not in calls
        assert "--ca-checksum cafe --node-name gpu-1 --worker" in calls
    else:
        assert "docker run" in calls and "--ca-checksum cafe --worker" in calls
    assert "--label amd.com/gpu.product-name=MI355X" in calls
    print(json.dumps({"steps": steps, "rccl_env": rccl}))


@pytest.mark.parametrize("tools_from", ["prebuilt", "node-build"])
def test_terraform_mi355x_host_script_runs_on_mi355x(tmp_path, tools_from):
    """The bare-metal-mi355x-rancher-k8s-host module's host script (what Terraform's
    remote-exec runs), rendered from the module's own templatefile() call for concrete
    module inputs (terraform/plan.py) and run on the box: the node tools, then burn-in,
    labels, RCCL env and the RKE2 join.  ``prebuilt``: the CLI's staged gfx950 binaries
    (node/tools.py) are installed -- hipcc is never called, even on a re-run -- and the
    tool step's time is printed; ``node-build``: nothing staged, the node builds them from
    the shipped sources with hipcc/g++.  Paths relocated under tmp_path;
    sudo/curl/docker/hostnamectl/usermod/lsmod stubbed (the stub curl serves an installer
    that records its arguments)."""
    import os
    import re
    import subprocess

    from triton_kubernetes_amd.node import tools as node_tools
    from triton_kubernetes_amd.ops.build import CSRC
    from triton_kubernetes_amd.parallel.rccl_env import parse_env_file
    from triton_kubernetes_amd.terraform.generate import MODULES_DIR
    from triton_kubernetes_amd.terraform.plan import plan_module

    inputs = {"hostname": "gpu-tf-1", "host": "10.0.0.5", "rancher_api_url": "https://rancher.example",
              "rancher_cluster_registration_token": "regtok", "rancher_cluster_ca_checksum": "cafe",
              "rancher_host_labels": {"worker": "true"}, "gpu_count": "1", "gpu_burnin": "quick",
              "rccl_env": {"NCCL_DEBUG": "INFO"}, "k8s_distribution": "rke2"}
    planned = plan_module(os.path.join(MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host"), inputs, check_files=False)
    assert planned.ok, planned.errors
    (rendered,) = planned.rendered["install_mi355x_node.sh.tftpl"]
    tools, etc, prebuilt = tmp_path / "tools", tmp_path / "etc", tmp_path / "prebuilt"
    prebuilt.mkdir()
    if tools_from == "prebuilt":
        assert set(node_tools.stage(str(prebuilt)).values()) == {"prebuilt"}
    script = (rendered.replace("/opt/triton-kubernetes/bin", str(tools))
              .replace("/opt/triton-kubernetes/src", CSRC).replace(node_tools.PREBUILT_DIR, str(prebuilt))
              .replace("/etc/", f"{etc}/").replace("/var/lib/triton-kubernetes", str(tmp_path / "var")))
    bindir = tmp_path / "bin"
    bindir.mkdir()
    log = tmp_path / "calls.log"
    _stub(bindir, "sudo", 'exec "$@"')
    hipcc_log = tmp_path / "hipcc.log"
    _stub(bindir, "hipcc", f'echo "hipcc $*" >> {hipcc_log}; exec /opt/rocm/bin/hipcc "$@"')
    script = script.replace("$R/bin/hipcc", "hipcc")  # the node's compiler: the counting stub
    for name in ("docker", "hostnamectl", "usermod"):
        _stub(bindir, name, f'echo "{name} $*" >> {log}')
    _stub(bindir, "curl", CURL_STUB.format(log=log))
    _stub(bindir, "lsmod", "echo 'Module Size Used by'; test -c /dev/kfd && echo 'amdgpu 1 0'")
    env = dict(os.environ, PATH=f"{bindir}:{os.environ.get('PATH', '/usr/bin:/bin')}")
    proc = subprocess.run(["bash", "-s"], input=script, capture_output=True, text=True, env=env, timeout=280)
    assert proc.returncode == 0, proc.stderr[-3000:]
    for exe in ("amdgpu-topo-labeller", "gpu-burnin", "rccl-ready"):
        assert os.access(tools / exe, os.X_OK), exe
    tool_ms = int(re.search(r"node tools: (\d+) ms", proc.stdout).group(1))
    hipcc_calls = hipcc_log.read_text().splitlines() if hipcc_log.exists() else []
    print(json.dumps({"tools_from": tools_from, "node_tools_ms": tool_ms, "hipcc_calls": len(hipcc_calls)}))
    if tools_from == "prebuilt":
        assert hipcc_calls == [] and proc.stdout.count("prebuilt binary installed") == 3
        again = subprocess.run(["bash", "-s"], input=script, capture_output=True, text=True, env=env, timeout=280)
        assert again.returncode == 0, again.stderr[-3000:]
        assert not hipcc_log.exists() and again.stdout.count("installed copy is current") == 3
    else:
        assert len(hipcc_calls) == 2 and proc.stdout.count("building with") == 3
    # default (rccl_slim off): the node's rccl-ready runs on the installed /opt/rocm RCCL
    assert not (tools / "rccl-ready-slim").exists()
    dyn = subprocess.run(["readelf", "-d", str(tools / "rccl-ready")], capture_output=True, text=True).stdout
    assert "(RPATH)" not in dyn and "rccl-slim" not in dyn, [ln for ln in dyn.splitlines() if "PATH" in ln]
    ready = subprocess.run(["timeout", "-k", "5", "120", str(tools / "rccl-ready"), "--ngpus", "1", "--iters", "3",
                            "--expect-rccl", "/opt/rocm/lib/librccl.so"], capture_output=True, text=True)
    assert ready.returncode == 0, ready.stdout[-2000:] + ready.stderr[-2000:]
    doc = json.loads([ln for ln in ready.stdout.splitlines() if ln.startswith("{")][-1])
    assert doc["ok"] and doc["rccl_mapped"], doc
    burn = json.loads((etc / "triton-kubernetes/gpu-burnin.json").read_text())
    assert burn["ok"], burn
    labels = (etc / "triton-kubernetes/gpu-labels").read_text()
    assert "amd.com/gpu.product-name=MI355X" in labels
    assert parse_env_file((etc / "rccl/rccl.env").read_text())["NCCL_DEBUG"] == "INFO"
    calls = log.read_text()
    assert "hostnamectl set-hostname gpu-tf-1" in calls and "docker" not in calls  # RKE2: no Docker
    assert "system-agent-install --server https://rancher.example --label cattle.io/os=linux" in calls
    assert "--token regtok --ca-checksum cafe --node-name gpu-tf-1 --worker --label amd.com/" in calls
    # the burn-in's coverage travels with the node
    assert "--label amd.com/gpu.burnin-level=quick" in calls and "--label amd.com/gpu.burnin=passed" in calls
    assert "--label amd.com/gpu.burnin-hbm-tested-gib=1" in calls


@pytest.mark.parametrize("dist", ["rke2", "rke1"])
def test_node_agent_exec_mode_on_mi355x(tmp_path, monkeypatch, dist):
    """The production node agent mode (``exec``) over HTTP on the box: GPU steps run in
    process (arena burn-in, sysfs labels, discovered RCCL env), runtime/agent steps run
    their fixed argv against stubbed docker/hostnamectl (no container runtime on the box).
    RKE2: the agent fetches the (fake) server's system-agent-install.sh and runs it."""
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.plan import build_host_plan
    from triton_kubernetes_amd.parallel.transport import AgentTransport, HostRef
    from triton_kubernetes_amd.rancher.fake import FakeRancher

    bindir = tmp_path / "bin"
    bindir.mkdir()
    log = tmp_path / "calls.log"
    _stub(bindir, "docker", f'echo "docker $*" >> {log}; [ "$1" = version ] && echo 24.0.7; exit 0')
    _stub(bindir, "hostnamectl", f'echo "hostnamectl $*" >> {log}')
    import os

    monkeypatch.setenv("PATH", f"{bindir}:{os.environ.get('PATH', '/usr/bin:/bin')}")
    monkeypatch.setenv("TK_FAKE_SYSTEM_AGENT_LOG", str(log))  # what the fake's installer appends to
    fake = FakeRancher().start()
    agent = NodeAgent(name="w-exec", mode="exec", devices=[0], token="exec-token-123456", root=str(tmp_path / "root"))
    url = agent.serve()
    try:
        cfg = {"hostname": "gpu-exec-1", "rancher_host_labels": {"worker": "true"}, "gpu_count": 1,
               "gpu_burnin": "quick", "rccl_env": {"NCCL_DEBUG": "WARN"}, "k8s_distribution": dist}
        server = fake.url  # loopback: the default allow-list (both distributions' plans are checked)
        cid, token, checksum = fake.registration("exec", dist) if dist == "rke2" else ("", "regtok123", "cafe0123")
        plan = build_host_plan(cfg, server, token, checksum, mi355x=True)
        res = AgentTransport(token="exec-token-123456").run_plan(HostRef("agent+" + url), plan)
        joined = fake.k8s_nodes(cid) if dist == "rke2" else []
    finally:
        agent.stop()
        fake.stop()
    assert res["ok"], res
    names = [s["name"] for s in res["steps"]]
    assert names == plan.step_names() and all(s["ok"] for s in res["steps"])
    calls = log.read_text()
    assert "hostnamectl set-hostname gpu-exec-1" in calls
    if dist == "rke2":
        assert "docker" not in calls
        assert f"system-agent-install --server {fake.url} --label cattle.io/os=linux" in calls
        assert f"--ca-checksum {checksum} --node-name gpu-exec-1 --worker --label amd.com/" in calls
        # the installer checked the CA and registered the node, with the GPU labels
        (node,) = joined
        assert node["metadata"]["name"] == "gpu-exec-1"
        assert node["metadata"]["labels"]["amd.com/gpu.product-name"] == "MI355X"
    else:
        assert "docker version" in calls and "--ca-checksum cafe0123 --worker --label amd.com/" in calls
    assert "--label amd.com/gpu.count=1" in calls
    assert (tmp_path / "root/etc/rccl/rccl.env").read_text().count("NCCL_DEBUG") == 1
    print(json.dumps({s["name"]: round(s["ms"], 2) for s in res["steps"]}))


def test_exec_agent_rke2_teardown_then_another_cluster_on_mi355x(tmp_path, monkeypatch):
    """Destroy-time host teardown on the box (node/cleanup.py): an exec-mode agent joins
    cluster A through the fake's RKE2 installer (which models the host under TK_HOST_ROOT:
    connection info, RKE2 state and the vendor uninstallers, rancher/fake/hostsim.py); a
    join to cluster B is refused while A's install is there; ``/v1/cleanup`` runs the
    uninstallers at their fixed paths and removes the state; then B's join succeeds, with
    the GPU steps re-run on the card each time."""
    import os

    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.plan import build_host_plan
    from triton_kubernetes_amd.parallel.transport import AgentTransport, HostRef
    from triton_kubernetes_amd.rancher.fake import FakeRancher, hostsim

    bindir = tmp_path / "bin"
    bindir.mkdir()
    log = tmp_path / "calls.log"
    _stub(bindir, "hostnamectl", f'echo "hostnamectl $*" >> {log}')
    root = tmp_path / "root"
    monkeypatch.setenv("PATH", f"{bindir}:{os.environ.get('PATH', '/usr/bin:/bin')}")
    monkeypatch.setenv("TK_FAKE_SYSTEM_AGENT_LOG", str(log))
    monkeypatch.setenv("TK_HOST_ROOT", str(root))  # the fake installer models this host
    fake = FakeRancher().start()
    agent = NodeAgent(name="w-teardown", mode="exec", devices=[0], token="exec-token-123456", root=str(root))
    url = agent.serve()
    transport, ref = AgentTransport(token="exec-token-123456"), HostRef("agent+" + url)
    cfg = {"hostname": "gpu-td-1", "rancher_host_labels": {"worker": "true"}, "gpu_count": 1,
           "gpu_burnin": "quick", "k8s_distribution": "rke2"}
    try:
        cid_a, tok_a, ck_a = fake.registration("a", "rke2")
        first = transport.run_plan(ref, build_host_plan(cfg, fake.url, tok_a, ck_a, mi355x=True))
        assert first["ok"], first
        assert (root / hostsim.CONNECTION_INFO.lstrip("/")).exists()
        cid_b, tok_b, ck_b = fake.registration("b", "rke2")
        plan_b = build_host_plan(cfg, fake.url, tok_b, ck_b, mi355x=True)
        refused = transport.run_plan(ref, plan_b)
        assert not refused["ok"] and "another cluster" in json.dumps(refused), refused
        rep = transport.cleanup_host(ref)
        assert rep["ok"], rep
        ran = [a["what"] for a in rep["actions"] if a.get("status") == "ok"]
        assert any(w.endswith("rke2-uninstall.sh") for w in ran), rep
        assert any(w.endswith("rancher-system-agent-uninstall.sh") for w in ran), rep
        assert not (root / hostsim.CONNECTION_INFO.lstrip("/")).exists()
        assert not (root / "var/lib/rancher").exists()
        second = transport.run_plan(ref, plan_b)
        assert second["ok"], second
        (node,) = fake.k8s_nodes(cid_b)
        assert node["metadata"]["labels"]["amd.com/gpu.product-name"] == "MI355X"
        burn = [s for s in second["steps"] if s["name"] == "gpu_burnin"][0]
        assert burn["ok"], burn
    finally:
        agent.stop()
        fake.stop()
    # the SSH / Terraform path's teardown: the same steps as a script (node/cleanup.py,
    # markers ::tk-cleanup), run on this host model after B's join (sudo stubbed: no root here)
    from triton_kubernetes_amd.parallel.transport import LocalTransport

    _stub(bindir, "sudo", 'exec "$@"')
    script_rep = LocalTransport(env={"TK_HOST_ROOT": str(root), "PATH": os.environ["PATH"]}).cleanup_host(
        HostRef("local"))
    assert script_rep["ok"], script_rep
    assert [a["what"] for a in script_rep["actions"] if a.get("status") == "ok"] == [
        "/usr/local/bin/rancher-system-agent-uninstall.sh", "/usr/local/bin/rke2-killall.sh",
        "/usr/local/bin/rke2-uninstall.sh"], script_rep
    assert not (root / hostsim.CONNECTION_INFO.lstrip("/")).exists() and not (root / "var/lib/rancher").exists()
    print(json.dumps({"cleanup_ms": rep.get("ms"), "actions": rep["actions"], "script_actions": script_rep["actions"]}))


def test_exec_agent_rke1_teardown_then_another_cluster_on_mi355x(tmp_path, monkeypatch):
    """VERDICT r5 #3 on the box: an exec-mode agent joins RKE1 cluster A through a docker
    with Docker's own semantics (``fixtures/fake_docker.py``: the tagged agent, RKE's
    containers, the kubelet's pods), cluster B is refused while A's join stands,
    ``/v1/cleanup`` removes the agent and every pod container (the machine owner's stays),
    then B joins -- the GPU steps running on the card each time."""
    import os
    import subprocess
    import sys

    from triton_kubernetes_amd import versions
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.plan import build_host_plan
    from triton_kubernetes_amd.parallel.transport import AgentTransport, HostRef
    from triton_kubernetes_amd.rancher.fake import FakeRancher

    fake_docker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "fake_docker.py")
    bindir = tmp_path / "bin"
    bindir.mkdir()
    _stub(bindir, "docker", f'exec {sys.executable} {fake_docker} "$@"')
    _stub(bindir, "hostnamectl", "exit 0")
    root = tmp_path / "root"
    monkeypatch.setenv("PATH", f"{bindir}:{os.environ.get('PATH', '/usr/bin:/bin')}")
    monkeypatch.setenv("TK_HOST_ROOT", str(root))  # the fake docker keeps this host's containers

    def containers():
        path = root / "var/lib/docker/fake-containers.json"
        return json.loads(path.read_text()) if path.exists() else []

    subprocess.run(["docker", "run", "-d", "--name", "owners-nginx", "nginx:1.25"], check=True, capture_output=True)
    fake = FakeRancher().start()
    agent = NodeAgent(name="w-rke1", mode="exec", devices=[0], token="exec-token-123456", root=str(root))
    url = agent.serve()
    transport, ref = AgentTransport(token="exec-token-123456"), HostRef("agent+" + url)
    cfg = {"hostname": "gpu-rke1-1", "rancher_host_labels": {"worker": "true"}, "gpu_count": 1,
           "gpu_burnin": "quick", "k8s_distribution": "rke1"}
    try:
        first = transport.run_plan(ref, build_host_plan(cfg, fake.url, "regtokA123", "cafe0123", mi355x=True))
        assert first["ok"], first
        names = sorted(c["name"] for c in containers())
        assert any(c["image"] == versions.AGENT_IMAGE and not c["name"].startswith("k8s_") for c in containers())
        assert sum(n.startswith("k8s_") for n in names) == 4 and "kubelet" in names
        plan_b = build_host_plan(cfg, fake.url, "regtokB456", "cafe0123", mi355x=True)
        refused = transport.run_plan(ref, plan_b)
        assert not refused["ok"] and "another cluster" in json.dumps(refused), refused
        rep = transport.cleanup_host(ref)
        assert rep["ok"], rep
        assert [c["name"] for c in containers()] == ["owners-nginx"], containers()
        second = transport.run_plan(ref, plan_b)
        assert second["ok"], second
        agents = [c for c in containers() if c["image"] == versions.AGENT_IMAGE and not c["name"].startswith("k8s_")]
        assert len(agents) == 1 and "regtokB456" in agents[0]["args"]
        burn = [s for s in second["steps"] if s["name"] == "gpu_burnin"][0]
        assert burn["ok"], burn
    finally:
        agent.stop()
        fake.stop()
    print(json.dumps({"cleanup_ms": rep.get("ms"), "actions": rep["actions"]}))
