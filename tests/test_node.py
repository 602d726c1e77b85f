"""Node layer: bootstrap plans (shell + agent renderers), GPU labels, KFD topology, node agent."""

import base64
import json
import os
import subprocess

import pytest

from triton_kubernetes_amd.node.agent import NodeAgent
from triton_kubernetes_amd.node.labels import agent_label_flags, labels_from_topology, product_name, synthetic_topology
from triton_kubernetes_amd.node.plan import BootstrapPlan, build_host_plan, parse_step_markers
from triton_kubernetes_amd.ops.topo import kfd_topology
from triton_kubernetes_amd.parallel.transport import HostRef, LocalTransport

WORKER = {"hostname": "gpu-1", "rancher_host_labels": {"worker": "true"}}
GPU_WORKER = dict(WORKER, gpu_count=8, gpu_burnin="quick", rccl_env={"NCCL_MIN_NCHANNELS": "32"})


def _bash_syntax_ok(script: str) -> None:
    proc = subprocess.run(["bash", "-n"], input=script, capture_output=True, text=True, check=False)
    assert proc.returncode == 0, proc.stderr


def test_plan_steps_and_order():
    # RKE2 (default): no container runtime or docker login (RKE2 brings containerd, registries
    # come from the cluster's rkeConfig); RKE1: the reference's Docker + rancher-agent steps
    plain = build_host_plan(WORKER, "https://r", "tok", "sum")
    assert plain.step_names() == ["firewall", "hostname", "agent"] and plain.distribution == "rke2"
    assert plain.gpu is None
    rke1 = build_host_plan(dict(WORKER, k8s_distribution="rke1"), "https://r", "tok", "sum")
    assert rke1.step_names() == ["firewall", "runtime", "hostname", "agent"]
    reg = dict(GPU_WORKER, rancher_registry="reg.io", rancher_registry_username="u", rancher_registry_password="p")
    gpu = build_host_plan(dict(reg, k8s_distribution="rke1"), "https://r", "tok", "sum", mi355x=True)
    # burn-in precedes labels so the agent's topology prefetch overlaps it; the link check
    # precedes the burn-in (idle GPUs, not beside the clearing of the burn-in's release)
    assert gpu.step_names() == ["firewall", "runtime", "hostname", "registry_login", "gpu_preflight",
                                "gpu_links", "gpu_burnin", "gpu_labels", "gpu_health", "rccl_env", "rccl_local", "agent"]
    gpu2 = build_host_plan(reg, "https://r", "tok", "sum", mi355x=True)
    assert gpu2.step_names() == ["firewall", "hostname", "gpu_preflight", "gpu_links", "gpu_burnin", "gpu_labels",
                                 "gpu_health", "rccl_env", "rccl_local", "agent"]
    # gpu_health = off: no RAS verdict step
    off = build_host_plan(dict(reg, gpu_health="off"), "https://r", "tok", "sum", mi355x=True)
    assert "gpu_health" not in off.step_names()
    assert gpu2.steps[-1].params == {"server": "https://r", "role": "worker", "distribution": "rke2"}
    with pytest.raises(ValueError):
        build_host_plan(dict(WORKER, k8s_distribution="k3s"), "https://r", "tok", "sum")
    assert gpu.gpu == {"product": "MI355X", "count": 8, "burnin": "quick", "physical": 8, "compute_partition": "spx",
                       "memory_partition": "nps1"}
    # the single-target RCCL copy is opt-in (a modified vendor binary)
    assert "rccl-ready-slim" not in gpu.render_shell()
    slim = build_host_plan(dict(GPU_WORKER, rccl_slim="on"), "https://r", "t", "s", mi355x=True)
    assert slim.step_names().index("rccl_slim") == slim.step_names().index("rccl_local") - 1
    _bash_syntax_ok(slim.render_shell())
    assert "rccl-ready-slim" in slim.render_shell() and "--expect-rccl" in slim.render_shell()
    off = build_host_plan(dict(GPU_WORKER, gpu_burnin="off", gpu_count=1), "https://r", "t", "s", mi355x=True)
    assert "gpu_burnin" not in off.step_names() and "rccl_local" not in off.step_names()


@pytest.mark.parametrize("mi355x", [False, True])
def test_rendered_shell_is_valid_bash(mi355x):
    plan = build_host_plan(dict(GPU_WORKER, hostname="x; rm -rf /"), "https://r", "t'ok", "sum", mi355x=mi355x)
    script = plan.render_shell()
    _bash_syntax_ok(script)
    assert "'x; rm -rf /'" in script  # quoted, never spliced raw
    if mi355x:
        assert "--label" in script and 'NCCL_MIN_NCHANNELS="32"' in script


def test_plan_json_roundtrip():
    plan = build_host_plan(GPU_WORKER, "https://r", "tok", "sum", mi355x=True)
    back = BootstrapPlan.from_json(json.loads(json.dumps(plan.to_json())))
    assert back == plan


def test_step_markers():
    out = "noise\n::tk-step firewall start 0\n::tk-step firewall ok 12\n::tk-step agent failed 7\n"
    assert parse_step_markers(out) == {"firewall": {"status": "ok", "ms": 12}, "agent": {"status": "failed", "ms": 7}}


def _fake_bin(d, name, body):
    p = d / name
    p.write_text("#!/bin/bash\n" + body + "\n")
    p.chmod(0o755)


@pytest.mark.parametrize("dist", ["rke2", "rke1"])
def test_local_transport_runs_plan_with_stub_tools(tmp_path, dist):
    """The rendered script runs end to end with stub sudo/docker/curl; markers + the join argv come back."""
    bindir = tmp_path / "bin"
    bindir.mkdir()
    log = tmp_path / "sudo.log"
    _fake_bin(bindir, "sudo", f'echo "$*" >> {log}; cat >/dev/null 2>&1 || true')
    _fake_bin(bindir, "docker", "exit 0")
    _fake_bin(bindir, "curl", f'echo "curl $*" >> {log}; while [ $# -gt 0 ]; do [ "$1" = -o ] && : > "$2"; shift; done')
    env = {"PATH": f"{bindir}:/usr/bin:/bin"}
    plan = build_host_plan(dict(WORKER, k8s_distribution=dist), "https://rancher.example", "regtok", "cafe",
                           mi355x=False)
    res = LocalTransport(env=env).run_plan(HostRef("local"), plan)
    assert res["ok"], res
    assert [s["name"] for s in res["steps"]] == plan.step_names()
    calls = log.read_text()
    assert "hostnamectl set-hostname gpu-1" in calls
    if dist == "rke1":
        assert "--server https://rancher.example --token regtok --ca-checksum cafe --worker" in calls
    else:
        assert "https://rancher.example/system-agent-install.sh" in calls
        assert ("--server https://rancher.example --label cattle.io/os=linux "
                "--token regtok --ca-checksum cafe --node-name gpu-1 --worker") in calls


def test_a_failing_command_mid_step_fails_the_step(tmp_path):
    """errexit holds inside every step body: a download that fails in the middle of the
    join step fails it (the step is not judged by its last command)."""
    bindir = tmp_path / "bin"
    bindir.mkdir()
    log = tmp_path / "calls.log"
    _fake_bin(bindir, "sudo", f'echo "$*" >> {log}')
    _fake_bin(bindir, "curl", "exit 6")  # could not resolve host
    plan = build_host_plan(WORKER, "https://rancher.example", "t", "s")
    res = LocalTransport(env={"PATH": f"{bindir}:/usr/bin:/bin"}).run_plan(HostRef("local"), plan)
    assert not res["ok"] and "agent" in (res.get("error") or "")
    assert "--server" not in log.read_text()  # the installer never ran


def test_local_transport_reports_failed_step(tmp_path):
    bindir = tmp_path / "bin"
    bindir.mkdir()
    _fake_bin(bindir, "sudo", 'case "$*" in hostnamectl*) exit 3;; esac; cat >/dev/null')
    _fake_bin(bindir, "docker", "exit 0")
    plan = build_host_plan(WORKER, "https://r", "t", "s")
    res = LocalTransport(env={"PATH": f"{bindir}:/usr/bin:/bin"}).run_plan(HostRef("local"), plan)
    assert not res["ok"]
    assert "hostname" in (res.get("error") or "")


def test_labels_from_synthetic_topology():
    labels = labels_from_topology(synthetic_topology(8))
    assert labels["amd.com/gpu.count"] == "8"
    assert labels["amd.com/gpu.product-name"] == "MI355X"
    assert labels["amd.com/gpu.family"] == "AI"
    assert labels["amd.com/gpu.vram"] == "288G"
    assert labels["amd.com/gpu.compute-partition"] == "spx"
    assert labels["amd.com/xgmi.fully-connected"] == "true"
    assert labels["amd.com/xgmi.links-per-gpu"] == "7"
    assert labels["amd.com/xgmi.hive-id"] == "0xabc123"
    assert labels_from_topology({"gpus": []}) == {"amd.com/gpu.present": "false", "amd.com/rdma.count": "0"}
    flags = agent_label_flags({"b": "2", "a": "1"})
    assert flags == ["--label", "a=1", "--label", "b=2"]


def test_product_name_device_id_wins():
    # amd_smi's market name for an MI355X OAM part does not carry the X
    assert product_name("AMD Instinct MI355 OAM", "0x75a3") == "MI355X"
    assert product_name("AMD Instinct MI300X", "0xdead") == "MI300X"
    assert product_name("weird name!", "") == "weird-name"


def test_partial_xgmi_mesh_not_fully_connected():
    topo = synthetic_topology(4)
    topo["gpus"][0]["links"] = [lk for lk in topo["gpus"][0]["links"] if lk["peer"] != 3]
    labels = labels_from_topology(topo)
    assert labels["amd.com/xgmi.fully-connected"] == "false"
    assert labels["amd.com/xgmi.links-per-gpu"] == "2"


def _kfd_node(root, idx, props, name="", links=()):
    d = root / str(idx)
    (d / "io_links").mkdir(parents=True)
    (d / "properties").write_text("".join(f"{k} {v}\n" for k, v in props.items()))
    (d / "name").write_text(name + "\n")
    for i, (to, typ) in enumerate(links):
        ld = d / "io_links" / str(i)
        ld.mkdir()
        (ld / "properties").write_text(f"node_from {idx}\nnode_to {to}\ntype {typ}\nweight 15\n")


def test_kfd_topology_fixture(tmp_path):
    """A CPU node + two gfx950 GPU nodes linked by xGMI (type 11), as KFD sysfs lays it out."""
    _kfd_node(tmp_path, 0, {"simd_count": 0, "cpu_cores_count": 96})
    gpu = {"simd_count": 1024, "simd_per_cu": 4, "gfx_target_version": 90500, "device_id": 0x75a3,
           "hive_id": 0x1234, "domain": 0, "location_id": 0x0500}
    _kfd_node(tmp_path, 1, gpu, "", [(0, 2), (2, 11)])
    _kfd_node(tmp_path, 2, dict(gpu, location_id=0x0600), "", [(0, 2), (1, 11)])
    doc = kfd_topology(str(tmp_path))
    assert doc["source"] == "kfd" and len(doc["gpus"]) == 2
    g0 = doc["gpus"][0]
    assert g0["compute_units"] == 256 and g0["target_graphics_version"] == "gfx950"
    assert g0["bdf"] == "0000:05:00.0"
    assert g0["links"] == [{"peer": 1, "type": "XGMI", "hops": 1, "p2p": True}]
    labels = labels_from_topology(doc)
    assert labels["amd.com/gpu.product-name"] == "MI355X"
    assert labels["amd.com/xgmi.fully-connected"] == "true"
    assert labels["amd.com/xgmi.hive-id"] == "0x1234"


def test_agent_sim_plan_without_rancher_reaches_agent_step(tmp_path):
    """GPU steps run against synthetic GPUs; files land under the agent root."""
    calls = []

    def burn(dev, level):
        calls.append((dev, level))
        return {"ok": True, "device": dev}

    agent = NodeAgent("n1", "sim", devices=list(range(8)), root=str(tmp_path), token="t",
                      topology_override=synthetic_topology(8), burnin_override=burn)
    plan = build_host_plan(GPU_WORKER, "http://127.0.0.1:9", "tok", "sum", mi355x=True)
    plan.steps = [s for s in plan.steps if s.action != "agent"]
    res = agent.run_plan(plan)
    assert res["ok"], res
    assert sorted(calls) == [(d, "quick") for d in range(8)]
    assert res["capacity"] == {"amd.com/gpu": 8}
    assert res["labels"]["amd.com/gpu.count"] == "8"
    assert (tmp_path / "etc/triton-kubernetes/gpu-labels").read_text().startswith("amd.com/")
    assert 'NCCL_MIN_NCHANNELS="32"' in (tmp_path / "etc/rccl/rccl.env").read_text()


def test_agent_burnin_failure_stops_plan(tmp_path):
    agent = NodeAgent("n1", "sim", devices=[0, 1], root=str(tmp_path), token="t",
                      topology_override=synthetic_topology(2),
                      burnin_override=lambda d, lvl: {"ok": d != 1, "failures": ["hbm"]})
    res = agent.run_plan(build_host_plan(dict(GPU_WORKER, gpu_count=2), "http://127.0.0.1:9", "t", "s", mi355x=True))
    assert not res["ok"] and res["error"].startswith("gpu_burnin")
    assert "gpu_labels" not in [s["name"] for s in res["steps"]]


def test_agent_preflight_counts_gpus(tmp_path):
    agent = NodeAgent("n1", "sim", devices=[0], root=str(tmp_path), token="t",
                      topology_override=synthetic_topology(1))
    res = agent.run_plan(build_host_plan(GPU_WORKER, "http://127.0.0.1:9", "t", "s", mi355x=True))
    assert not res["ok"] and "expected 8 GPUs, found 1" in res["error"]


def test_agent_http_requires_token(tmp_path):
    from triton_kubernetes_amd.cloud.http import HTTPClient, HTTPError

    agent = NodeAgent("n1", "sim", root=str(tmp_path), token="sekrit")
    url = agent.serve()
    try:
        with pytest.raises(Exception) as exc:
            HTTPClient(base_url=url).request("GET", "/v1/info")
        assert "401" in str(exc.value) or isinstance(exc.value, HTTPError)
        info = HTTPClient(base_url=url).request("GET", "/v1/info", headers={"X-TK-Agent-Token": "sekrit"}).json()
        assert info["name"] == "n1"
    finally:
        agent.stop()


def test_agent_rejects_bad_mode():
    with pytest.raises(ValueError):
        NodeAgent("n", "shell")
    assert NodeAgent("n").token  # a token is always generated


def test_exec_mode_validates_hostname(tmp_path):
    agent = NodeAgent("n1", "exec", root=str(tmp_path), token="t")
    plan = build_host_plan(dict(WORKER, hostname="bad host;reboot"), "http://127.0.0.1:9", "t", "s")
    plan.steps = [s for s in plan.steps if s.action == "hostname"]
    res = agent.run_plan(plan)
    assert not res["ok"] and "invalid hostname" in res["error"]
    assert os.path.exists(tmp_path) and not agent.history[-1]["ok"]


def test_agent_janitor_frees_burnin_arena_when_idle(tmp_path, monkeypatch):
    """The resident burn-in arena is released after an idle period, re-armed by the next
    plan, and released (cache off) at stop."""
    import time

    from triton_kubernetes_amd.ops import probe

    events = []
    monkeypatch.setattr(probe, "release_scratch", lambda: events.append("release") or 0)
    monkeypatch.setattr(probe, "set_scratch_cache", lambda on: events.append(f"cache={on}"))
    agent = NodeAgent("n1", "sim", devices=[0], root=str(tmp_path), token="t",
                      topology_override=synthetic_topology(1), burnin_override=lambda d, lvl: {"ok": True})
    agent._start_janitor(0.1)
    plan = build_host_plan(dict(GPU_WORKER, gpu_count=1), "http://127.0.0.1:9", "t", "s", mi355x=True)
    plan.steps = [s for s in plan.steps if s.action != "agent"]
    assert agent.run_plan(plan)["ok"]
    assert events == []  # still within the idle window
    deadline = time.time() + 5
    while events.count("release") < 1 and time.time() < deadline:
        time.sleep(0.02)
    assert events == ["release"]
    assert agent.run_plan(plan)["ok"]  # re-arms: released again after the next idle period
    while events.count("release") < 2 and time.time() < deadline:
        time.sleep(0.02)
    assert events == ["release", "release"]
    agent.stop()
    assert events[-2:] == ["release", "cache=False"]


def test_presize_fd_table_and_procstat():
    """Grows the fd table once (in a child, so the test process is untouched) and reports
    per-process counters."""
    import sys

    code = (
        "import os, resource\n"
        "from triton_kubernetes_amd.utils import procstat\n"
        "before = procstat.snapshot()\n"
        "n = procstat.presize_fd_table(4096)\n"
        "fd = os.open('/dev/null', os.O_RDONLY)\n"
        "after = procstat.snapshot()\n"
        "d = procstat.delta(before, after)\n"
        "print(n, fd, resource.getrlimit(resource.RLIMIT_NOFILE)[0] >= min(4096, resource.getrlimit(resource.RLIMIT_NOFILE)[1]),"
        " d['threads'] >= 1, d['cpu_s'] >= 0, 'fds' in after)\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=root, check=True).stdout.split()
    n, fd = int(out[0]), int(out[1])
    assert 0 < n <= 4096
    assert fd < 64  # the lowest free descriptor is still handed out first
    assert out[2:] == ["True", "True", "True", "True"]


def test_step_markers_name_steps_whose_bodies_assign_variables(tmp_path):
    """Regression (found running the rendered bootstrap on an MI355X box): a step body that
    assigns a variable named like a _tk_step local (bash scoping is dynamic) must not rename
    the step in its ::tk-step markers."""
    from triton_kubernetes_amd.node.plan import Step

    plan = build_host_plan(WORKER, "https://r", "t", "s", mi355x=False)
    plan.steps = [Step("clobber", "firewall", "n=1; t0=2; rc=3; name=4; true"), Step("after", "hostname", "true")]
    proc = subprocess.run(["bash", "-s"], input=plan.render_shell(), capture_output=True, text=True, check=False)
    assert proc.returncode == 0, proc.stderr
    steps = parse_step_markers(proc.stdout)
    assert list(steps) == ["clobber", "after"] and all(v["status"] == "ok" for v in steps.values())


def test_burnin_labels_formatting():
    from triton_kubernetes_amd.node.labels import burnin_labels

    gib = 1 << 30
    res = {0: {"ok": True, "memtest": {"bytes": 280 * gib, "hbm_bytes": 288 * gib}},
           1: {"ok": True, "memtest": {"bytes": 276 * gib, "hbm_bytes": 288 * gib}}}
    assert burnin_labels("full", res) == {"amd.com/gpu.burnin": "passed", "amd.com/gpu.burnin-level": "full",
                                          "amd.com/gpu.burnin-hbm-tested-gib": "276",
                                          "amd.com/gpu.burnin-hbm-tested-pct": "95.8"}
    res[1]["ok"] = False
    assert burnin_labels("full", res)["amd.com/gpu.burnin"] == "failed"
    assert burnin_labels("quick", {})["amd.com/gpu.burnin"] == "failed"


def test_shell_plan_carries_burnin_labels():
    from triton_kubernetes_amd.node.plan import BURNIN_LABEL_FILE, build_host_plan

    cfg = {"hostname": "g", "rancher_host_labels": {"worker": "true"}, "gpu_count": 8, "gpu_burnin": "full"}
    script = build_host_plan(cfg, "https://r", "tok", "ca", mi355x=True).render_shell()
    assert ("gpu-burnin --all --level full --compute-partition spx --memory-partition nps1 "
            "--labels /tmp/tk-burnin-labels") in script
    assert f"sudo rm -f {BURNIN_LABEL_FILE}" in script
    assert f"[ -r {BURNIN_LABEL_FILE} ] && echo {BURNIN_LABEL_FILE}" in script


def test_link_labels_verdicts():
    from triton_kubernetes_amd.node.labels import link_labels

    pairs = {f"{i}-{j}": 60.0 for i in range(4) for j in range(4) if i != j}
    ok = link_labels({"pairs": pairs, "peer_access": {p: True for p in pairs}})
    assert ok["status"] == "passed" and ok["labels"]["amd.com/xgmi.p2p-min-gbps"] == "60"
    bad = dict(pairs, **{"2-3": 20.0})
    v = link_labels({"pairs": bad, "peer_access": {p: True for p in bad}})
    assert v["status"] == "degraded" and v["degraded"] == ["2-3"] and v["labels"]["amd.com/xgmi.link-check"] == "degraded"
    err = link_labels({"pairs": pairs, "peer_access": dict({p: True for p in pairs}, **{"0-1": False})})
    assert err["status"] == "error"
    assert link_labels({"pairs": {}, "errors": []})["status"] == "skipped"
    # full speed, wrong data: degraded whatever the bandwidth says
    bad_data = link_labels({"pairs": pairs, "peer_access": {p: True for p in pairs}, "data_errors": {"1-0": 3}},
                           min_gbps=0.0)
    assert bad_data["status"] == "degraded" and bad_data["degraded"] == ["1-0"] and bad_data["corrupt"] == ["1-0"]


def test_link_check_absolute_floor_fails_a_uniformly_slow_fabric():
    """relative-to-median alone passes a fabric whose every link is slow; the
    absolute floor (default 38 GB/s: half of one xGMI link's ~76.8 GB/s one way) fails it."""
    from triton_kubernetes_amd.node.labels import DEFAULT_MIN_LINK_GBPS, link_labels
    from triton_kubernetes_amd.ops import probe

    assert DEFAULT_MIN_LINK_GBPS == probe.DEFAULT_MIN_LINK_GBPS == probe.XGMI_LINK_ONE_WAY_GBPS / 2 - 0.4
    n = 8
    every = [f"{i}-{j}" for i in range(n) for j in range(n) if i != j]
    acc = {p: True for p in every}
    slow = link_labels({"pairs": {p: 25.0 for p in every}, "peer_access": acc, "method": "kernel-read"})
    assert slow["status"] == "degraded" and slow["below_floor"] == sorted(every) and len(slow["degraded"]) == 56
    assert slow["labels"]["amd.com/xgmi.p2p-method"] == "kernel-read"
    # the same matrix with the floor off (0) passes: only the relative rule is left
    assert link_labels({"pairs": {p: 25.0 for p in every}, "peer_access": acc}, min_gbps=0.0)["status"] == "passed"
    # one bad link among healthy ones: relative rule
    one = {p: 70.0 for p in every}
    one["3-5"] = 30.0
    v = link_labels({"pairs": one, "peer_access": acc})
    assert v["status"] == "degraded" and v["degraded"] == ["3-5"] and v["below_floor"] == ["3-5"]
    one["3-5"] = 40.0  # above the floor, but 0.57 of the median: passes at 0.5, fails at 0.6
    assert link_labels({"pairs": one, "peer_access": acc})["status"] == "passed"
    assert link_labels({"pairs": one, "peer_access": acc}, min_frac=0.6)["degraded"] == ["3-5"]
    # a missing peer (no peer access, the kernel read could not run): error
    missing = {p: 70.0 for p in every if p != "6-7"}
    e = link_labels({"pairs": missing, "peer_access": dict(acc, **{"6-7": False}),
                     "errors": ["6->7: peer read failed"]})
    assert e["status"] == "error" and "6->7: peer read failed" in e["errors"]


def test_multi_gpu_plan_checks_links():
    from triton_kubernetes_amd.node.plan import build_host_plan

    cfg = {"hostname": "g", "rancher_host_labels": {"worker": "true"}, "gpu_count": 8, "gpu_burnin": "quick",
           "gpu_link_min_frac": 0.6}
    plan = build_host_plan(cfg, "https://r", "tok", "ca", mi355x=True)
    names = plan.step_names()
    assert names.index("gpu_links") < names.index("gpu_burnin") < names.index("gpu_labels")
    assert "gpu-burnin --p2p --min-link-frac 0.6 --min-link-gbps 38.0" in plan.render_shell()
    step = next(st for st in plan.steps if st.name == "gpu_links")
    assert step.params == {"min_frac": 0.6, "min_gbps": 38.0, "method": "kernel-read"}
    floor = build_host_plan(dict(cfg, gpu_link_min_gbps=50), "https://r", "tok", "ca", mi355x=True)
    assert "--min-link-gbps 50.0" in floor.render_shell()
    one = build_host_plan(dict(cfg, gpu_count=1), "https://r", "tok", "ca", mi355x=True)
    assert "gpu_links" not in one.step_names()


def test_one_node_cluster_gate_shares_the_rccl_local_sweep():
    """A gate communicator spanning exactly the node's GPUs (a one-node cluster) is swept by
    the plan's rccl_local step instead of a second init, and the gate answers from it."""
    import tempfile

    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.labels import synthetic_topology
    from triton_kubernetes_amd.node.plan import BootstrapPlan, Step

    agent = NodeAgent(name="n", mode="sim", devices=list(range(8)), token="t" * 24, root=tempfile.mkdtemp(),
                      topology_override=synthetic_topology(8))
    plan = BootstrapPlan("n", "worker", "http://r", "tok", "ca", steps=[Step("rccl_local", "rccl_local", "true")])
    try:
        # no pending gate: the synthetic node simulates its local check
        assert agent.run_plan(plan)["steps"][0]["detail"] == {"simulated": True}
        gate_sizes = [1 << 20, 64 << 20]
        prep = agent.rccl_prepare(None, world=8, rank_base=0, ndev=8, max_bytes=64 << 20, sizes=gate_sizes)
        uid = base64.b64decode(prep["uid"])
        detail = agent.run_plan(plan)["steps"][0]["detail"]
        assert detail["shared_with"] == "cluster_gate"
        assert detail["sizes"] == sorted({1 << 20, 16 << 20, 64 << 20, 256 << 20})
        assert agent._gates == {}  # taken by the step
        res = agent.rccl_gate(0, 8, uid, gate_sizes, ndev=8)
        assert res["shared_with"] == "rccl_local" and res["pipelined"] and res["sizes"] == gate_sizes
        assert res["ranks"] == list(range(8)) and res["ok"]
        # a gate over more than this node (another node's ranks) is never taken by the step
        agent.rccl_prepare(None, world=16, rank_base=0, ndev=8, sizes=gate_sizes)
        assert agent.run_plan(plan)["steps"][0]["detail"] == {"simulated": True}
        assert len(agent._gates) == 1
        # sizes the local sweep did not cover: a fresh communicator measures them
        prep = agent.rccl_prepare(None, world=8, rank_base=0, ndev=8, sizes=[1 << 20])
        agent._gates = {k: v for k, v in agent._gates.items() if k == base64.b64decode(prep["uid"])}
        agent.run_plan(plan)
        res = agent.rccl_gate(0, 8, base64.b64decode(prep["uid"]), [3 << 20], ndev=8)
        assert "shared_with" not in res and res["sizes"] == [3 << 20]
    finally:
        agent.stop()


def test_gpu_links_cli_verdict(monkeypatch, capsys):
    """``triton-kubernetes gpu links``: the pair matrix against the node median; a slow
    link fails (exit 1) with the same labels the agent and the host script write."""
    from triton_kubernetes_amd.ops import cli, probe

    monkeypatch.setattr(probe, "device_count", lambda: 3)

    def matrix(devs, nbytes=64 << 20, iters=3, method="kernel-read"):
        pairs = {f"{i}-{j}": 100.0 for i in devs for j in devs if i != j}
        pairs["2-0"] = slow
        return {"pairs": pairs, "peer_access": {k: True for k in pairs}, "errors": [], "bytes": nbytes,
                "method": method}

    monkeypatch.setattr(probe, "link_matrix", matrix)
    slow = 90.0
    assert cli.main(["links"]) == 0
    doc = json.loads(capsys.readouterr().out)
    assert doc["status"] == "passed" and doc["labels"]["amd.com/xgmi.link-check"] == "passed"
    assert len(doc["pairs"]) == 6
    slow = 20.0
    assert cli.main(["links", "--min-frac", "0.5"]) == 1
    doc = json.loads(capsys.readouterr().out)
    assert doc["status"] == "degraded" and doc["degraded"]
    # every link at 30 GB/s: the median rule passes, the absolute floor does not
    slow = 30.0
    monkeypatch.setattr(probe, "link_matrix", lambda devs, nbytes=0, iters=3, method="kernel-read": {
        "pairs": {f"{i}-{j}": 30.0 for i in devs for j in devs if i != j}, "peer_access": {}, "errors": [],
        "method": method})
    assert cli.main(["links"]) == 1
    assert json.loads(capsys.readouterr().out)["status"] == "degraded"
    assert cli.main(["links", "--min-gbps", "20"]) == 0


def test_agent_applies_the_node_rccl_env_to_its_own_gate(tmp_path, monkeypatch):
    """The agent's cluster gate runs RCCL in the agent process, and RCCL reads its settings
    once per process: the node's /etc/rccl/rccl.env goes into the agent's environment before
    its first RCCL call; the rccl_env step reports configured settings that differ (they take
    effect at the next start); the process's own settings win."""
    import os

    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.plan import Step
    from triton_kubernetes_amd.parallel.rccl_env import render_env_file

    env = {k: v for k, v in os.environ.items() if not k.startswith(("NCCL_", "RCCL_", "HSA_"))}
    env["NCCL_DEBUG"] = "INFO"  # set by the unit / operator: kept
    monkeypatch.setattr(os, "environ", env)
    agent = NodeAgent(name="n", mode="sim", devices=[0, 1], root=str(tmp_path))
    try:
        # first boot, no file: RCCL detects the RDMA ports itself, nothing is set
        assert agent.apply_node_rccl_env() == {} and "NCCL_IB_HCA" not in env

        # the bring-up's rccl_env step: the file gets the discovered and the configured values;
        # the configured ones that differ from this process's environment are reported, not
        # changed under the running agent (RCCL threads read the environment)
        topo = {"gpus": [], "nics": [{"name": "mlx5_0", "port": 1, "link_layer": "Ethernet", "roce_v2_gid_index": 3}]}
        step = Step("rccl_env", "rccl_env", "", {"env": {"NCCL_SOCKET_IFNAME": "=bond0", "NCCL_DEBUG": "WARN",
                                                          "HSA_FORCE_FINE_GRAIN_PCIE": "1"}})
        out = agent._run_step(None, step, {"labels": {}, "capacity": {}, "taints": [], "topology": topo})
        assert out["agent_env_differs"] == ["NCCL_DEBUG", "NCCL_SOCKET_IFNAME"]
        assert "NCCL_SOCKET_IFNAME" not in env and env["NCCL_DEBUG"] == "INFO"
        assert "NCCL_IB_HCA" not in env and 'NCCL_IB_HCA="=mlx5_0:1"' in (tmp_path / "etc/rccl/rccl.env").read_text()

        # a later start reads the file (HIP's HSA_* settings too: HIP reads them once, at its
        # initialisation); the unit's own values still win
        (tmp_path / "etc/rccl/rccl.env").write_text(render_env_file({"NCCL_SOCKET_IFNAME": "=bond1", "NCCL_DEBUG": "TRACE",
                                                                     "HSA_NO_SCRATCH_RECLAIM": "1"}))
        again = agent.apply_node_rccl_env()
        assert again == {"NCCL_SOCKET_IFNAME": "=bond1", "HSA_NO_SCRATCH_RECLAIM": "1"} and env["NCCL_DEBUG"] == "INFO"
    finally:
        agent.stop()


def test_sequential_plans_run_the_burn_in_after_the_rccl_check():
    """A shell runs one step after another: the burn-in goes after the node's RCCL check (its
    release is cleared by the driver for seconds after it); an agent keeps the burn-in first
    and overlaps it with the gate's communicator start."""
    from triton_kubernetes_amd.node.plan import build_host_plan
    from triton_kubernetes_amd.terraform import catalog

    cfg = {"hostname": "g", "rancher_host_labels": {"worker": "true"}, "gpu_count": 8}
    agent = build_host_plan(cfg, "https://r", "tok", "ca", mi355x=True).step_names()
    shell = build_host_plan(cfg, "https://r", "tok", "ca", mi355x=True, sequential=True).step_names()
    assert agent.index("gpu_burnin") < agent.index("rccl_local")
    assert shell.index("gpu_links") < shell.index("rccl_local") < shell.index("gpu_burnin") < shell.index("agent")
    assert sorted(agent) == sorted(shell)
    one = dict(cfg, gpu_count=1)  # no RCCL check on one GPU: the order stays
    assert build_host_plan(one, "https://r", "tok", "ca", mi355x=True, sequential=True).step_names() == \
        build_host_plan(one, "https://r", "tok", "ca", mi355x=True).step_names()
    script = open(os.path.join(catalog.MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host", "files",
                               "install_mi355x_node.sh.tftpl")).read()
    assert script.index("gpu-burnin --p2p") < script.index("$RCCL_READY --ngpus") < script.index("gpu-burnin --all")


# a reader that stops early (grep -q, head) ends its writer with SIGPIPE, and under pipefail
# that fails the pipeline even when the match was found: "amdgpu not loaded" on a node
# whose lsmod output outgrew one pipe write
_EARLY_READER = r"\|\s*(grep\s+-[A-Za-z]*q|head\b)"


def test_rendered_shell_has_no_early_exit_readers():
    import re

    from triton_kubernetes_amd.terraform import generate

    reg = dict(GPU_WORKER, rancher_registry="reg.io", rancher_registry_username="u", rancher_registry_password="p",
               rccl_slim="on")
    scripts = {"plan": build_host_plan(reg, "https://r", "t", "s", mi355x=True, sequential=True).render_shell(),
               "plan-rke1": build_host_plan(dict(reg, k8s_distribution="rke1"), "https://r", "t", "s",
                                            mi355x=True).render_shell()}
    for mod in generate.modules():
        for name, text in generate.rendered_files(mod).items():
            if name.endswith((".sh", ".tftpl")):
                scripts[f"{mod}/{name}"] = text
    bad = {k: m.group(0) for k, s in scripts.items() for m in [re.search(_EARLY_READER, s)] if m}
    assert not bad, bad


def test_agent_stop_before_a_quick_exit_skips_the_rccl_drain(monkeypatch, tmp_path):
    """``main`` leaves with ``_exit`` right after ``stop()``: the communicators' teardown is not
    waited for then (``drain_rccl=False``); a plain ``stop()`` still drains."""
    from triton_kubernetes_amd.ops import rccl

    drained = []
    monkeypatch.setattr(rccl, "drain", lambda *a, **k: drained.append(1))
    for drain, want in ((False, []), (True, [1])):
        drained.clear()
        agent = NodeAgent("n1", "sim", devices=[0], root=str(tmp_path), token="t",
                          topology_override=synthetic_topology(1), burnin_override=lambda d, lvl: {"ok": True})
        agent._used_rccl = True
        agent.stop(drain_rccl=drain)
        assert drained == want and "rccl_drain" in agent.stop_ms
