"""Cluster RCCL gate for nodes without agents: ``rccl-ready --cluster`` per node over the
host transport (``readiness/process_gate.py``), with the CPU stand-in of the tool."""

import os
import stat
import sys
import time

import pytest

from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.parallel.transport import HostRef, LocalTransport
from triton_kubernetes_amd.rancher.client import RancherClient
from triton_kubernetes_amd.rancher.fake import FakeRancher, tunnel_params
from triton_kubernetes_amd.readiness.process_gate import ProcessGate, gate_script
from triton_kubernetes_amd.readiness.waiter import ReadinessSpec, wait_ready

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "fake_rccl_ready.py")


@pytest.fixture
def tools(tmp_path):
    d = tmp_path / "bin"
    d.mkdir()
    exe = d / "rccl-ready"
    exe.write_text(f"#!/bin/sh\nexec {sys.executable} {FIXTURE} \"$@\"\n")
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)
    env = tmp_path / "rccl.env"
    env.write_text('NCCL_IB_HCA="=mlx5_0:1"\n')
    return str(d), str(env)


def _gate(tools, n=3, gpus=8, env=None, timeout=60.0):
    d, env_file = tools
    hosts = [HostRef("local") for _ in range(n)]
    return ProcessGate(LocalTransport(env=env), hosts, [gpus] * n, [1 << 20, 64 << 20], iters=5, timeout=timeout,
                       tools_dir=d, env_file=env_file)


def test_process_gate_one_communicator_over_every_node(tools):
    res = _gate(tools).run()
    assert res["ok"] and res["world"] == 24 and res["nodes"] == 3 and res["mode"] == "process"
    assert [r["rank_base"] for r in res["ranks"]] == [0, 8, 16]
    assert all(r["world"] == 24 and r["rc"] == 0 for r in res["ranks"])
    assert res["min_peak_busbw_gbps"] == 100.0
    # each node's /etc/rccl/rccl.env was sourced before the tool ran
    assert {r["env"] for r in res["ranks"]} == {"=mlx5_0:1"}


def test_process_gate_fails_fast_when_a_node_fails(tools):
    t0 = time.monotonic()
    with pytest.raises(TKError, match="exited 2"):
        _gate(tools, env={"FAKE_RCCL_FAIL_BASE": "8"}, timeout=60).run()
    assert time.monotonic() - t0 < 20  # not the deadline: the others were killed


def _alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    # a zombie has exited; /proc says so
    try:
        with open(f"/proc/{pid}/stat") as fh:
            return fh.read().split(")")[-1].split()[0] != "Z"
    except OSError:
        return False


class _SSHLike(LocalTransport):
    """Like ssh without a pty: the spawned process is a client whose death does not signal
    the 'remote' shell (a grandchild here); only the channel's stdin closing reaches it."""

    def spawn(self, host, script):
        import subprocess

        client = "import subprocess, sys; sys.exit(subprocess.run(['bash', '-c', sys.argv[1]]).returncode)"
        return subprocess.Popen([sys.executable, "-c", client, script], stdin=subprocess.PIPE,
                                stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=self._env())


def test_failed_gate_leaves_no_rank_process_behind(tools, tmp_path):
    """a node whose peer failed is blocked in communicator init; killing the gate
    (its ssh client) must take that node's rccl-ready down too, not leave it holding GPUs."""
    piddir = tmp_path / "pids"
    piddir.mkdir()
    d, env_file = tools
    gate = ProcessGate(_SSHLike(env={"FAKE_RCCL_FAIL_BASE": "16", "FAKE_RCCL_PIDDIR": str(piddir)}),
                       [HostRef("local")] * 3, [8] * 3, [1 << 20, 64 << 20], iters=5, timeout=60, tools_dir=d,
                       env_file=env_file)
    with pytest.raises(TKError, match="exited 2"):
        gate.run()
    pids = [int(p.name.split(".")[0]) for p in piddir.iterdir()]
    # the root (rank base 0) was running -- blocked waiting for its peers -- when the gate
    # failed; a peer killed before it got to record itself cannot outlive the gate either
    assert "0" in [p.read_text() for p in piddir.iterdir()]
    deadline = time.monotonic() + 10
    while any(_alive(p) for p in pids) and time.monotonic() < deadline:
        time.sleep(0.1)
    assert not [p for p in pids if _alive(p)]


def test_gate_tool_timeout_is_the_init_budget():
    s = gate_script("/x", 8, 0, 8, [1 << 20], 5, None, timeout_s=3600)
    assert "--timeout-s 300 " in s
    assert "--timeout-s 20 " in gate_script("/x", 8, 0, 8, [1 << 20], 5, None, timeout_s=20)


def test_process_gate_deadline_without_unique_id(tools):
    with pytest.raises(TKError, match="no unique id"):
        _gate(tools, n=2, env={"FAKE_RCCL_NO_UID": "1"}, timeout=1.5).run()


def test_gate_script_shape():
    s = gate_script("/opt/triton-kubernetes/bin", 16, 8, 8, [1 << 20, 256 << 20], 5, "ab" * 128)
    assert s.startswith("set -a; [ -r /etc/rccl/rccl.env ] && . /etc/rccl/rccl.env; set +a; ")
    # installed RCCL by default; the verified opt-in wrapper only when the node has it
    assert "t=/opt/triton-kubernetes/bin/rccl-ready; [ -x /opt/triton-kubernetes/bin/rccl-ready-slim ]" in s
    assert "--cluster --world 16 --rank-base 8 --ngpus 8 --max-mib 256 --iters 5" in s and "--uid abab" in s
    assert "--uid-out" in gate_script("/x", 8, 0, 8, [1 << 20], 5, None)


def test_waiter_runs_process_gate_for_ssh_nodes(tools):
    fake = FakeRancher(bootstrap_password="b00tstrap-only").start()
    try:
        client = RancherClient(fake.url)
        outs = client.bootstrap("n3w-passw0rd-123", fake.url, "b00tstrap-only", timeout=10)
        client = RancherClient(fake.url, outs["rancher_access_key"], outs["rancher_secret_key"])
        info = client.ensure_cluster("ssh-gpu")
        from triton_kubernetes_amd.cloud.http import HTTPClient

        for host, roles in (("cp", {"etcd": True, "controlplane": True}), ("g1", {"worker": True}),
                            ("g2", {"worker": True})):
            HTTPClient(base_url=fake.url).request("POST", "/v3/connect/register", data=b"{}", headers={
                "X-API-Tunnel-Token": info.registration_token,
                "X-API-Tunnel-Params": tunnel_params(host, roles, {}, {}),
                "X-Cattle-Agent-Kind": "system-agent"})  # an RKE2 cluster (the default)
        spec = ReadinessSpec(info.cluster_id, ["cp", "g1", "g2"], timeout=30, rccl_gate=True,
                             rccl_process_hosts=[HostRef("local"), HostRef("local")], rccl_process_ndev=[8, 8])
        rep = wait_ready(client, spec, host_transport=LocalTransport(), tools_dir=tools[0])
        assert rep.rccl["ok"] and rep.rccl["world"] == 16 and "rccl_gate" in rep.phases
        # no GPU nodes: the report says the gate was skipped, and why
        spec2 = ReadinessSpec(info.cluster_id, ["cp"], timeout=10, rccl_gate=False,
                              rccl_skip_reason="no MI355X nodes in the cluster")
        rep2 = wait_ready(client, spec2)
        assert rep2.rccl == {"ok": None, "skipped": "no MI355X nodes in the cluster"}
        assert "rccl_gate" not in rep2.phases
    finally:
        fake.stop()


def test_mixed_agent_and_process_nodes_share_one_gate(tools):
    """Agent nodes join the process gate through their API, with the same unique id."""
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.labels import synthetic_topology
    from triton_kubernetes_amd.parallel.transport import AgentTransport

    token = "mixed-gate-token-12345"
    agent = NodeAgent(name="a", mode="sim", devices=list(range(8)), token=token, root=str(tools[1]) + ".d",
                      topology_override=synthetic_topology(8))
    url = agent.serve()
    try:
        d, env_file = tools
        for hosts in ([HostRef("local"), HostRef("agent+" + url)], [HostRef("agent+" + url), HostRef("local")]):
            gate = ProcessGate(LocalTransport(env={"FAKE_RCCL_AGENT_RANKS": "8"}), hosts, [8, 8], [1 << 20, 64 << 20],
                               iters=5, timeout=60, tools_dir=d, env_file=env_file,
                               agent_transport=AgentTransport(token=token))
            res = gate.run()
            assert res["ok"] and res["mode"] == "mixed" and res["world"] == 16, res
            assert sorted((r["kind"], r["rank_base"]) for r in res["ranks"]) == \
                sorted([(("process" if h.scheme == "ssh" or h.address == "local" else "agent"), b)
                        for h, b in zip(hosts, (0, 8))])
        assert agent._gates == {}  # the agent's communicator was consumed, nothing pending
    finally:
        agent.stop()


def test_spec_from_state_routes_each_delivery_kind():
    """All-agent clusters keep the pipelined agent gate; SSH-only clusters get the process
    gate; mixed clusters get one process gate whose agent members join via their API."""
    import json as _json

    from triton_kubernetes_amd.backend import MemoryBackend
    from triton_kubernetes_amd.readiness.waiter import spec_from_state
    from triton_kubernetes_amd.state import State
    from triton_kubernetes_amd.terraform.catalog import MODULES_DIR
    from triton_kubernetes_amd.terraform.catalog import module_source as _src

    def module_source(name):
        return _src(MODULES_DIR, name, "")

    def state_with(hosts):
        st = State("m", {})
        st.set_manager({"source": module_source("bare-metal-rancher")})
        key = st.add_cluster("baremetal", "c", {"source": module_source("bare-metal-rancher-k8s"), "name": "c"})
        for i, h in enumerate(hosts):
            st.add_node(key, f"g-{i}", {"source": module_source("bare-metal-mi355x-rancher-k8s-host"),
                                        "hostname": f"g-{i}", "host": h, "gpu_count": 8, "ssh_user": "u"})
        return st, key

    be = MemoryBackend()
    be.write_tfstate("m", _json.dumps({"module_outputs": {
        "cluster-manager": {"rancher_url": "http://r", "rancher_access_key": "a", "rancher_secret_key": "s"},
        "cluster_baremetal_c": {"rancher_cluster_id": "c-1"}}}).encode())
    st, key = state_with(["agent+http://a:1", "agent+http://b:1"])
    _, spec = spec_from_state(st, be, key, rccl_gate=True)
    assert spec.rccl_gate and spec.rccl_hosts == ["http://a:1", "http://b:1"] and not spec.rccl_process_hosts
    st, key = state_with(["10.0.0.1", "10.0.0.2"])
    _, spec = spec_from_state(st, be, key, rccl_gate=True)
    assert spec.rccl_gate and not spec.rccl_hosts and [h.address for h in spec.rccl_process_hosts] == ["10.0.0.1",
                                                                                                      "10.0.0.2"]
    st, key = state_with(["agent+http://a:1", "10.0.0.2"])
    _, spec = spec_from_state(st, be, key, rccl_gate=True)
    assert spec.rccl_gate and not spec.rccl_hosts and not spec.rccl_skip_reason
    assert [h.address for h in spec.rccl_process_hosts] == ["agent+http://a:1", "10.0.0.2"]
    assert spec.rccl_process_ndev == [8, 8]
