"""The cluster RCCL gate end to end on the CPU: node agents + ``ClusterGate`` over the
libtk_rccl C ABI, served by the ABI stub (``ops/csrc/tk_rccl_stub.cpp``).

On a one-GPU pool the multi-GPU gate paths -- one agent driving 8 ranks, 8 agents forming
a 64-rank communicator, a member failing mid-init -- never run on hardware, so the first
8-GPU node would be their first execution.  The stub keeps RCCL's semantics the callers
depend on (a communicator exists once every rank joined under one unique id; the sweep is
a collective; a waiting rank only leaves by its timeout or a cancel) and refuses what RCCL
refuses (a rank claimed twice, one unique id with two world sizes, a GPU twice in one
process).  Every library call is logged, so the tests check what the agents asked for.
The grouped-init sequence inside the real library is checked separately
(``tests/test_rccl_group.py``).
"""

import json
import os
import tempfile
import time

import pytest

from triton_kubernetes_amd.node.agent import NodeAgent
from triton_kubernetes_amd.node.labels import synthetic_topology
from triton_kubernetes_amd.ops import native, rccl
from triton_kubernetes_amd.parallel.transport import AgentTransport
from triton_kubernetes_amd.readiness.gate import ClusterGate, members_from

TOKEN = "gate-stub-token-0123"
SIZES = [1 << 20, 16 << 20]


@pytest.fixture
def stub(tmp_path, monkeypatch):
    from triton_kubernetes_amd.ops.build import build

    build(only=["libtk_rccl_stub.so"])
    monkeypatch.setenv("TK_RCCL_LIB", os.path.join(native.LIB_DIR, "libtk_rccl_stub.so"))
    monkeypatch.setenv("TK_RCCL_STUB_DIR", str(tmp_path / "rendezvous"))
    monkeypatch.setenv("TK_RCCL_STUB_LOG", str(tmp_path / "calls.jsonl"))
    monkeypatch.setattr(native, "_cache", {})  # load the stub, whatever this process loaded before
    return tmp_path


def _calls(tmp_path):
    path = tmp_path / "calls.jsonl"
    return [json.loads(ln) for ln in path.read_text().splitlines()] if path.exists() else []


def _agents(n, ndev=8):
    out = []
    for i in range(n):
        a = NodeAgent(name=f"gpu-{i}", mode="sim", devices=list(range(ndev)), token=TOKEN, root=tempfile.mkdtemp(),
                      topology_override=synthetic_topology(ndev), burnin_override=lambda d, lvl: {"ok": True},
                      gate_backend="rccl")
        out.append((a, a.serve()))
    return out


def _stop(agents):
    for a, _ in agents:
        a.stop()


def _eventually(check, timeout_s=10.0):
    """check() until it holds: the members release their ranks on their own threads, and a
    loaded machine (the suite under -n 8) takes longer than a fixed sleep."""
    deadline = time.monotonic() + timeout_s
    while not check() and time.monotonic() < deadline:
        time.sleep(0.05)
    return check()


def _left(tmp_path):
    d = tmp_path / "rendezvous"
    return sorted(os.listdir(d)) if d.exists() else []


def test_one_agent_drives_eight_ranks(stub):
    agents = _agents(1)
    try:
        gate = ClusterGate(AgentTransport(token=TOKEN), members_from([u for _, u in agents], [8]), SIZES,
                           timeout_s=30).prepare_async()
        res = gate.run()
        assert res["ok"] and res["pipelined"] and res["world"] == 8, res
        assert res["ranks"][0]["ranks"] == list(range(8))
        begins = [c for c in _calls(stub) if c["op"] == "begin"]
        assert [(c["world"], c["rank_base"], c["devices"]) for c in begins] == [(8, 0, list(range(8)))]
        assert [c["rc"] for c in _calls(stub) if c["op"] == "sweep"] == [0]
        assert _left(stub) == [] and rccl.pending_gates() == 0
    finally:
        _stop(agents)


def test_eight_agents_form_one_64_rank_communicator(stub):
    agents = _agents(8)
    try:
        members = members_from([u for _, u in agents], [8] * 8)
        t0 = time.monotonic()
        gate = ClusterGate(AgentTransport(token=TOKEN), members, SIZES, timeout_s=60).prepare_async()
        res = gate.run()
        assert res["ok"] and res["pipelined"] and res["world"] == 64 and res["nodes"] == 8, res
        assert sorted(r for m in res["ranks"] for r in m["ranks"]) == list(range(64))
        begins = [c for c in _calls(stub) if c["op"] == "begin"]
        assert sorted(c["rank_base"] for c in begins) == list(range(0, 64, 8))
        assert {c["uid"] for c in begins} == {begins[0]["uid"]} and {c["world"] for c in begins} == {64}
        assert all(c["devices"] == list(range(8)) for c in begins)  # every node its own GPUs 0..7
        assert [c["rc"] for c in _calls(stub) if c["op"] == "sweep"] == [0] * 8
        assert _left(stub) == [] and time.monotonic() - t0 < 30
        for a, _ in agents:
            assert not a._gates and not a._sweeping
    finally:
        _stop(agents)


def test_member_lost_after_prepare_fails_fast_and_releases_everyone(stub):
    """A node that prepared its ranks dies before the gate runs: the other 7 would wait for
    its ranks until their timeout; the gate cancels them instead and names the node."""
    agents = _agents(8)
    lost = agents[3]
    try:
        gate = ClusterGate(AgentTransport(token=TOKEN), members_from([u for _, u in agents], [8] * 8), SIZES,
                           timeout_s=120).prepare_async()
        gate._join()
        assert gate.prepared
        lost[0].stop()  # aborts its pending communicator: its 8 ranks are gone
        t0 = time.monotonic()
        res = gate.run()
        took = time.monotonic() - t0
        assert not res["ok"] and took < 20, (took, res)
        assert any(lost[1] in e for e in res["errors"]), res["errors"]
        assert _eventually(lambda: len([c for c in _calls(stub) if c["op"] == "cancel"]) == 7), _calls(stub)
        assert all(c["rc"] == -4 for c in _calls(stub) if c["op"] == "sweep")
        assert _eventually(lambda: not [f for d in _left(stub) for f in os.listdir(stub / "rendezvous" / d)
                                        if f.startswith("rank-")])
        assert _eventually(lambda: all(not a._gates and not a._sweeping for a, _ in agents))
    finally:
        _stop([a for a in agents if a is not lost])


def test_member_unreachable_at_prepare_falls_back_then_fails_fast(stub):
    agents = _agents(4)
    dead_url = agents[2][1]
    agents[2][0].stop()
    try:
        gate = ClusterGate(AgentTransport(token=TOKEN), members_from([u for _, u in agents], [8] * 4), SIZES,
                           timeout_s=120).prepare_async()
        t0 = time.monotonic()
        res = gate.run()
        assert not res["ok"] and not res["pipelined"] and res["prepare_error"]
        assert time.monotonic() - t0 < 20
        assert any(dead_url in e for e in res["errors"])
        assert _eventually(lambda: not [f for d in _left(stub) for f in os.listdir(stub / "rendezvous" / d)
                                        if f.startswith("rank-")])
    finally:
        _stop([a for i, a in enumerate(agents) if i != 2])


def test_contract_violations_are_refused(stub):
    """What RCCL refuses, the stub refuses -- so a layout bug in the gate shows on the CPU."""
    uid = rccl.unique_id()
    g = rccl.GateComm(uid, 16, 0, list(range(8)))
    with pytest.raises(rccl.RCCLError, match="rank 0 of this unique id claimed twice"):
        rccl.GateComm(uid, 16, 0, list(range(8)))
    with pytest.raises(rccl.RCCLError, match="unique id used with world 16 and 24"):
        rccl.GateComm(uid, 24, 8, list(range(8)))
    with pytest.raises(rccl.RCCLError, match="device 1 given to ranks 9 and 10 of one process"):
        rccl.GateComm(uid, 16, 8, [0, 1, 1, 3, 4, 5, 6, 7])
    with pytest.raises(ValueError, match="at most 256 ranks"):
        rccl.GateComm(rccl.unique_id(), 512, 0, list(range(8))).sweep(SIZES, dtype="bf16")
    g.abort()
    assert rccl.pending_gates() == 0
