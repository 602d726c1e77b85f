"""A gate communicator init that runs out of HBM beside held burn-in spans.

A full burn-in's span leaves ``probe.SPAN_HEADROOM`` free on each GPU and is held until the
node's RCCL inits are through; the gate's communicator allocates into that headroom.  On a
node of 8 xGMI peers the headroom was an unmeasured constant.  When the init fails for lack
of memory, the agent releases every held span and retries once (``gate_retry: oom``); the
footprint a successful init measured sets the node's headroom from then on.

The ABI stub models the allocation (``ops/csrc/tk_rccl_stub.cpp``: ``TK_RCCL_STUB_HBM_FREE``
holds each GPU's free bytes, an init needs ``TK_RCCL_STUB_FOOTPRINT_MIB`` per GPU).  The
burn-in child here is a stand-in ``gpu-burnin`` that holds its span -- the free bytes stay
low -- until the release hold lets go, as the real child does: the retry can only pass if
the agent really released it.
"""

import base64
import json
import os
import stat
import sys
import tempfile

import pytest

from triton_kubernetes_amd.node.agent import NodeAgent
from triton_kubernetes_amd.node.labels import synthetic_topology
from triton_kubernetes_amd.node.plan import BootstrapPlan, Step
from triton_kubernetes_amd.ops import native, probe, rccl
from triton_kubernetes_amd.parallel.transport import AgentTransport
from triton_kubernetes_amd.readiness.gate import ClusterGate, members_from

TOKEN = "gate-oom-token-0123456"
SIZES = [1 << 20, 16 << 20]
HELD = 300 << 20  # what a held span leaves free (MiB-sized: below the footprint)
RELEASED = 200 << 30
FOOTPRINT_MIB = 8000


@pytest.fixture
def oom_node(tmp_path, monkeypatch):
    from triton_kubernetes_amd.ops.build import build

    build(only=["libtk_rccl_stub.so"])
    free = tmp_path / "hbm-free"
    free.write_text(str(RELEASED))
    monkeypatch.setenv("TK_RCCL_LIB", os.path.join(native.LIB_DIR, "libtk_rccl_stub.so"))
    monkeypatch.setenv("TK_RCCL_STUB_DIR", str(tmp_path / "rendezvous"))
    monkeypatch.setenv("TK_RCCL_STUB_LOG", str(tmp_path / "calls.jsonl"))
    monkeypatch.setenv("TK_RCCL_STUB_HBM_FREE", str(free))
    monkeypatch.setenv("TK_RCCL_STUB_FOOTPRINT_MIB", str(FOOTPRINT_MIB))
    monkeypatch.setattr(native, "_cache", {})
    monkeypatch.setattr(probe, "SPAN_HEADROOM", probe.SPAN_HEADROOM)  # restored after the test
    # the stand-in burn-in child: its verdict, then the span held (free stays low) until
    # stdin closes -- the release hold letting go -- then the span released
    exe = tmp_path / "gpu-burnin"
    exe.write_text(f"""#!{sys.executable}
import json, sys
free = {str(free)!r}
open(free, "w").write({str(HELD)!r})
print(json.dumps({{"ok": True}}), flush=True)
if "--hold-stdin" in sys.argv:
    sys.stdin.read()
open(free, "w").write({str(RELEASED)!r})
""")
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)
    yield tmp_path, exe, free
    probe.set_release_hold(None)
    probe.wait_frees()


def _calls(tmp_path):
    path = tmp_path / "calls.jsonl"
    return [json.loads(ln) for ln in path.read_text().splitlines()] if path.exists() else []


def _agent(ndev=8):
    a = NodeAgent(name="gpu-0", mode="sim", devices=list(range(ndev)), token=TOKEN, root=tempfile.mkdtemp(),
                  topology_override=synthetic_topology(ndev), burnin_override=lambda d, lvl: {"ok": True},
                  gate_backend="rccl")
    return a


def _hold_span(agent, exe):
    """A burn-in child holding its span, held by the agent's own release hold (which waits,
    as for a link matrix still to measure, until released)."""
    agent._links_pending = True
    probe.set_release_hold(agent._await_rccl_inits)
    doc, _ = probe._child_verdict([str(exe), "--burnin-child", "--device", "0"], 0, 30, "burn-in")
    assert doc == {"ok": True}


def test_is_oom_error_reads_rccl_failures():
    assert rccl.is_oom_error("ncclCommInitRank: unhandled cuda error (run with NCCL_DEBUG=INFO for details) "
                             "[rccl: Cuda failure 'out of memory'] (device 3: 120 MiB free)")
    assert rccl.is_oom_error("ncclCommInitRank: unhandled system error (device 0: 800 MiB free)")
    assert rccl.is_oom_error("hipMalloc(&b.send, max_bytes): hipErrorOutOfMemory")
    assert not rccl.is_oom_error("ncclCommInitRank: unhandled system error (device 0: 250000 MiB free)")
    assert not rccl.is_oom_error("communicator not ready after 600000 ms")
    assert not rccl.is_oom_error("gate canceled while its communicator waited for peers")
    assert not rccl.is_oom_error("")


def test_whole_node_gate_retries_once_after_releasing_held_spans(oom_node):
    tmp_path, exe, free = oom_node
    agent = _agent()
    url = agent.serve()
    try:
        _hold_span(agent, exe)
        assert int(free.read_text()) == HELD
        gate = ClusterGate(AgentTransport(token=TOKEN), members_from([url], [8]), SIZES, timeout_s=30).prepare_async()
        res = gate.run()
        assert res["ok"], res
        rank = res["ranks"][0]
        assert rank["gate_retry"] == "oom" and "out of memory" in rank["first_error"]
        assert rank["spans_released_ms"] >= 0
        assert int(free.read_text()) == RELEASED  # the child let go of its span
        ops = [c["op"] for c in _calls(tmp_path) if c["op"].startswith("begin")]
        assert ops == ["begin-oom", "begin"]  # one failed init, one retry
        # the footprint the retried init measured is kept, and sizes the span's headroom
        # ... and the out-of-memory init doubles the headroom the next burn-in leaves
        floor = (4 << 30) + 7 * (512 << 20)
        fp = json.loads(open(agent.path(agent.FOOTPRINT_FILE)).read())
        assert fp == {"8": float(FOOTPRINT_MIB), "oom:8": 2.0 * floor / (1 << 20)}
        measured = int(FOOTPRINT_MIB * agent.HEADROOM_MARGIN * (1 << 20)) + (1 << 30)
        want = max(measured, 2 * floor)
        assert agent.span_headroom(8) == want > floor
        assert probe.SPAN_HEADROOM == want
        assert rank["phase_ms"]["footprint_total_mib"] == FOOTPRINT_MIB
        assert rank["phase_ms"]["footprint_kept"] == 1.0  # the answer says it counted
    finally:
        agent.stop()
    # a later agent on this node starts with the measured headroom
    again = NodeAgent(name="gpu-0", mode="sim", devices=list(range(8)), token=TOKEN, root=agent.root,
                      topology_override=synthetic_topology(8), gate_backend="rccl")
    assert again.span_headroom(8) == want and again.span_headroom(4) == (4 << 30) + 3 * (512 << 20)


def test_rccl_local_step_retries_and_the_gate_reports_it(oom_node):
    tmp_path, exe, free = oom_node
    agent = _agent()
    plan = BootstrapPlan("n", "worker", "http://r", "tok", "ca", steps=[Step("rccl_local", "rccl_local", "true")])
    try:
        _hold_span(agent, exe)
        prep = agent.rccl_prepare(None, world=8, rank_base=0, ndev=8, max_bytes=16 << 20, sizes=SIZES)
        uid = base64.b64decode(prep["uid"])
        detail = agent.run_plan(plan)["steps"][0]["detail"]
        assert detail["gate_retry"] == "oom" and detail["shared_with"] == "cluster_gate" and detail["ok"]
        res = agent.rccl_gate(0, 8, uid, SIZES, ndev=8)
        assert res["ok"] and res["shared_with"] == "rccl_local" and res["gate_retry"] == "oom"
        assert int(free.read_text()) == RELEASED
    finally:
        agent.stop()


def test_no_second_retry_when_the_release_does_not_free_enough(oom_node, monkeypatch):
    """The retry happens once: a GPU that is still short after the release fails the gate
    with the out-of-memory error, instead of looping."""
    tmp_path, exe, free = oom_node
    monkeypatch.setenv("TK_RCCL_STUB_FOOTPRINT_MIB", str(RELEASED // (1 << 20) + 1))  # never fits
    agent = _agent()
    url = agent.serve()
    try:
        _hold_span(agent, exe)
        res = ClusterGate(AgentTransport(token=TOKEN), members_from([url], [8]), SIZES, timeout_s=30).run()
        assert not res["ok"] and "out of memory" in res["errors"][0] and "failed again" in res["errors"][0]
        assert res["retry"] is None  # the node retried by itself; the cluster gate does not again
        ops = [c["op"] for c in _calls(tmp_path) if c["op"].startswith("begin")]
        assert ops == ["begin-oom", "begin-oom"]
    finally:
        agent.stop()


def test_other_failures_are_not_retried(oom_node, monkeypatch):
    """Only an out-of-memory init is retried: a peer that never comes is not."""
    tmp_path, exe, free = oom_node
    agent = _agent(ndev=2)
    try:
        prep = agent.rccl_prepare(None, world=4, rank_base=0, ndev=2, sizes=SIZES)  # ranks 2, 3 never join
        with pytest.raises(rccl.RCCLError, match="not ready"):
            agent.rccl_gate(0, 4, base64.b64decode(prep["uid"]), SIZES, ndev=2, timeout_s=0.3)
        assert [c["op"] for c in _calls(tmp_path) if c["op"].startswith("begin")] == ["begin"]
    finally:
        agent.stop()


def test_multi_node_gate_retries_every_member_with_released_spans(oom_node):
    """Two nodes: one runs out of memory.  The cluster gate releases every member's spans
    and runs the whole gate again under a new id."""
    tmp_path, exe, free = oom_node
    a, b = _agent(4), _agent(4)
    ua, ub = a.serve(), b.serve()
    try:
        _hold_span(a, exe)
        gate = ClusterGate(AgentTransport(token=TOKEN), members_from([ua, ub], [4, 4]), SIZES, timeout_s=30)
        res = gate.prepare_async().run()
        assert res["ok"], res
        assert res["retry"]["why"] == "oom" and len(res["retry"]["first_errors"]) >= 1
        assert all(r["gate_retry"] == "oom" for r in res["ranks"])
        assert int(free.read_text()) == RELEASED
        worlds = {c["uid"] for c in _calls(tmp_path) if c["op"] == "begin"}
        assert len(worlds) == 1  # the retry's communicator: one new unique id for both nodes
    finally:
        a.stop()
        b.stop()


def test_an_implausible_footprint_never_becomes_the_headroom(oom_node, monkeypatch):
    """A "footprint" of a burn-in span's size (what a device-wide free-memory delta read
    while the burn-in child allocated, before the per-process accounting) is not kept: it
    would have left the next full burn-in almost nothing to test."""
    tmp_path, exe, free = oom_node
    monkeypatch.setenv("TK_RCCL_STUB_FOOTPRINT_MIB", str(290 * 1024))
    free.write_text(str(300 << 30))
    agent = _agent()
    url = agent.serve()
    try:
        res = ClusterGate(AgentTransport(token=TOKEN), members_from([url], [8]), SIZES, timeout_s=30).run()
        assert res["ok"], res
        assert res["ranks"][0]["phase_ms"]["footprint_kept"] == 0.0
        assert not os.path.exists(agent.path(agent.FOOTPRINT_FILE))
        assert agent.span_headroom(8) == (4 << 30) + 7 * (512 << 20)
    finally:
        agent.stop()


def test_a_device_wide_footprint_is_kept_only_from_a_quiet_window(oom_node, monkeypatch):
    """Without per-process accounting (an agent inside a PID namespace: the KFD keys its
    entries by host pids) the footprint is the device's used-memory delta, which a burn-in
    child allocating its span meanwhile inflates.  It is kept only when none of the agent's
    burn-ins started, ran or was alive across the init."""
    tmp_path, exe, free = oom_node
    monkeypatch.setenv("TK_RCCL_STUB_FOOTPRINT_KIND", "2")
    monkeypatch.setenv("TK_RCCL_STUB_FOOTPRINT_MIB", "900")
    agent = _agent()
    url = agent.serve()
    try:
        _hold_span(agent, exe)  # a child alive (holding its span) across the gate
        free.write_text(str(RELEASED))
        res = ClusterGate(AgentTransport(token=TOKEN), members_from([url], [8]), SIZES, timeout_s=30).run()
        assert res["ok"] and res["ranks"][0]["phase_ms"]["footprint_kind"] == 2.0
        assert res["ranks"][0]["phase_ms"]["footprint_kept"] == 0.0
        assert not os.path.exists(agent.path(agent.FOOTPRINT_FILE))
        agent._links_pending = False
        probe.wait_frees()  # the child released and exited: a quiet window now
        res = ClusterGate(AgentTransport(token=TOKEN), members_from([url], [8]), SIZES, timeout_s=30).run()
        assert res["ok"] and res["ranks"][0]["phase_ms"]["footprint_kept"] == 1.0
        assert json.loads(open(agent.path(agent.FOOTPRINT_FILE)).read()) == {"8": 900.0}
    finally:
        agent.stop()
