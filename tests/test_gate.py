"""Cluster RCCL gate orchestration (readiness/gate.py) against a recording fake transport."""

import threading

import pytest

from triton_kubernetes_amd.readiness.gate import ClusterGate, members_from
from triton_kubernetes_amd.state import State


class FakeAgents:
    """Answers the agent RCCL endpoints; records (url, path, body)."""

    def __init__(self, fail_prepare_on=None, fail_gate=False):
        self.calls = []
        self.mu = threading.Lock()
        self.pending = {}
        self.fail_prepare_on = fail_prepare_on
        self.fail_gate = fail_gate

    def post(self, host, path, body):
        url = host.agent_url
        with self.mu:
            self.calls.append((url, path, dict(body)))
        if path == "/v1/rccl-uid":
            return {"uid": "UID-" + str(len(self.calls))}
        if path == "/v1/rccl-prepare":
            if url == self.fail_prepare_on:
                raise RuntimeError("agent unreachable")
            uid = body.get("uid") or "UID-" + str(len(self.calls))  # no uid: host the rendezvous
            with self.mu:
                self.pending[(url, uid)] = dict(body, uid=uid)
            return {"ok": True, "uid": uid}
        if path == "/v1/rccl-gate":
            with self.mu:
                pipelined = self.pending.pop((url, body["uid"]), None) is not None
            return {"ok": not self.fail_gate, "busbw_gbps": [10.0 + body["rank"]], "pipelined": pipelined}
        if path == "/v1/rccl-abort":
            with self.mu:
                self.pending.pop((url, body["uid"]), None)
            return {"ok": True}
        raise AssertionError(path)

    def paths(self):
        return [c[1] for c in self.calls]


def test_members_rank_layout():
    ms = members_from(["agent+http://a:1", "http://b:2", "agent+http://c:3"], [8, 8, 4])
    assert [(m.url, m.rank_base, m.ndev) for m in ms] == [("http://a:1", 0, 8), ("http://b:2", 8, 8),
                                                          ("http://c:3", 16, 4)]
    assert [m.rank_base for m in members_from(["u1", "u2"])] == [0, 1]


def test_pipelined_gate_runs_prepared_communicators():
    fake = FakeAgents()
    gate = ClusterGate(fake, members_from(["http://a", "http://b"], [8, 8]), [1 << 20], 3).prepare_async()
    res = gate.run()
    assert res["ok"] and res["pipelined"] and res["world"] == 16 and res["nodes"] == 2
    prep = [c for c in fake.calls if c[1] == "/v1/rccl-prepare"]
    assert sorted((c[0], c[2]["rank_base"], c[2]["ndev"], c[2]["world"]) for c in prep) == [
        ("http://a", 0, 8, 16), ("http://b", 8, 8, 16)]
    # one request to the first member takes its unique id; the others join with it
    assert "uid" not in prep[0][2] and "/v1/rccl-uid" not in fake.paths()
    runs = [c for c in fake.calls if c[1] == "/v1/rccl-gate"]
    assert {c[2]["uid"] for c in runs} == {prep[1][2]["uid"]} == {gate.uid}
    assert all(r["pipelined"] for r in res["ranks"])
    assert res["min_peak_busbw_gbps"] == 10.0
    gate.abort()  # after run: no-op
    assert "/v1/rccl-abort" not in fake.paths()


def test_failed_prepare_falls_back_and_releases():
    fake = FakeAgents(fail_prepare_on="http://b")
    gate = ClusterGate(fake, members_from(["http://a", "http://b"]), [1 << 20]).prepare_async()
    res = gate.run()
    assert res["ok"] and not res["pipelined"] and "agent unreachable" in res["prepare_error"]
    # the half-prepared uid was aborted, a fresh one used for the gate
    aborts = [c for c in fake.calls if c[1] == "/v1/rccl-abort"]
    assert len(aborts) == 2
    gate_uids = {c[2]["uid"] for c in fake.calls if c[1] == "/v1/rccl-gate"}
    assert gate_uids.isdisjoint({c[2]["uid"] for c in aborts})
    assert not fake.pending


def test_abort_without_run_releases_every_agent():
    fake = FakeAgents()
    gate = ClusterGate(fake, members_from(["http://a", "http://b", "http://c"]), [1 << 20]).prepare_async()
    gate.abort()
    assert fake.paths().count("/v1/rccl-abort") == 3 and not fake.pending
    assert gate.uid is None


def test_gate_failure_reported():
    fake = FakeAgents(fail_gate=True)
    res = ClusterGate(fake, members_from(["http://a"]), [1 << 20]).run()
    assert not res["ok"] and not res["pipelined"]


def _state_with_nodes(hosts):
    st = State("mgr")
    ck = st.add_cluster("baremetal", "c", {"name": "c"})
    src = "github.com/joyent/triton-kubernetes//terraform/modules/{}?ref=master"
    for i, (h, gpu) in enumerate(hosts):
        mod = "bare-metal-mi355x-rancher-k8s-host" if gpu else "bare-metal-rancher-k8s-host"
        cfg = {"source": src.format(mod), "hostname": f"n{i}", "host": h}
        if gpu:
            cfg["gpu_count"] = str(gpu)
        st.add_node(ck, f"n{i}", cfg)
    return st, ck


def test_from_state_membership():
    st, ck = _state_with_nodes([("agent+http://g1", 8), ("10.0.0.5", 0), ("agent+http://g2", 4)])
    gate = ClusterGate.from_state(st, ck, FakeAgents(), [1 << 20])
    assert gate is not None and gate.world == 12
    assert [(m.url, m.rank_base, m.ndev) for m in gate.members] == [("http://g1", 0, 8), ("http://g2", 8, 4)]
    st2, ck2 = _state_with_nodes([("agent+http://g1", 8), ("10.0.0.9", 8)])  # SSH-managed GPU node
    assert ClusterGate.from_state(st2, ck2, FakeAgents(), [1 << 20]) is None
    st3, ck3 = _state_with_nodes([("10.0.0.5", 0)])
    assert ClusterGate.from_state(st3, ck3, FakeAgents(), [1 << 20]) is None


def test_empty_gate_rejected():
    with pytest.raises(ValueError):
        ClusterGate(FakeAgents(), [], [1])


# --- the agent side of an abort (the pop -> sweeping window) -------------------------


def _sim_agent(tmp_path, gpus=2):
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.labels import synthetic_topology

    a = NodeAgent(name="g", mode="sim", devices=list(range(gpus)), token="t" * 24, root=str(tmp_path))
    a.topology_override = synthetic_topology(gpus)
    return a


def test_abort_before_the_gate_request_fails_it_at_once(tmp_path):
    from triton_kubernetes_amd.node.agent_gate import GateAborted

    a = _sim_agent(tmp_path)
    try:
        uid = b"U" * 128
        res = a.rccl_abort(uid)
        assert not res["aborted"] and not res["canceled"]
        with pytest.raises(GateAborted):
            a.rccl_gate(0, 4, uid, [1 << 20], ndev=2)
        with pytest.raises(GateAborted):
            a.rccl_prepare(uid, 4, 0, ndev=2)
        assert not a._gates and not a._sweeping
        # another uid is unaffected
        assert a.rccl_gate(0, 2, b"V" * 128, [1 << 20], ndev=2)["ok"]
    finally:
        a.stop()


def test_abort_while_the_communicator_starts_cancels_the_request(tmp_path, monkeypatch):
    """The abort lands after the gate request took its (absent) pending entry and before its
    fresh communicator exists: the request fails at once and releases what it made."""
    from triton_kubernetes_amd.node import agent_gate
    from triton_kubernetes_amd.node.agent_gate import GateAborted

    a = _sim_agent(tmp_path)
    started, go = threading.Event(), threading.Event()
    aborted = []

    class SlowGate(agent_gate._SimGate):
        def __init__(self, devices):
            started.set()
            go.wait(5)
            super().__init__(devices)

        def abort(self):
            aborted.append(self)

    monkeypatch.setattr(agent_gate, "_SimGate", SlowGate)
    uid = b"W" * 128
    out = {}

    def req():
        try:
            out["res"] = a.rccl_gate(0, 4, uid, [1 << 20], ndev=2)
        except GateAborted as exc:
            out["err"] = exc

    t = threading.Thread(target=req)
    t.start()
    try:
        assert started.wait(5)
        res = a.rccl_abort(uid)
        assert res["canceled"]  # found the request in its reserved slot
        go.set()
        t.join(5)
        assert isinstance(out.get("err"), GateAborted) and len(aborted) == 1
        assert not a._sweeping
    finally:
        go.set()
        a.stop()


def test_abort_during_prepare_releases_the_new_communicator(tmp_path, monkeypatch):
    from triton_kubernetes_amd.node import agent_gate
    from triton_kubernetes_amd.node.agent_gate import GateAborted

    a = _sim_agent(tmp_path)
    uid = b"X" * 128
    aborted = []

    class RacingGate(agent_gate._SimGate):
        def __init__(self, devices):
            a.rccl_abort(uid)  # lands while the prepare is starting its init
            super().__init__(devices)

        def abort(self):
            aborted.append(self)

    monkeypatch.setattr(agent_gate, "_SimGate", RacingGate)
    try:
        with pytest.raises(GateAborted):
            a.rccl_prepare(uid, 4, 0, ndev=2)
        assert len(aborted) == 1 and uid not in a._gates
    finally:
        a.stop()


def test_aborted_uids_expire(tmp_path, monkeypatch):
    a = _sim_agent(tmp_path)
    try:
        uid = b"Y" * 128
        a.rccl_abort(uid)
        monkeypatch.setattr(type(a), "ABORTED_TTL_S", -1.0)
        assert a.rccl_gate(0, 2, uid, [1 << 20], ndev=2)["ok"]
    finally:
        a.stop()
