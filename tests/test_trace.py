"""The tracer and the agent's plan history stay bounded in a long-lived process (the node
agent is a daemon that serves requests for months; tests/test_gpu_soak.py runs one through
cluster after cluster on the GPU)."""

import threading

from triton_kubernetes_amd.utils.trace import Tracer


def test_tracer_keeps_the_most_recent_spans():
    t = Tracer(max_spans=100)
    for i in range(1000):
        with t.span(f"s{i}"):
            pass
    assert 100 <= len(t.spans) <= 125
    assert t.spans[-1].name == "s999"
    assert t.dropped == 1000 - len(t.spans)
    rep = t.report()
    assert rep["dropped"] == t.dropped and len(rep["spans"]) == len(t.spans)
    t.reset()
    assert t.spans == [] and t.dropped == 0


def test_tracer_bound_holds_under_threads():
    t = Tracer(max_spans=50)

    def work(k):
        for i in range(500):
            with t.span(f"t{k}-{i}"):
                pass
            t.mark("m")

    ths = [threading.Thread(target=work, args=(k,)) for k in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert len(t.spans) <= 50 + 50 // 4
    assert t.dropped + len(t.spans) == 4 * 500 * 2


def test_agent_history_is_bounded(tmp_path):
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.plan import BootstrapPlan, Step

    agent = NodeAgent(name="h", mode="sim", root=str(tmp_path))
    for i in range(NodeAgent.HISTORY_KEEP + 10):
        agent.run_plan(BootstrapPlan(f"h{i}", "worker", "http://r", "tok", "ca", steps=[Step("hostname", "hostname", "true")]))
    assert len(agent.history) == NodeAgent.HISTORY_KEEP
    assert agent.history[-1]["hostname"] == f"h{NodeAgent.HISTORY_KEEP + 9}"
