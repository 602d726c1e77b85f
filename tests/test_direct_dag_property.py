"""The DirectExecutor's dependency-driven walk (``executor/direct.py:_apply_report``) over
generated module graphs: a module starts only after every module it references finished
``ok``; one whose dependency failed is ``blocked`` and never runs; every module runs at
most once; no more than ``parallelism`` run at a time; and a cycle ends the walk with
``dependency cycle`` instead of hanging."""

import random
import threading
import time

from hypothesis import given, settings
from hypothesis import strategies as st

from triton_kubernetes_amd.backend.memory import MemoryBackend
from triton_kubernetes_amd.executor.direct import DirectExecutor, ModuleRun


class _State:
    name = "dag"


class DagExecutor(DirectExecutor):
    def __init__(self, graph, fail, parallelism, seed):
        super().__init__(parallelism=parallelism)
        self.graph, self.fail = graph, set(fail)
        self.rng = random.Random(seed)
        self.mu = threading.Lock()
        self.started, self.finished = {}, {}
        self.running = self.max_running = 0
        self.runs_of = {}

    def plan(self, state):
        return {k: ModuleRun(k, None, {}, set(deps), hash=k) for k, deps in self.graph.items()}

    @staticmethod
    def _prefetch_tls(runs, tf):
        return None

    def _apply_module(self, run, outputs, name):
        with self.mu:
            self.runs_of[run.key] = self.runs_of.get(run.key, 0) + 1
            self.started[run.key] = (time.monotonic(), dict(self.finished))
            self.running += 1
            self.max_running = max(self.max_running, self.running)
            pause = self.rng.random() * 0.002
        time.sleep(pause)
        with self.mu:
            self.running -= 1
            self.finished[run.key] = "failed" if run.key in self.fail else "ok"
        if run.key in self.fail:
            raise RuntimeError("boom")
        return {"out": run.key}, None


@st.composite
def graphs(draw):
    n = draw(st.integers(1, 12))
    keys = [f"m{i}" for i in range(n)]
    graph = {k: set(draw(st.lists(st.sampled_from(keys[:i]), max_size=3))) if i else set()
             for i, k in enumerate(keys)}
    fail = draw(st.lists(st.sampled_from(keys), max_size=2, unique=True))
    return graph, fail, draw(st.integers(1, 4)), draw(st.integers(0, 2 ** 16))


def _expected(graph, fail):
    status = {}
    for k in sorted(graph, key=lambda x: int(x[1:])):  # deps have lower indices
        if any(status[d] in ("failed", "blocked") for d in graph[k]):
            status[k] = "blocked"
        else:
            status[k] = "failed" if k in fail else "ok"
    return status


@settings(max_examples=120, deadline=None)
@given(graphs())
def test_walk_respects_dependencies_failures_and_parallelism(case):
    graph, fail, width, seed = case
    ex = DagExecutor(graph, fail, width, seed)
    report = ex._apply_report(_State(), MemoryBackend())
    want = _expected(graph, fail)
    assert {k: r.status for k, r in report.runs.items()} == want
    assert all(n == 1 for n in ex.runs_of.values())
    assert set(ex.runs_of) == {k for k, s in want.items() if s != "blocked"}  # a blocked module never runs
    for k, (_, done_then) in ex.started.items():
        assert all(done_then.get(d) == "ok" for d in graph[k]), (k, graph[k], done_then)
    assert ex.max_running <= width


def test_a_cycle_ends_the_walk():
    graph = {"a": set(), "b": {"c"}, "c": {"b"}, "d": {"a", "c"}}
    ex = DagExecutor(graph, [], 4, 0)
    report = ex._apply_report(_State(), MemoryBackend())
    st_ = {k: r.status for k, r in report.runs.items()}
    assert st_["a"] == "ok" and st_["b"] == st_["c"] == "failed"
    assert report.runs["b"].error == "dependency cycle" and st_["d"] in ("failed", "blocked")
    assert set(ex.runs_of) == {"a"}


def test_a_chain_of_dependents_of_a_failure_is_blocked_not_a_cycle():
    """m10 sorts before m4 and m7, which depend on the failed m0: in the pass where m0's
    failure is seen, m10 was still undecided when nothing was left running, and the walk
    called it a dependency cycle.  The walk now settles each pass to a fixed point."""
    graph = {"m0": set(), "m1": set(), "m2": {"m0"}, "m3": {"m0"}, "m4": {"m0"}, "m5": set(), "m6": {"m0", "m3"},
             "m7": {"m0"}, "m8": set(), "m9": set(), "m10": {"m4", "m7", "m8"}, "m11": set()}
    for seed in range(20):
        report = DagExecutor(graph, ["m0", "m1"], 4, seed)._apply_report(_State(), MemoryBackend())
        assert report.runs["m10"].status == "blocked", (seed, report.runs["m10"].error)
