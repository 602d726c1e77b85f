"""parallel/fanout.py: bounded fan-out with retries, and the process-wide worker pools."""

import threading
import time

from triton_kubernetes_amd.parallel.fanout import describe_failures, fan_out, shared_pool


def test_fan_out_runs_concurrently_and_times_tasks():
    barrier = threading.Barrier(8, timeout=5)

    def task(i):
        barrier.wait()  # only completes if all 8 run at once
        return i * i

    rep = fan_out(list(range(8)), task, key=str, width=8)
    assert rep.ok and [r.value for r in rep.results] == [i * i for i in range(8)]
    assert all(r.seconds >= 0 for r in rep.results) and rep.wall >= 0


def test_fan_out_retries_with_backoff_and_reports():
    calls = {}

    def flaky(i):
        calls[i] = calls.get(i, 0) + 1
        if i == 1 and calls[i] < 3:
            raise RuntimeError("transient")
        if i == 2:
            raise ValueError("permanent")
        return i

    rep = fan_out([0, 1, 2], flaky, width=3, retries=2, backoff=0.001,
                  retry_on=lambda e: isinstance(e, RuntimeError))
    by = rep.by_key()
    assert by["1"].ok and by["1"].attempts == 3
    assert not by["2"].ok and by["2"].attempts == 1  # not retried
    assert describe_failures(rep) == "2: ValueError: permanent"


def test_cancel_on_failure_stops_pending_work():
    started = []

    def task(i):
        started.append(i)
        if i == 0:
            raise RuntimeError("boom")
        time.sleep(0.01)
        return i

    rep = fan_out(list(range(20)), task, width=1, cancel_on_failure=True)
    assert not rep.ok and started == [0]
    assert all(r.error == "canceled" for r in rep.results[1:])


def test_shared_pool_is_reused():
    a = shared_pool("t-pool", 2)
    assert shared_pool("t-pool", 99) is a
    names = set(a.map(lambda _: threading.current_thread().name, range(20)))
    assert len(names) <= 2 and all(n.startswith("t-pool") for n in names)
    assert shared_pool("t-other", 1) is not a
