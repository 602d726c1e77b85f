"""Bounded parallel fan-out with retries and per-task timing.

The reference's only parallelism is Terraform's graph walk at its default
``-parallelism=10`` (``shell/run_terraform.go:38``), so bringing up more than
10 nodes serialises into waves.  :func:`fan_out` runs every independent
per-host task concurrently (default width 64), retries idempotent tasks with
exponential backoff, and records start/end times for the bring-up report.
"""

import concurrent.futures as cf
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Generic, List, Optional, Sequence, TypeVar

from ..utils.trace import span

T = TypeVar("T")
R = TypeVar("R")

DEFAULT_WIDTH = 64


@dataclass
class TaskResult(Generic[R]):
    key: str
    ok: bool
    value: Optional[R] = None
    error: Optional[str] = None
    attempts: int = 0
    start: float = 0.0
    end: float = 0.0

    @property
    def seconds(self) -> float:
        return self.end - self.start


@dataclass
class FanOutReport:
    results: List[TaskResult] = field(default_factory=list)
    wall: float = 0.0

    @property
    def ok(self) -> bool:
        return all(r.ok for r in self.results)

    @property
    def failures(self) -> List[TaskResult]:
        return [r for r in self.results if not r.ok]

    def by_key(self) -> Dict[str, TaskResult]:
        return {r.key: r for r in self.results}


def fan_out(items: Sequence[T], fn: Callable[[T], R], key: Callable[[T], str] = str, width: int = DEFAULT_WIDTH,
            retries: int = 0, backoff: float = 0.5, retry_on: Callable[[BaseException], bool] = lambda e: True,
            name: str = "fanout", cancel_on_failure: bool = False) -> FanOutReport:
    """Run ``fn`` over ``items`` with at most ``width`` in flight."""
    report = FanOutReport()
    if not items:
        return report
    stop = threading.Event()

    def run_one(item: T) -> TaskResult:
        k = key(item)
        res: TaskResult = TaskResult(k, False, start=time.time())
        delay = backoff
        with span(name, key=k):
            while True:
                res.attempts += 1
                if stop.is_set():
                    res.error = "canceled"
                    break
                try:
                    res.value = fn(item)
                    res.ok = True
                    break
                except BaseException as exc:  # noqa: BLE001 - collected per task
                    res.error = f"{type(exc).__name__}: {exc}" if not str(exc).startswith(type(exc).__name__) \
                        else str(exc)
                    if res.attempts > retries or not retry_on(exc):
                        if cancel_on_failure:
                            stop.set()
                        break
                    time.sleep(delay)
                    delay *= 2
        res.end = time.time()
        return res

    t0 = time.time()
    w = max(1, min(width, len(items)))
    if w == 1:
        report.results = [run_one(i) for i in items]
    else:
        with cf.ThreadPoolExecutor(max_workers=w, thread_name_prefix=name) as pool:
            report.results = list(pool.map(run_one, items))
    report.wall = time.time() - t0
    return report


_POOLS: Dict[str, cf.ThreadPoolExecutor] = {}
_POOLS_MU = threading.Lock()


def shared_pool(name: str, width: int) -> cf.ThreadPoolExecutor:
    """A process-wide, never shut down worker pool (one per ``name``; ``width`` of the
    first request wins).  Bring-up paths reuse its threads — and the keep-alive HTTP
    connections those threads hold — instead of creating threads per operation, which
    contends with HIP/RCCL work in GPU processes.  A task must never wait on work it
    submitted to the same pool."""
    with _POOLS_MU:
        pool = _POOLS.get(name)
        if pool is None:
            pool = _POOLS[name] = cf.ThreadPoolExecutor(max_workers=max(1, width), thread_name_prefix=name)
        return pool


def describe_failures(report: FanOutReport) -> str:
    return "; ".join(f"{r.key}: {r.error}" for r in report.failures)


__all__: List[Any] = ["fan_out", "FanOutReport", "TaskResult", "describe_failures", "DEFAULT_WIDTH", "shared_pool"]
