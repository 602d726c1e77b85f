"""Per-phase tracing (the reference records no timings at all).

``with span("apply", executor="direct"):`` records a wall-clock interval into
the process-global :data:`TRACER`.  Spans nest per thread, carry attributes,
and export as a JSON timing report or a Chrome trace (``chrome://tracing`` /
Perfetto) — the bring-up metric (create -> kubectl-ready) is read from them.

Enable file output with ``TK_TRACE=/path/trace.json`` (written at exit by the
CLI) or programmatically via :meth:`Tracer.dump_chrome`.
"""

import contextlib
import json
import os
import threading
import time
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, Iterator, List, Optional


@dataclass
class Span:
    name: str
    start: float
    end: float = 0.0
    thread: str = ""
    parent: Optional[str] = None
    attrs: Dict[str, Any] = field(default_factory=dict)
    error: Optional[str] = None

    @property
    def duration(self) -> float:
        return max(0.0, self.end - self.start)


class Tracer:
    """``max_spans``: the most recent spans kept.  A CLI run records a few hundred, but a
    node agent is a daemon that records spans for every request it serves, for months; the
    oldest go first (``dropped`` counts them)."""

    MAX_SPANS = 20000

    def __init__(self, max_spans: int = MAX_SPANS):
        self._mu = threading.Lock()
        self._local = threading.local()
        self.spans: List[Span] = []
        self.t0 = time.time()
        self.enabled = True
        self.max_spans = max_spans
        self.dropped = 0

    def _keep(self, sp: Span) -> None:
        """Append under ``_mu``; past 1.25 x the bound, trim to it (amortised)."""
        self.spans.append(sp)
        if len(self.spans) > self.max_spans + self.max_spans // 4:
            cut = len(self.spans) - self.max_spans
            del self.spans[:cut]
            self.dropped += cut

    def _stack(self) -> List[Span]:
        st = getattr(self._local, "stack", None)
        if st is None:
            st = self._local.stack = []
        return st

    @contextlib.contextmanager
    def span(self, name: str, **attrs: Any) -> Iterator[Span]:
        stack = self._stack()
        sp = Span(name, time.time(), thread=threading.current_thread().name,
                  parent=stack[-1].name if stack else None, attrs=dict(attrs))
        stack.append(sp)
        try:
            yield sp
        except BaseException as exc:
            sp.error = f"{type(exc).__name__}: {exc}"
            raise
        finally:
            sp.end = time.time()
            stack.pop()
            if self.enabled:
                with self._mu:
                    self._keep(sp)

    def mark(self, name: str, **attrs: Any) -> None:
        now = time.time()
        with self._mu:
            self._keep(Span(name, now, now, threading.current_thread().name, None, dict(attrs)))

    def reset(self) -> None:
        with self._mu:
            self.spans.clear()
            self.dropped = 0
            self.t0 = time.time()

    def find(self, name: str) -> List[Span]:
        with self._mu:
            return [s for s in self.spans if s.name == name]

    def report(self) -> Dict[str, Any]:
        with self._mu:
            spans = sorted(self.spans, key=lambda s: s.start)
        return {
            "t0": self.t0,
            "spans": [dict(asdict(s), duration=s.duration, rel_start=s.start - self.t0) for s in spans],
            "dropped": self.dropped,
        }

    def chrome_events(self) -> List[Dict[str, Any]]:
        pid = os.getpid()
        with self._mu:
            spans = list(self.spans)
        tids: Dict[str, int] = {}
        events = []
        for s in spans:
            tid = tids.setdefault(s.thread, len(tids))
            events.append({"name": s.name, "ph": "X", "ts": (s.start - self.t0) * 1e6, "dur": s.duration * 1e6,
                           "pid": pid, "tid": tid, "args": dict(s.attrs, error=s.error) if s.error else s.attrs})
        return events

    def dump_chrome(self, path: str) -> None:
        with open(path, "w", encoding="utf-8") as fh:
            json.dump({"traceEvents": self.chrome_events()}, fh)


TRACER = Tracer()


def span(name: str, **attrs: Any):
    return TRACER.span(name, **attrs)
