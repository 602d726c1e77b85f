"""Cluster-wide RCCL gate: one communicator across every GPU of the cluster's MI355X workers.

Each node agent owns its node's GPUs and joins as ranks ``rank_base .. rank_base+ndev-1``
(``ops/rccl.py:GateComm``).  The gate has two halves:

* :meth:`ClusterGate.prepare_async`: ask the rank-0 agent to start its ranks under a new
  ``ncclUniqueId`` (it keeps one ready) and return the id, then ask every other agent to
  *start* its communicator init with it (RCCL non-blocking mode).  This needs
  only the cluster membership, which is known as soon as the node modules are in the
  document, so ``create cluster`` starts it together with the apply.  Communicator
  bring-up then overlaps node bootstrap instead of following it.
* :meth:`ClusterGate.run`: after the readiness waiter has seen the cluster active, all
  nodes Ready and ``amd.com/gpu`` allocatable, every agent finishes its init if needed,
  runs the verified all-reduce sweep and tears the communicator down.

If preparation failed, ``run`` falls back to a fresh uid and a plain (non-pipelined)
gate.  :meth:`ClusterGate.abort` releases prepared communicators when the gate will not
run, for example when a node failed and the apply raised.

A gate fails fast: RCCL gives a rank waiting for an absent peer no way out but its own
timeout, so when one member's gate request fails (unreachable agent, failed init), ``run``
at once cancels the others' (``/v1/rccl-abort`` on a running sweep, ``tkr_gate_cancel``)
instead of letting every node wait out ``timeout_s``; the result names each member's error.
"""

import concurrent.futures as cf
import threading
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence

from ..parallel.fanout import shared_pool
from ..parallel.transport import HostRef
from ..utils.trace import span


@dataclass
class GateMember:
    url: str  # agent base URL (without the "agent+" scheme prefix)
    rank_base: int
    ndev: int

    @property
    def host(self) -> HostRef:
        return HostRef("agent+" + self.url)


def members_from(urls: Sequence[str], ndevs: Optional[Sequence[int]] = None) -> List[GateMember]:
    out: List[GateMember] = []
    base = 0
    for i, u in enumerate(urls):
        n = int(ndevs[i]) if ndevs else 1
        out.append(GateMember(u[len("agent+"):] if u.startswith("agent+") else u, base, n))
        base += n
    return out


class ClusterGate:
    def __init__(self, transport: Any, members: List[GateMember], sizes: Sequence[int], iters: int = 5,
                 timeout_s: float = 300.0):
        if not members:
            raise ValueError("a cluster gate needs at least one member")
        self.transport = transport
        self.members = members
        self.timeout_s = float(timeout_s)
        self.world = sum(m.ndev for m in members)
        self.sizes = list(sizes)
        self.iters = iters
        self.uid: Optional[str] = None
        self.prepared = False
        self.prepare_error: Optional[str] = None
        self.done = False
        self._thread: Optional[cf.Future] = None
        self._mu = threading.Lock()

    # --- construction from the state document ---------------------------------------------------------
    @classmethod
    def from_state(cls, state, cluster_key: str, transport: Any, sizes: Sequence[int],
                   iters: int = 5) -> Optional["ClusterGate"]:
        """Gate over the cluster's MI355X host modules; None unless every one is an agent host."""
        from ..node.partition import logical_gpus
        from ..terraform.catalog import module_from_source

        urls: List[str] = []
        ndevs: List[int] = []
        for host in sorted(state.nodes(cluster_key)):
            cfg = state.module(state.nodes(cluster_key)[host]) or {}
            info = module_from_source(str(cfg.get("source", "")))
            if info is None or not info.mi355x:
                continue
            addr = str(cfg.get("host", ""))
            if not addr.startswith("agent+"):
                return None  # SSH-managed GPU node: no agent to hold a communicator
            urls.append(addr)
            ndevs.append(logical_gpus(cfg))  # RCCL ranks: GPUs x compute partitions
        if not urls:
            return None
        return cls(transport, members_from(urls, ndevs), sizes, iters)

    # --- pipelined init ---------------------------------------------------------------------------------
    def _prepare(self) -> None:
        try:
            with span("gate.prepare", world=self.world):
                # the first member hosts the rendezvous: one request takes its unique id and
                # starts its ranks; the others join with that id
                m0 = self.members[0]
                first = self.transport.post(m0.host, "/v1/rccl-prepare", {
                    "world": self.world, "rank_base": m0.rank_base, "ndev": m0.ndev, "max_bytes": max(self.sizes),
                    "sizes": self.sizes})
                uid = first["uid"]
                with self._mu:
                    self.uid = uid  # abort() can release member 0 even if a later post fails
                if len(self.members) > 1:
                    def one(m: GateMember) -> Dict[str, Any]:
                        return self.transport.post(m.host, "/v1/rccl-prepare", {
                            "uid": uid, "world": self.world, "rank_base": m.rank_base, "ndev": m.ndev,
                            "max_bytes": max(self.sizes), "sizes": self.sizes})

                    list(shared_pool("tk-gate", 64).map(one, self.members[1:]))
            with self._mu:
                self.prepared = True
        except Exception as exc:  # noqa: BLE001 - run() falls back to an unprepared gate
            with self._mu:
                self.prepare_error = f"{type(exc).__name__}: {exc}"

    def prepare_async(self) -> "ClusterGate":
        # its own pool: _prepare itself fans out on "tk-gate"
        self._thread = shared_pool("tk-gate-prepare", 4).submit(self._prepare)
        return self

    def _join(self) -> None:
        if self._thread is not None:
            self._thread.result()
            self._thread = None

    # --- the gate ---------------------------------------------------------------------------------------
    def run(self) -> Dict[str, Any]:
        self._join()
        pipelined = self.prepared
        if not pipelined:
            if self.uid is not None:
                self.abort()
            self.uid = self.transport.post(self.members[0].host, "/v1/rccl-uid", {})["uid"]
        uid = self.uid
        results = self._gate_all(uid)
        retry = None
        if not all(r.get("ok") for r in results) and any(_oom(r.get("error")) for r in results):
            # a member's communicator init ran out of device memory beside its held burn-in
            # spans (node/agent_gate.py): every member releases its spans, and the gate runs
            # once more under a new id
            first = [f"{m.url}: {r['error']}" for m, r in zip(self.members, results) if _oom(r.get("error"))]
            with span("gate.retry", world=self.world, why="oom"):
                self.uid = uid = self.transport.post(self.members[0].host, "/v1/rccl-uid", {})["uid"]
                results = self._gate_all(uid, release_holds=True)
            retry = {"why": "oom", "first_errors": first}
        self.done = True
        ok = all(r.get("ok") for r in results)
        busbw = [max(r.get("busbw_gbps") or [0.0]) for r in results]
        errors = [f"{m.url}: {r['error']}" for m, r in zip(self.members, results) if r.get("error")]
        return {"ok": ok, "world": self.world, "nodes": len(self.members), "pipelined": pipelined,
                "prepare_error": self.prepare_error, "errors": errors, "retry": retry,
                "min_peak_busbw_gbps": min(busbw) if busbw else 0.0, "ranks": results}

    def _gate_all(self, uid: str, release_holds: bool = False) -> List[Dict[str, Any]]:
        """Every member's ``/v1/rccl-gate`` at once; the first failure cancels the rest."""
        def one(m: GateMember) -> Dict[str, Any]:
            body = {"uid": uid, "rank": m.rank_base, "world": self.world, "ndev": m.ndev,
                    "sizes": self.sizes, "iters": self.iters, "timeout_s": self.timeout_s}
            if release_holds:
                body["release_holds"] = True
            try:
                return self.transport.post(m.host, "/v1/rccl-gate", body)
            except Exception as exc:  # noqa: BLE001 - reported per member
                return {"ok": False, "error": f"{type(exc).__name__}: {exc}"}

        if len(self.members) == 1:
            return [one(self.members[0])]
        futures = {shared_pool("tk-gate", 64).submit(one, m): i for i, m in enumerate(self.members)}
        out: List[Dict[str, Any]] = [{} for _ in self.members]
        canceled = False
        for fut in cf.as_completed(futures):
            i = futures[fut]
            out[i] = fut.result()
            if not out[i].get("ok") and not canceled:
                canceled = True
                with span("gate.cancel", world=self.world, failed=self.members[i].url):
                    for j, m in enumerate(self.members):
                        if j != i and not any(f.done() for f, k in futures.items() if k == j):
                            try:
                                self.transport.post(m.host, "/v1/rccl-abort", {"uid": uid})
                            except Exception:  # noqa: BLE001 - its own timeout still ends it
                                pass
        return out

    def abort(self) -> None:
        """Release pending communicators on every agent (no-op once the gate ran)."""
        self._join()
        if self.done or self.uid is None:
            return
        uid = self.uid
        for m in self.members:
            try:
                self.transport.post(m.host, "/v1/rccl-abort", {"uid": uid})
            except Exception:  # noqa: BLE001 - best effort; agents also expire stale gates
                pass
        self.prepared = False
        self.uid = None


def _oom(error: Optional[str]) -> bool:
    """A member's init ran out of device memory, and that member has not retried it already
    (a node that is the whole gate retries by itself, node/agent_gate.py)."""
    if not error:
        return False
    from ..ops.rccl import OOM_RETRIED_MARK, is_oom_error

    return is_oom_error(error) and OOM_RETRIED_MARK not in error


__all__ = ["ClusterGate", "GateMember", "members_from"]
