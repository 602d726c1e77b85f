"""The node agent's share of the cluster-wide RCCL gate (N2).

A cluster gate is one RCCL communicator over every GPU of the worker tier: rank ``r`` of
world ``W``, this node holding ranks ``rank_base .. rank_base+ndev-1`` (``ops/rccl.py``
``GateComm``: grouped ``ncclCommInitRank`` over the node's GPUs in one process).  The
readiness waiter (``readiness/gate.py``) drives it over the agent API:

* ``POST /v1/rccl-uid`` / ``rccl-prepare`` -- a unique id (kept one ahead, off the
  bring-up path) and a non-blocking init of this node's ranks, which overlaps the burn-in;
* ``POST /v1/rccl-gate`` -- the verified all-reduce sweep on those ranks;
* ``POST /v1/rccl-abort`` -- release them (another member failed): a pending init is
  aborted and a sweep waiting for peers is canceled at once.

On a one-node cluster the pending communicator spans exactly the node's GPUs, so the
``rccl_local`` plan step sweeps it and the gate answers from that sweep
(:meth:`AgentGateMixin._take_node_gate`).  Pending communicators expire after
``GATE_TTL_S``.  Agents with synthetic GPUs use :class:`_SimGate` unless ``gate_backend``
is ``rccl`` (the ABI stub, ``ops/csrc/tk_rccl_stub.cpp``).
"""

import base64
import secrets
import time
from typing import Any, Dict, List, Optional, Tuple

from ..utils.trace import span


class _SimGate:
    """Stand-in for ops.rccl.GateComm on agents with synthetic GPUs (no RCCL)."""

    def __init__(self, devices: List[int]):
        self.devices = list(devices)

    def sweep(self, sizes, iters=10, warmup=3, dtype="f32", timeout_s=600.0, async_teardown=True):
        from ..ops.rccl import SweepResult

        n = len(sizes)
        return SweepResult(len(self.devices), dtype, list(sizes), [0.0] * n, [0.0] * n, [0.0] * n, [0] * n, 0.0,
                           {"simulated": 1.0})

    def abort(self) -> None:
        pass

    def cancel(self) -> None:
        pass


class GateAborted(RuntimeError):
    """The gate was aborted (``/v1/rccl-abort``) before or while this request ran."""


class _Reserved:
    """A gate request's slot in ``_sweeping`` while its communicator is being created: an
    abort that lands in that window marks it, and the request then releases what it made."""

    devices: List[int] = []

    def __init__(self) -> None:
        self.canceled = False

    def cancel(self) -> None:
        self.canceled = True


class AgentGateMixin:
    """Mixin of :class:`~.agent.NodeAgent`: this node's ranks of cluster RCCL gates.

    Abort ordering.  ``ClusterGate._gate_all`` (readiness/gate.py) sends ``/v1/rccl-abort``
    to the other members while their gate requests are in flight, so an abort can land
    before a member's request, between its take of the pending communicator and its sweep,
    or during the sweep.  Every transition of a uid (pending -> sweeping, aborted) happens
    under one hold of ``_gate_mu``, and an aborted uid is remembered for ``ABORTED_TTL_S``:
    a later prepare or gate request for it fails at once instead of starting a fresh init
    that would wait out its whole timeout for peers that are gone."""

    # --- RCCL gate (this node's ranks) ---------------------------------------------------------
    # Gate communicators pending by uid: started by /v1/rccl-prepare, consumed by
    # /v1/rccl-gate, released by /v1/rccl-abort, stop(), or expiry.
    GATE_TTL_S = 900.0
    ABORTED_TTL_S = 900.0

    def _is_aborted(self, uid: bytes) -> bool:
        """(Caller holds ``_gate_mu``.)  ``uid`` was aborted recently; expires old entries."""
        aborted = self.__dict__.setdefault("_aborted_uids", {})
        now = time.time()
        for k in [k for k, t in aborted.items() if now - t > self.ABORTED_TTL_S]:
            del aborted[k]
        return uid in aborted

    # the longest a burn-in child keeps the HBM it tested for this agent's RCCL inits
    RELEASE_HOLD_S = 20.0

    def _await_rccl_inits(self) -> None:
        """Return once no RCCL communicator init of this agent is running and the running
        plan's link matrix is measured, or after :attr:`RELEASE_HOLD_S`
        (``ops/probe.py:set_release_hold``: a burn-in child's ~300 GB release, which the
        driver clears for seconds, would hold up the device-code load of an init still
        running, and run beside the peer reads of the link check)."""
        from ..ops import rccl

        deadline = time.monotonic() + self.RELEASE_HOLD_S
        release_now = self._release_event()
        while ((rccl.inits_running() > 0 or rccl.preloads_running() > 0 or getattr(self, "_links_pending", False))
               and time.monotonic() < deadline and not release_now.is_set()):
            time.sleep(0.005)

    # --- a gate communicator that ran out of HBM beside held burn-in spans ----------------------
    # A full burn-in's span leaves ``probe.SPAN_HEADROOM`` of each GPU free, and the gate's
    # communicator init allocates into it while the span is held (the hold above).  On a node
    # of 8 xGMI peers that headroom was a constant nobody had measured, so an init can run
    # out of memory there.  Then every held span is released and the init is retried once
    # (``gate_retry: oom`` in the answer), and the footprint each successful init measured
    # (this process's VRAM around it, or the device's from a window without burn-in
    # activity: ``tk_rccl_probe.hip:proc_vram``) sets the node's headroom from then on
    # (:meth:`_note_gate_footprint`), the constant staying the floor; an out-of-memory init
    # doubles it (:meth:`_note_gate_oom`).

    FOOTPRINT_FILE = "/etc/triton-kubernetes/gate-footprint.json"
    HEADROOM_MARGIN = 1.25  # measured footprint x this, plus the floor's first GiB
    # a larger "footprint" is not a communicator's: 8 ranks of RCCL on MI355X take ~1 GiB per
    # GPU (profiles/round6/gate_footprint.jsonl: 0.8 GiB for one, device code included)
    FOOTPRINT_MAX_MIB = 32 * 1024

    def _release_event(self):
        ev = self.__dict__.get("_release_now")
        if ev is None:
            import threading

            ev = self.__dict__.setdefault("_release_now", threading.Event())
        return ev

    def _release_held_spans(self) -> float:
        """Every burn-in child still holding the HBM it tested releases it now; returns once
        they have exited (ms).  The driver clears the release afterwards, which the retried
        init's allocations wait for."""
        from ..ops import probe

        t0 = time.perf_counter()
        ev = self._release_event()
        ev.set()
        try:
            probe.wait_frees()
        finally:
            ev.clear()
        return round((time.perf_counter() - t0) * 1e3, 1)

    def _new_gate(self, uid: bytes, world: int, rank_base: int, devices: List[int], **kw: Any) -> Any:
        """A gate communicator (its init starts now), with the agent's burn-in activity at
        its start (``window``: a device-wide footprint is kept only for a quiet window)."""
        from ..ops import probe, rccl

        window = probe.activity()
        gate = rccl.GateComm(uid, world, rank_base, devices, **kw)
        gate.window = window
        return gate

    def _sweep_oom_retry(self, first, remake, sweep):
        """``sweep(first())``; when that fails because the communicator's init ran out of
        device memory (``ops/rccl.is_oom_error``), release the held spans and run
        ``sweep(remake())`` once.  Returns ``(result, retry detail or None)``."""
        from ..ops import rccl

        try:
            return sweep(first()), None
        except rccl.RCCLError as exc:
            if not rccl.is_oom_error(str(exc)):
                raise
            first_error = str(exc)
        self._note_gate_oom(len(self.devices))
        with span("node.rccl_gate_retry", node=self.name, why="oom"):
            released_ms = self._release_held_spans()
            try:
                res = sweep(remake())
            except rccl.RCCLError as exc:
                # once only: the cluster gate sees it was retried (RETRIED_MARK) and does not
                raise rccl.RCCLError(f"{exc} {rccl.OOM_RETRIED_MARK}") from exc
        return res, {"gate_retry": "oom", "first_error": first_error[:400], "spans_released_ms": released_ms}

    def _note_gate_footprint(self, ndev: int, phase_ms: Dict[str, float], window: Any = None) -> bool:
        """Keep the largest per-GPU footprint a gate communicator over ``ndev`` of this node's
        GPUs measured (``footprint_total_mib``: the communicator and its sweep buffers), and
        size the burn-in span's headroom from it (never below the constant floor).

        A device-wide measurement (``footprint_kind`` 2: no per-process accounting here)
        counts everything allocated on the GPU meanwhile; it is kept only when none of this
        agent's burn-ins started, ran or was alive from the init's start (``window``) to now.
        Returns whether it was kept (``footprint_kept`` in ``phase_ms``)."""
        from ..ops import probe

        mib = float(phase_ms.get("footprint_total_mib") or 0.0)
        kept = 0.0 < mib <= self.FOOTPRINT_MAX_MIB  # else not measured here (-1), or not a communicator's
        if kept and int(phase_ms.get("footprint_kind") or 0) != 1:
            kept = window is not None and window[1] == 0 and probe.activity() == window
        phase_ms["footprint_kept"] = 1.0 if kept else 0.0  # the answer says whether it counted
        if kept:
            self._keep_footprint(str(int(ndev)), mib)
        return kept

    def _note_gate_oom(self, ndev: int) -> None:
        """An init ran out of HBM beside held spans: the next burn-in of this node leaves
        twice the headroom it left (at most :attr:`FOOTPRINT_MAX_MIB`), whatever is measured."""
        from ..ops import probe

        held = max(probe.SPAN_HEADROOM, self.span_headroom(ndev))  # what the spans left free
        self._keep_footprint(f"oom:{int(ndev)}", min(self.FOOTPRINT_MAX_MIB, 2.0 * held / (1 << 20)))

    def _keep_footprint(self, key: str, mib: float) -> None:
        import json

        from ..ops import probe

        with self._gate_mu:
            fp = self.__dict__.setdefault("_gate_footprints", self._load_gate_footprints())
            if mib <= float(fp.get(key, 0.0)):
                return
            fp[key] = round(mib, 1)
            doc = dict(fp)
        # kept on the node (exec mode), or under a sim agent's own root; a sim agent with root
        # / models no host and never writes to the machine it runs on
        if self.mode == "exec" or self._host_is_sandbox():
            try:
                self.write_file(self.FOOTPRINT_FILE, json.dumps(doc, sort_keys=True))
            except Exception:  # noqa: BLE001 - a read-only root only loses the memory of it
                pass
        probe.set_span_headroom(self.span_headroom(len(self.devices)))

    def _load_gate_footprints(self) -> Dict[str, float]:
        import json

        try:
            with open(self.path(self.FOOTPRINT_FILE), "r", encoding="utf-8") as fh:
                doc = json.load(fh)
            return {str(k): float(v) for k, v in doc.items()} if isinstance(doc, dict) else {}
        except (OSError, ValueError, TypeError):
            return {}

    def span_headroom(self, ndev: int) -> int:
        """HBM a full burn-in span leaves free on each GPU of this node: the constant floor
        (4 GiB + 512 MiB per further GPU), the largest gate footprint this node has measured
        for ``ndev`` GPUs (x :attr:`HEADROOM_MARGIN`, plus 1 GiB), or twice the headroom an
        init ran out of memory beside, whichever is most."""
        floor = (4 << 30) + (512 << 20) * max(0, ndev - 1)
        fp = self.__dict__.get("_gate_footprints")
        if fp is None:
            fp = self.__dict__.setdefault("_gate_footprints", self._load_gate_footprints())
        mib = float(fp.get(str(int(ndev)), 0.0))
        bumped = int(float(fp.get(f"oom:{int(ndev)}", 0.0)) * (1 << 20))  # after an out-of-memory init
        return max(floor, int(mib * self.HEADROOM_MARGIN * (1 << 20)) + (1 << 30), bumped)

    def _gate_devices(self, ndev: int) -> List[int]:
        devs = self.devices or [0]
        if ndev < 1 or ndev > len(devs):
            raise ValueError(f"gate wants {ndev} GPUs, agent has {len(devs)}")
        return devs[:ndev]

    def _expire_gates(self) -> None:
        now = time.time()
        with self._gate_mu:
            stale = [k for k, e in self._gates.items() if now - e[1] > self.GATE_TTL_S]
            gates = [self._gates.pop(k)[0] for k in stale]
            for k in [k for k, e in self._gate_results.items() if now - e[1] > self.GATE_TTL_S]:
                del self._gate_results[k]
        for g in gates:
            g.abort()

    @property
    def _sim_gate(self) -> bool:
        """Synthetic GPUs without the RCCL ABI: the gate is simulated (no library call)."""
        return self.topology_override is not None and self.gate_backend != "rccl"

    def _make_uid(self) -> bytes:
        if self._sim_gate:  # synthetic GPUs (tests / dry runs)
            return secrets.token_bytes(128)
        from ..ops import rccl

        self._used_rccl = True
        return rccl.unique_id()

    def _refill_uid(self) -> None:
        uid = self._make_uid()
        with self._uid_mu:
            if self._spare_uid is None:
                self._spare_uid = uid

    def new_uid(self) -> bytes:
        """A fresh RCCL unique id (a bootstrap rendezvous address, specific to no cluster):
        the spare if one is ready, otherwise made now; either way the next spare is made on
        the agent's pool, off this request."""
        with self._uid_mu:
            uid, self._spare_uid = self._spare_uid, None
        if uid is None:
            uid = self._make_uid()
        try:
            self._pool.submit(self._refill_uid)
        except RuntimeError:  # pool shut down: the agent is stopping
            pass
        return uid

    def rccl_prepare(self, uid: Optional[bytes], world: int, rank_base: int, ndev: int = 1,
                     max_bytes: int = 0, sizes: Optional[List[int]] = None) -> Dict[str, Any]:
        """Start this node's share of a cluster communicator (non-blocking init; with
        ``max_bytes`` the init thread also allocates the sweep buffers).  ``uid`` None: this
        node hosts the rendezvous — it takes a new unique id and returns it for the others.
        ``sizes``: the gate's message sizes, so a node that is the whole gate can sweep them
        in its ``rccl_local`` step (:meth:`_take_node_gate`)."""
        devs = self._gate_devices(ndev)
        self._expire_gates()
        if uid is None:
            uid = self.new_uid()
        with self._gate_mu:
            if self._is_aborted(uid):
                raise GateAborted("gate aborted before this node's prepare")
        with span("node.rccl_prepare", node=self.name, rank_base=rank_base, world=world):
            if self._sim_gate:  # synthetic GPUs (tests / dry runs)
                gate: Any = _SimGate(devs)
            else:
                from ..ops import rccl

                self._used_rccl = True
                gate = self._new_gate(uid, world, rank_base, devs, blocking=False, prealloc_bytes=max_bytes)
        with self._gate_mu:
            aborted = self._is_aborted(uid)  # an abort that landed during the init's start
            old = self._gates.pop(uid, None)
            if not aborted:
                self._gates[uid] = (gate, time.time(), {"world": world, "rank_base": rank_base,
                                                        "sizes": [int(x) for x in (sizes or [])]})
        if old is not None:
            old[0].abort()
        if aborted:
            gate.abort()
            raise GateAborted("gate aborted during this node's prepare")
        return {"ok": True, "ranks": list(range(rank_base, rank_base + len(devs))), "devices": devs,
                "uid": base64.b64encode(uid).decode()}

    def rccl_abort(self, uid: bytes) -> Dict[str, Any]:
        """Release this node's ranks of gate ``uid``: a pending communicator is aborted, and a
        sweep waiting for peers is canceled (it fails at once instead of at its timeout:
        another member of the gate failed)."""
        with self._gate_mu:
            self._is_aborted(uid)
            self.__dict__.setdefault("_aborted_uids", {})[uid] = time.time()
            entry = self._gates.pop(uid, None)
            done = self._gate_results.pop(uid, None)
            running = self._sweeping.get(uid)
        if entry is not None:
            entry[0].abort()
        if running is not None:
            running.cancel()
        return {"ok": True, "aborted": entry is not None or done is not None, "canceled": running is not None}

    def _take_node_gate(self) -> Optional[Tuple[bytes, Any, Dict[str, Any]]]:
        """A pending gate communicator that spans exactly this node's GPUs (a one-node
        cluster: world == ndev, every rank here), taken out of the pending set.

        Its all-reduce over the node's GPUs IS the node-level RCCL check, so ``rccl_local``
        sweeps it instead of initialising a second communicator over the same GPUs on the
        bring-up path, and the cluster gate later answers from that sweep."""
        devs = list(self.devices)
        with self._gate_mu:
            for uid, (gate, _, meta) in list(self._gates.items()):
                if (meta.get("world") == len(devs) and meta.get("rank_base") == 0
                        and list(getattr(gate, "devices", [])) == devs):
                    del self._gates[uid]
                    return uid, gate, meta
        return None

    def rccl_gate(self, rank: int, world: int, uid: bytes, sizes: List[int], iters: int = 10,
                  ndev: int = 1, timeout_s: float = 600.0, release_holds: bool = False) -> Dict[str, Any]:
        """Run this node's ranks ``rank .. rank+ndev-1`` of the cluster gate: the pending
        communicator from rccl_prepare when there is one, else a fresh init.
        ``release_holds``: the cluster gate's retry after a member's init ran out of device
        memory -- the burn-in spans this node still holds are released first."""
        key = uid  # the request's uid: /v1/rccl-abort names this one
        with self._gate_mu:
            if self._is_aborted(key):
                raise GateAborted("gate aborted before this node's sweep")
            entry = self._gates.pop(uid, None)
            done = self._gate_results.pop(uid, None)
            # registered for cancel in the same hold that took it: no window in which an abort
            # finds the gate neither pending nor sweeping
            self._sweeping[key] = entry[0] if entry is not None else _Reserved()
        if done is not None:
            with self._gate_mu:
                self._sweeping.pop(key, None)
            res = done[0]
            if set(sizes) <= set(res.sizes):  # the rccl_local step swept this communicator
                idx = [res.sizes.index(x) for x in sizes]
                pick = lambda xs: [xs[i] for i in idx]  # noqa: E731
                from ..ops.rccl import SweepResult

                sub = SweepResult(res.world, res.dtype, list(sizes), pick(res.time_us), pick(res.algbw_gbps),
                                  pick(res.busbw_gbps), pick(res.errors), res.init_ms, dict(res.phase_ms))
                with span("node.rccl_gate", node=self.name, rank=rank, world=world, pipelined=True,
                          shared_with="rccl_local"):
                    out = sub.to_json()
                out.update(pipelined=True, shared_with="rccl_local",
                           ranks=list(range(rank, rank + len(self._gate_devices(ndev)))))
                if len(done) > 2 and done[2]:
                    out.update(done[2])  # the rccl_local step's retry, reported with the gate
                return out
            # sizes the local sweep did not cover: the node is the whole gate, so a fresh
            # communicator under a new id (every rank is here) measures them
            uid = self._make_uid()
        pipelined = entry is not None
        retry: Optional[Dict[str, Any]] = None
        with span("node.rccl_gate", node=self.name, rank=rank, world=world, pipelined=pipelined):
            try:
                if release_holds:
                    # the cluster gate's retry after a member's init ran out of device memory:
                    # this node's held spans go before its communicator allocates
                    retry = {"gate_retry": "oom", "spans_released_ms": self._release_held_spans()}
                if entry is not None:
                    gate = entry[0]
                else:
                    if self._sim_gate:
                        gate = _SimGate(self._gate_devices(ndev))
                    else:
                        from ..ops import rccl

                        self._used_rccl = True
                        gate = self._new_gate(uid, world, rank, self._gate_devices(ndev), blocking=False)
                    with self._gate_mu:
                        slot = self._sweeping.get(key)
                        canceled = isinstance(slot, _Reserved) and slot.canceled
                        if not canceled:
                            self._sweeping[key] = gate
                    if canceled:  # aborted while the communicator was being created
                        gate.abort()
                        raise GateAborted("gate aborted while this node's communicator started")
                # the communicator teardown is not part of the readiness answer: it is
                # joined in stop() (or by the next process-exit drain), not here.  A node that
                # is the whole gate retries an init that ran out of memory by itself (every
                # rank is here); a member of a larger gate reports it, and the cluster gate
                # retries every member under a new id (readiness/gate.py)
                first_gate = gate

                def remake():
                    nonlocal gate
                    from ..ops import rccl

                    fresh = self._new_gate(self._make_uid(), world, 0, list(first_gate.devices), blocking=False)
                    with self._gate_mu:
                        canceled = self._is_aborted(key)  # an abort during the spans' release
                        if not canceled:
                            self._sweeping[key] = fresh
                    if canceled:
                        fresh.abort()
                        raise GateAborted("gate aborted while this node's communicator restarted")
                    gate = fresh
                    return fresh

                def sweep(g):
                    return g.sweep(sizes, iters=iters, warmup=2, async_teardown=True, timeout_s=timeout_s)

                if world == len(gate.devices) and rank == 0 and not self._sim_gate and retry is None:
                    res, retry = self._sweep_oom_retry(lambda: first_gate, remake, sweep)
                else:
                    res = sweep(gate)
            finally:
                with self._gate_mu:
                    self._sweeping.pop(key, None)
        self._note_gate_footprint(len(gate.devices), res.phase_ms, getattr(gate, "window", None))
        out = res.to_json()
        out["pipelined"] = pipelined
        out["ranks"] = list(range(rank, rank + len(gate.devices)))
        if retry:
            out.update(retry)
        return out


__all__ = ["AgentGateMixin", "GateAborted"]
