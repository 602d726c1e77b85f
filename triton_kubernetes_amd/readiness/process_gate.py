"""Cluster-wide RCCL gate for MI355X nodes without a node agent (SSH / Terraform delivery).

Agent hosts hold their ranks in a long-lived process (``gate.py``).  Nodes brought up over
SSH -- by the DirectExecutor or by the ``bare-metal-mi355x-rancher-k8s-host`` Terraform
module -- have the native tools installed under ``/opt/triton-kubernetes/bin`` instead, so
the gate runs one ``rccl-ready --cluster`` process per node over the host transport:

1. node 0 starts with ``--uid-out``: it makes the ``ncclUniqueId`` (its bootstrap root
   listens in that process), prints it as the first stdout line, then joins as ranks
   ``0 .. n0-1``;
2. as soon as that line arrives, every other node starts with ``--uid <hex>`` and its
   rank base, concurrently;
3. every process runs the same verified all-reduce sweep as the agents' gate (1 MiB and
   the configured largest size, warmup 2) over one communicator spanning every GPU of
   the cluster, prints one JSON line and exits; non-zero on a verification error or a
   ``--min-busbw`` miss.

Each node's ``/etc/rccl/rccl.env`` (discovered RDMA ports, per-node overrides, written by
the bootstrap) is sourced first, so the gate runs with the environment GPU pods get.
A node that opted in to the verified single-target RCCL (``rccl-ready-slim`` present,
``terraform/scripts.py``) runs the tool through that wrapper.

A deadline bounds the whole gate; on expiry or the first failure every process is killed
-- on the node too: the tool runs under a watchdog that reads the channel's stdin, which
stays open while the gate holds it; when the gate ends (or its ``ssh`` client is killed,
which closes the channel: ``ssh`` without a pty sends the remote side no SIGHUP) the
watchdog sees EOF and kills the ranks, so an aborted gate never leaves a node's GPUs held
by an orphaned ``rccl-ready`` blocked in communicator init.  The tool's own timeout is the
init budget (``INIT_TIMEOUT_S``), not the whole readiness budget.

A cluster that mixes both kinds of MI355X nodes gets ONE communicator too: agent hosts
(``agent+URL`` addresses) join through their API (``/v1/rccl-prepare`` with the unique id,
then ``/v1/rccl-gate``), process hosts through ``rccl-ready --cluster``; both run the same
sweep schedule, so their collectives match.  The id travels as base64 to agents and as hex
to processes; whichever kind the first node is, it hosts the rendezvous.
"""

import base64
import concurrent.futures as cf
import json
import os
import selectors
import shlex
import time
from typing import Any, Dict, List, Optional, Sequence

from ..errors import TKError
from ..node.plan import TOOLS_DIR
from ..parallel.transport import HostRef
from ..utils.trace import span

ENV_FILE = "/etc/rccl/rccl.env"
INIT_TIMEOUT_S = 300.0  # a node's rccl-ready gives up on communicator init after this


def gate_script(tools_dir: str, world: int, rank_base: int, ngpus: int, sizes: Sequence[int], iters: int,
                uid: Optional[str], min_busbw: float = 0.0, timeout_s: float = 600.0, env_file: str = ENV_FILE) -> str:
    args = ["--cluster", "--world", str(world), "--rank-base", str(rank_base),
            "--ngpus", str(ngpus), "--max-mib", str(max(1, max(sizes) >> 20)), "--iters", str(iters),
            "--timeout-s", str(int(max(1.0, min(timeout_s, INIT_TIMEOUT_S)))), "--min-busbw", str(min_busbw)]
    args += ["--uid", uid] if uid else ["--uid-out"]
    tool, slim = shlex.quote(os.path.join(tools_dir, "rccl-ready")), shlex.quote(os.path.join(tools_dir, "rccl-ready-slim"))
    return (f"set -a; [ -r {shlex.quote(env_file)} ] && . {shlex.quote(env_file)}; set +a; "
            f"t={tool}; [ -x {slim} ] && t={slim}; exec 3<&0; "
            f'"$t" {" ".join(shlex.quote(a) for a in args)} </dev/null & pid=$!; '
            # watchdog: the gate's end closes our stdin -> take the ranks down
            "( cat <&3 >/dev/null 2>&1; kill -TERM $pid 2>/dev/null; sleep 3; kill -KILL $pid 2>/dev/null ) "
            ">/dev/null 2>&1 & w=$!; "
            "exec 3<&-; wait $pid; rc=$?; kill $w 2>/dev/null; exit $rc")


class ProcessGate:
    def __init__(self, transport: Any, hosts: List[HostRef], ndevs: List[int], sizes: Sequence[int],
                 iters: int = 5, timeout: float = 600.0, tools_dir: str = TOOLS_DIR, min_busbw: float = 0.0,
                 env_file: str = ENV_FILE, agent_transport: Any = None):
        if not hosts or len(hosts) != len(ndevs):
            raise ValueError("a process gate needs one GPU count per host")
        if any(h.scheme == "agent" for h in hosts) and agent_transport is None:
            raise ValueError("agent hosts in a process gate need an agent transport")
        self.agent_transport = agent_transport
        self.transport, self.hosts, self.ndevs = transport, list(hosts), [int(n) for n in ndevs]
        self.world = sum(self.ndevs)
        self.sizes, self.iters, self.timeout = list(sizes), iters, timeout
        self.tools_dir, self.min_busbw, self.env_file = tools_dir, min_busbw, env_file
        self.bases = [sum(self.ndevs[:i]) for i in range(len(self.ndevs))]
        self._pending = ""

    def _script(self, i: int, uid: Optional[str]) -> str:
        return gate_script(self.tools_dir, self.world, self.bases[i], self.ndevs[i], self.sizes, self.iters, uid,
                           self.min_busbw, self.timeout, self.env_file)

    def _is_agent(self, i: int) -> bool:
        return self.hosts[i].scheme == "agent"

    def _agent_prepare(self, i: int, uid_b64: Optional[str]) -> str:
        body = {"world": self.world, "rank_base": self.bases[i], "ndev": self.ndevs[i], "max_bytes": max(self.sizes)}
        if uid_b64:
            body["uid"] = uid_b64
        return self.agent_transport.post(self.hosts[i], "/v1/rccl-prepare", body)["uid"]

    def _agent_gate(self, i: int, uid_b64: str) -> Dict[str, Any]:
        res = self.agent_transport.post(self.hosts[i], "/v1/rccl-gate", {
            "uid": uid_b64, "rank": self.bases[i], "world": self.world, "ndev": self.ndevs[i],
            "sizes": self.sizes, "iters": self.iters})
        res["results"] = [{"bytes": b, "busbw_gbps": bw, "errors": e} for b, bw, e in
                          zip(res.get("sizes", []), res.get("busbw_gbps", []), res.get("errors", []))]
        return res

    def run(self) -> Dict[str, Any]:
        deadline = time.monotonic() + self.timeout
        procs: Dict[int, Any] = {}
        futs: Dict[int, cf.Future] = {}
        outs: List[str] = [""] * len(self.hosts)
        errs: List[str] = [""] * len(self.hosts)
        sel = selectors.DefaultSelector()
        pool = cf.ThreadPoolExecutor(max_workers=max(1, 2 * sum(self._is_agent(i) for i in range(len(self.hosts)))),
                                     thread_name_prefix="tk-pgate")
        uid_b64 = None
        ok_run = False
        try:
            with span("gate.process", world=self.world, nodes=len(self.hosts)):
                # 1. the first node hosts the rendezvous
                if self._is_agent(0):
                    uid_b64 = self._agent_prepare(0, None)
                    uid = base64.b64decode(uid_b64).hex()
                else:
                    procs[0] = self.transport.spawn(self.hosts[0], self._script(0, None))
                    uid = self._read_uid(procs[0], deadline)
                    uid_b64 = base64.b64encode(bytes.fromhex(uid)).decode()
                    outs[0] += self._pending
                # 2. everyone else joins with it
                prep = {i: pool.submit(self._agent_prepare, i, uid_b64)
                        for i in range(1, len(self.hosts)) if self._is_agent(i)}
                for i in range(1, len(self.hosts)):
                    if not self._is_agent(i):
                        procs[i] = self.transport.spawn(self.hosts[i], self._script(i, uid))
                for f in prep.values():
                    f.result(timeout=max(1.0, deadline - time.monotonic()))
                # 3. agents run their ranks of the sweep while the processes run theirs
                futs = {i: pool.submit(self._agent_gate, i, uid_b64)
                        for i in range(len(self.hosts)) if self._is_agent(i)}
                # drain every process's pipes until all exit (or the deadline / a failure);
                # raw reads, so a partial line can never block the loop past the deadline
                for i, p in procs.items():
                    sel.register(p.stdout.fileno(), selectors.EVENT_READ, (i, "out"))
                    sel.register(p.stderr.fileno(), selectors.EVENT_READ, (i, "err"))
                open_pipes = 2 * len(procs)
                while open_pipes or any(not f.done() for f in futs.values()):
                    left = deadline - time.monotonic()
                    if left <= 0:
                        raise TKError(f"RCCL process gate timed out after {self.timeout:.0f}s")
                    if open_pipes:
                        ready = sel.select(timeout=min(left, 0.2))
                    else:
                        ready = []
                        cf.wait(list(futs.values()), timeout=min(left, 0.2), return_when=cf.FIRST_COMPLETED)
                    for key, _ in ready:
                        i, which = key.data
                        chunk = os.read(key.fd, 65536).decode(errors="replace")
                        if not chunk:
                            sel.unregister(key.fd)
                            open_pipes -= 1
                            continue
                        if which == "out":
                            outs[i] += chunk
                        else:
                            errs[i] += chunk
                    failed = [i for i, p in procs.items() if p.poll() not in (None, 0)]
                    if failed and (any(p.poll() is None for p in procs.values())
                                   or any(not f.done() for f in futs.values())):
                        # one node failed: the others would wait for it forever
                        raise TKError(f"RCCL process gate: node {self.hosts[failed[0]].address} exited "
                                      f"{procs[failed[0]].returncode}: {errs[failed[0]][-400:]}")
                    bad = [i for i, f in futs.items() if f.done() and f.exception() is not None]
                    if bad:
                        raise TKError(f"RCCL process gate: agent {self.hosts[bad[0]].address} failed: "
                                      f"{futs[bad[0]].exception()}")
                for p in procs.values():
                    p.wait(timeout=max(1.0, deadline - time.monotonic()))
                ok_run = True
        finally:
            sel.close()
            for p in procs.values():
                if p.poll() is None:
                    p.kill()
                    p.wait()
                if p.stdin is not None:  # EOF to the node-side watchdog (see module doc)
                    try:
                        p.stdin.close()
                    except OSError:
                        pass
            if not ok_run and uid_b64 is not None:
                for i in range(len(self.hosts)):  # release agents' pending communicators
                    if self._is_agent(i):
                        try:
                            self.agent_transport.post(self.hosts[i], "/v1/rccl-abort", {"uid": uid_b64})
                        except Exception:  # noqa: BLE001 - best effort; agents expire stale gates
                            pass
            pool.shutdown(wait=False, cancel_futures=True)
        ranks = []
        for i in range(len(self.hosts)):
            if self._is_agent(i):
                doc = dict(futs[i].result())
                doc.update(host=self.hosts[i].address, rc=0, rank_base=self.bases[i], kind="agent")
            else:
                p = procs[i]
                line = next((ln for ln in reversed(outs[i].splitlines()) if ln.startswith("{") and '"uid"' not in ln),
                            "")
                doc = json.loads(line) if line else {"ok": False}
                doc.update(host=self.hosts[i].address, rc=p.returncode, rank_base=self.bases[i], kind="process")
                if p.returncode:
                    doc["stderr"] = errs[i][-400:]
            ranks.append(doc)
        busbw = [max((r.get("busbw_gbps", 0.0) for r in d.get("results", [])), default=0.0) for d in ranks]
        ok = all(d.get("ok") and d["rc"] == 0 for d in ranks)
        kinds = {d["kind"] for d in ranks}
        return {"ok": ok, "world": self.world, "nodes": len(self.hosts),
                "mode": "process" if kinds == {"process"} else "mixed", "pipelined": False,
                "min_peak_busbw_gbps": min(busbw) if busbw else 0.0, "ranks": ranks}

    def _read_uid(self, proc: Any, deadline: float) -> str:
        """Rank 0's first stdout line; what follows it stays in ``self._pending``."""
        sel = selectors.DefaultSelector()
        fd = proc.stdout.fileno()
        sel.register(fd, selectors.EVENT_READ)
        buf = ""
        try:
            while True:
                left = deadline - time.monotonic()
                if left <= 0:
                    raise TKError("RCCL process gate: no unique id from the first node")
                if not sel.select(timeout=min(left, 1.0)):
                    if proc.poll() is not None:
                        raise TKError(f"RCCL process gate: first node exited {proc.returncode}: "
                                      f"{proc.stderr.read()[-400:]}")
                    continue
                chunk = os.read(fd, 65536).decode(errors="replace")
                if not chunk:
                    raise TKError(f"RCCL process gate: first node closed its output "
                                  f"(exit {proc.wait()}): {proc.stderr.read()[-400:]}")
                buf += chunk
                while "\n" in buf:
                    line, buf = buf.split("\n", 1)
                    if line.startswith("{") and '"uid"' in line:
                        self._pending = buf
                        return json.loads(line)["uid"]
        finally:
            sel.close()


__all__ = ["ProcessGate", "gate_script"]
