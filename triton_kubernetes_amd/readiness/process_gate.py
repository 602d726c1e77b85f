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
A deadline bounds the whole gate; on expiry or the first failure every process is killed.
"""

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


def gate_script(tools_dir: str, world: int, rank_base: int, ngpus: int, sizes: Sequence[int], iters: int,
                uid: Optional[str], min_busbw: float = 0.0, timeout_s: float = 600.0, env_file: str = ENV_FILE) -> str:
    argv = [os.path.join(tools_dir, "rccl-ready"), "--cluster", "--world", str(world), "--rank-base", str(rank_base),
            "--ngpus", str(ngpus), "--max-mib", str(max(1, max(sizes) >> 20)), "--iters", str(iters),
            "--timeout-s", str(int(timeout_s)), "--min-busbw", str(min_busbw)]
    argv += ["--uid", uid] if uid else ["--uid-out"]
    return (f"set -a; [ -r {shlex.quote(env_file)} ] && . {shlex.quote(env_file)}; set +a; "
            f"exec {' '.join(shlex.quote(a) for a in argv)}")


class ProcessGate:
    def __init__(self, transport: Any, hosts: List[HostRef], ndevs: List[int], sizes: Sequence[int],
                 iters: int = 5, timeout: float = 600.0, tools_dir: str = TOOLS_DIR, min_busbw: float = 0.0,
                 env_file: str = ENV_FILE):
        if not hosts or len(hosts) != len(ndevs):
            raise ValueError("a process gate needs one GPU count per host")
        self.transport, self.hosts, self.ndevs = transport, list(hosts), [int(n) for n in ndevs]
        self.world = sum(self.ndevs)
        self.sizes, self.iters, self.timeout = list(sizes), iters, timeout
        self.tools_dir, self.min_busbw, self.env_file = tools_dir, min_busbw, env_file
        self.bases = [sum(self.ndevs[:i]) for i in range(len(self.ndevs))]
        self._pending = ""

    def _script(self, i: int, uid: Optional[str]) -> str:
        return gate_script(self.tools_dir, self.world, self.bases[i], self.ndevs[i], self.sizes, self.iters, uid,
                           self.min_busbw, self.timeout, self.env_file)

    def run(self) -> Dict[str, Any]:
        deadline = time.monotonic() + self.timeout
        procs: List[Any] = []
        outs: List[str] = [""] * len(self.hosts)
        errs: List[str] = [""] * len(self.hosts)
        sel = selectors.DefaultSelector()
        try:
            with span("gate.process", world=self.world, nodes=len(self.hosts)):
                p0 = self.transport.spawn(self.hosts[0], self._script(0, None))
                procs.append(p0)
                uid = self._read_uid(p0, deadline)
                for i in range(1, len(self.hosts)):
                    procs.append(self.transport.spawn(self.hosts[i], self._script(i, uid)))
                # drain every process's pipes until all exit (or the deadline / a failure);
                # raw reads, so a partial line can never block the loop past the deadline
                outs[0] += self._pending
                for i, p in enumerate(procs):
                    sel.register(p.stdout.fileno(), selectors.EVENT_READ, (i, "out"))
                    sel.register(p.stderr.fileno(), selectors.EVENT_READ, (i, "err"))
                open_pipes = 2 * len(procs)
                while open_pipes:
                    left = deadline - time.monotonic()
                    if left <= 0:
                        raise TKError(f"RCCL process gate timed out after {self.timeout:.0f}s")
                    for key, _ in sel.select(timeout=min(left, 1.0)):
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
                    failed = [i for i, p in enumerate(procs) if p.poll() not in (None, 0)]
                    if failed and any(p.poll() is None for p in procs):
                        # one node failed: the others would wait for it forever
                        raise TKError(f"RCCL process gate: node {self.hosts[failed[0]].address} exited "
                                      f"{procs[failed[0]].returncode}: {errs[failed[0]][-400:]}")
                for p in procs:
                    p.wait(timeout=max(1.0, deadline - time.monotonic()))
        finally:
            sel.close()
            for p in procs:
                if p.poll() is None:
                    p.kill()
                    p.wait()
        ranks = []
        for i, p in enumerate(procs):
            line = next((ln for ln in reversed(outs[i].splitlines()) if ln.startswith("{") and '"uid"' not in ln), "")
            doc = json.loads(line) if line else {"ok": False}
            doc.update(host=self.hosts[i].address, rc=p.returncode, rank_base=self.bases[i])
            if p.returncode:
                doc["stderr"] = errs[i][-400:]
            ranks.append(doc)
        busbw = [max((r.get("busbw_gbps", 0.0) for r in d.get("results", [])), default=0.0) for d in ranks]
        ok = all(d.get("ok") and d["rc"] == 0 for d in ranks)
        return {"ok": ok, "world": self.world, "nodes": len(self.hosts), "mode": "process", "pipelined": False,
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
