#!/usr/bin/env python3
"""Stand-in for ``rccl-ready --cluster`` on CPU (tests only).

Speaks the same protocol as the native tool: with ``--uid-out`` it prints
``{"uid": <256 hex>}`` first (the hex encodes a TCP port this process listens on, like
RCCL's bootstrap root), then waits until processes holding the remaining
``world - ngpus`` ranks have connected; with ``--uid`` it connects to that port and
waits (an id that does not start with ``fa4e`` came from a simulated agent: no rendezvous).
Every process then prints one result line.  ``FAKE_RCCL_FAIL_BASE=<rank base>``
makes that process fail at once; ``FAKE_RCCL_NO_UID=1`` makes the root never print its id.
``FAKE_RCCL_PIDDIR=<dir>``: each process records its pid there.
The environment the gate script sourced is echoed back (``env``) so tests can check it.
"""

import argparse
import json
import os
import socket
import sys
import time


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cluster", action="store_true")
    ap.add_argument("--world", type=int)
    ap.add_argument("--rank-base", type=int)
    ap.add_argument("--ngpus", type=int)
    ap.add_argument("--uid")
    ap.add_argument("--uid-out", action="store_true")
    ap.add_argument("--max-mib", type=int)
    ap.add_argument("--iters", type=int)
    ap.add_argument("--timeout-s", type=float)
    ap.add_argument("--min-busbw", type=float)
    a = ap.parse_args()
    piddir = os.environ.get("FAKE_RCCL_PIDDIR")
    if piddir:  # tests check that an aborted gate leaves no rank process behind
        with open(os.path.join(piddir, f"{os.getpid()}.pid"), "w") as fh:
            fh.write(str(a.rank_base))
    if os.environ.get("FAKE_RCCL_FAIL_BASE") == str(a.rank_base):
        print('{"error":"injected failure"}', file=sys.stderr)
        return 2
    if a.uid_out:
        if os.environ.get("FAKE_RCCL_NO_UID") == "1":
            time.sleep(3600)
        srv = socket.socket()
        srv.bind(("127.0.0.1", 0))
        srv.listen(64)
        port = srv.getsockname()[1]
        print(json.dumps({"uid": ("fa4e" + f"{port:08x}").ljust(256, "0")}), flush=True)
        # ranks held by agents (FAKE_RCCL_AGENT_RANKS) do not connect to this stand-in
        have, conns = a.ngpus + int(os.environ.get("FAKE_RCCL_AGENT_RANKS", "0")), []
        while have < a.world:
            c, _ = srv.accept()
            have += int(c.recv(16).decode())
            conns.append(c)
        for c in conns:
            c.sendall(b"go")
            c.close()
    elif a.uid.startswith("fa4e"):
        port = int(a.uid[4:12], 16)
        c = socket.create_connection(("127.0.0.1", port), timeout=a.timeout_s)
        c.sendall(str(a.ngpus).encode())
        assert c.recv(2) == b"go"
        c.close()
    # else: the id came from an agent (a sim gate in tests): nothing to rendezvous with
    sizes = [1 << 20, a.max_mib << 20]
    print(json.dumps({"world": a.world, "rank_base": a.rank_base, "ngpus": a.ngpus, "init_ms": 1.0,
                      "results": [{"bytes": b, "busbw_gbps": 100.0 + a.rank_base, "errors": 0} for b in sizes],
                      "ok": True, "env": os.environ.get("NCCL_IB_HCA", "")}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
