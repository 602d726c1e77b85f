#!/usr/bin/env python3
"""CPU-only model of the intra-node topology-XML fusion RCCL runs inside every communicator
init (profiles/round1_rccl_init_breakdown.md): each of N local ranks allocates N x 102 MiB,
copies its own XML arena into its slot and ring-all-gathers the others over loopback TCP
sockets (RCCL's bootstrap transport).  It estimates what an N-GPU create adds to the RCCL
gate's init on this host; we cannot run RCCL with N > 1 ourselves (one GPU per box).

    python scripts/rccl_xml_allgather_model.py N
"""
import multiprocessing as mp
import socket
import sys
import threading
import time

SZ = 0x6630008  # RCCL's per-rank topology XML arena (102 MiB), profiles/round1_rccl_init_breakdown.md
def run(rank, n, base, q):
    buf = bytearray(SZ * n)  # calloc'd like RCCL's nLocalRanks x xmlMemSize
    mv = memoryview(buf)
    mv[rank*SZ:(rank+1)*SZ] = b"\x01" * SZ  # this rank's XML copy (the 15 ms memcpy)
    ls = socket.socket(); ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    ls.bind(("127.0.0.1", base + rank)); ls.listen(1)
    time.sleep(0.5)
    out = socket.create_connection(("127.0.0.1", base + (rank + 1) % n))
    inp, _ = ls.accept()
    q.put(("ready", rank))
    t0 = time.perf_counter()
    for s in range(n - 1):
        sb = (rank - s) % n; rb = (rank - s - 1) % n
        th = threading.Thread(target=out.sendall, args=(mv[sb*SZ:(sb+1)*SZ],)); th.start()
        got = 0
        while got < SZ:
            got += inp.recv_into(mv[rb*SZ+got:(rb+1)*SZ], SZ - got)
        th.join()
    q.put(("done", rank, time.perf_counter() - t0))
if __name__ == "__main__":
    n = int(sys.argv[1]); base = 29700 + n * 20
    q = mp.Queue(); ps = [mp.Process(target=run, args=(r, n, base, q)) for r in range(n)]
    t = time.perf_counter(); [p.start() for p in ps]
    res = [q.get() for _ in range(2 * n)]
    [p.join() for p in ps]
    print(n, "ranks: allgather max", round(max(r[2] for r in res if r[0] == "done") * 1e3, 1), "ms")
