"""Listen backlog of the in-process HTTP endpoints (utils/httpserver.py).

With socketserver's backlog of 5, a burst of connects to an endpoint that is busy
overflows the accept queue and the kernel drops the extra SYNs (1 s client retransmit):
32 sim workers read a 1.2 s ``module.host`` instead of ~0.1 s."""

import http.server
import socket

from triton_kubernetes_amd.k8s import webhook
from triton_kubernetes_amd.utils.httpserver import LISTEN_BACKLOG, Server


def _connects_before_accept(server_cls, n: int = 24) -> int:
    """Connections the kernel completes while the server accepts none."""
    srv = server_cls(("127.0.0.1", 0), http.server.BaseHTTPRequestHandler)
    socks, ok = [], 0
    try:
        for _ in range(n):
            s = socket.socket()
            s.settimeout(0.1)
            try:
                s.connect(srv.server_address)
                ok += 1
            except OSError:
                pass
            socks.append(s)
    finally:
        for s in socks:
            s.close()
        srv.server_close()
    return ok


def test_burst_of_connects_is_queued_not_dropped():
    assert Server.request_queue_size == LISTEN_BACKLOG >= 1024
    assert webhook._Server.request_queue_size >= 1024
    assert _connects_before_accept(Server) == 24
    # the stdlib default the endpoints used before: the burst overflows its queue
    assert _connects_before_accept(http.server.ThreadingHTTPServer) < 24
