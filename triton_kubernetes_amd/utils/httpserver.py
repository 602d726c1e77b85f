"""The threaded HTTP server every in-process endpoint uses (node agent, webhook, fakes).

``socketserver`` listens with a backlog of 5.  A create fans requests out to every
node at once (host modules, gate prepare, readiness polls), so a burst of connects to
one endpoint overflows that queue; the kernel drops the extra SYNs and each client
retransmits after 1 s (then 3 s).  At 32 sim workers that showed up as a 1.2 s
``module.host`` instead of ~0.1 s (``scripts/control_plane_scale.py``).  Go's
``net/http`` -- what a real Rancher server listens with -- uses the system's
``somaxconn``; so does this, capped by the kernel as usual.
"""

import http.server
import ssl
import sys

LISTEN_BACKLOG = 4096


class Server(http.server.ThreadingHTTPServer):
    request_queue_size = LISTEN_BACKLOG
    daemon_threads = True

    def handle_error(self, request, client_address):
        """A client that refused our certificate (or dropped the handshake) is that client's
        business: one line, not a traceback; anything else as ``socketserver`` reports it."""
        exc = sys.exc_info()[1]
        if isinstance(exc, (ssl.SSLError, ConnectionError, TimeoutError)):
            sys.stderr.write(f"{type(self).__name__}: TLS/connection from {client_address[0]}: {exc}\n")
            return
        super().handle_error(request, client_address)
