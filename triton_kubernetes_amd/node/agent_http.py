"""The node agent's HTTP API and its authentication.

Off loopback the agent serves only TLS, with a certificate for the node's address signed
by its cluster manager's CA (the handshake runs on the connection's own thread, with a
deadline); plain HTTP binds loopback only.  Every request carries the node's own token
(``X-TK-Agent-Token``, derived per node from the manager secret).  The read-only
endpoints (``GET /metrics``, ``GET /v1/health``) also take the node's scrape token
(``security.metrics_token``: all Prometheus holds), as a Bearer.  An unauthorised POST is
answered and its connection closed (its body is never read).  A plan the node's
allow-list refuses is answered 403 before any step runs.

API (JSON): ``GET /v1/info``, ``GET /v1/health``, ``GET /metrics``, ``POST /v1/plan``,
``POST /v1/rccl-uid``, ``/v1/rccl-prepare``, ``/v1/rccl-gate``, ``/v1/rccl-abort``,
``POST /v1/cleanup``, ``POST /v1/shutdown``.  Once the agent stops, connections still
open are answered 503.
"""

import base64
import binascii
import hmac
import http.server
import json
import socket
import threading
import urllib.parse
from typing import Any

from ..utils.httpserver import Server as HTTPServer
from .agent_gate import GateAborted
from .plan import BootstrapPlan
from .security import is_loopback, metrics_token

MAX_BODY = 16 << 20  # bytes: the largest request body the agent reads


class _BadRequest(Exception):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


class AgentHTTPMixin:
    """Mixin of :class:`~.agent.NodeAgent`: the HTTP(S) server."""

    def serve(self, host: str = "127.0.0.1", port: int = 0, ssl_context: Any = None) -> str:
        """Serve the API; HTTPS with ``ssl_context`` (the node's certificate), plain HTTP
        only on a loopback address."""
        if ssl_context is None and not is_loopback(host):
            raise ValueError(f"refusing to serve plain HTTP on {host}: give the agent its TLS credentials "
                             "(node credentials) or use --insecure-local, which binds loopback only")
        agent = self
        self.warm_native()

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def setup(self):
                # TLS handshake here, on this connection's own thread with a deadline: a
                # client that connects and stalls cannot block the accept loop
                if ssl_context is not None:
                    self.request.settimeout(10.0)
                    self.request.do_handshake()
                    self.request.settimeout(None)
                super().setup()
                # one request/response per segment: no Nagle/delayed-ACK stalls on keep-alive
                self.request.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

            def log_message(self, *args):
                pass

            def _reply(self, code: int, obj: Any):
                body = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                if self.close_connection:  # the client must not reuse this connection
                    self.send_header("Connection", "close")
                self.end_headers()
                self.wfile.write(body)

            def _body(self):
                """The request's JSON object.  A length that is not a count, or past
                :data:`MAX_BODY` (a plan is a few KiB), is refused before anything is read."""
                raw = self.headers.get("Content-Length") or "0"
                if not raw.isdigit():
                    raise _BadRequest(400, "Content-Length must be a byte count")
                n = int(raw)
                if n > MAX_BODY:
                    raise _BadRequest(413, f"request body over {MAX_BODY} bytes")
                doc = json.loads(self.rfile.read(n) or b"{}") if n else {}
                if not isinstance(doc, dict):
                    raise _BadRequest(400, "the request body must be a JSON object")
                return doc

            def _gone(self) -> bool:
                """The agent stopped: a keep-alive connection accepted before is not served."""
                if agent._stopped:
                    self.close_connection = True
                    self._reply(503, {"error": "agent stopped"})
                return agent._stopped

            def _auth(self, read_only: bool = False) -> bool:
                """The node's agent token; for the read-only endpoints (``read_only``) also its
                scrape token (``security.metrics_token``), which is all Prometheus holds."""
                given = self.headers.get("X-TK-Agent-Token", "")
                bearer = self.headers.get("Authorization", "")
                if not given and bearer.startswith("Bearer "):  # Prometheus' scrape authorization
                    given = bearer[len("Bearer "):]
                if hmac.compare_digest(given, agent.token):
                    return True
                return read_only and hmac.compare_digest(given, metrics_token(agent.token))

            def do_GET(self):
                if self._gone():
                    return None
                path = urllib.parse.urlsplit(self.path).path
                if not self._auth(read_only=path in ("/metrics", "/v1/health")):
                    return self._reply(401, {"error": "unauthorized"})
                if urllib.parse.urlsplit(self.path).path == "/v1/info":
                    with agent._gate_mu:
                        pending = len(agent._gates)
                    return self._reply(200, {"name": agent.name, "mode": agent.mode, "devices": agent.devices,
                                             "labels": agent.last_labels, "pending_gates": pending,
                                             # what the agent took from /etc/rccl/rccl.env at start
                                             "rccl_env_applied": sorted(getattr(agent, "rccl_env_applied", {})),
                                             "rccl_env_skipped": list(getattr(agent, "rccl_env_skipped", []))})
                if urllib.parse.urlsplit(self.path).path == "/metrics":
                    from .metrics import CONTENT_TYPE

                    try:
                        body = agent.metrics().encode()
                    except Exception as exc:  # noqa: BLE001
                        return self._reply(500, {"error": f"{type(exc).__name__}: {exc}"})
                    self.send_response(200)
                    self.send_header("Content-Type", CONTENT_TYPE)
                    self.send_header("Content-Length", str(len(body)))
                    self.end_headers()
                    self.wfile.write(body)
                    return None
                if urllib.parse.urlsplit(self.path).path == "/v1/health":
                    try:
                        q = urllib.parse.parse_qs(urllib.parse.urlsplit(self.path).query)
                        return self._reply(200, agent.health(int(q.get("max_uncorrectable", ["0"])[0]),
                                                             int(q.get("max_bad_pages", ["-1"])[0])))
                    except Exception as exc:  # noqa: BLE001
                        return self._reply(500, {"error": f"{type(exc).__name__}: {exc}"})
                return self._reply(404, {"error": "not found"})

            def do_POST(self):
                if self._gone():
                    return None
                if not self._auth():
                    # the request body is not read: this connection cannot carry another request
                    self.close_connection = True
                    return self._reply(401, {"error": "unauthorized"})
                path = urllib.parse.urlsplit(self.path).path
                try:
                    body = self._body()
                    if path == "/v1/plan":
                        try:
                            plan = BootstrapPlan.from_json(body["plan"])
                        except (AttributeError, KeyError, TypeError, ValueError) as exc:
                            raise _BadRequest(400, f"malformed plan: {type(exc).__name__}: {exc}") from exc
                        bad = agent.refusals(plan)
                        if bad:
                            return self._reply(403, {"error": bad[0]})
                        return self._reply(200, agent.run_plan(plan))
                    if path == "/v1/rccl-uid":
                        return self._reply(200, {"uid": base64.b64encode(agent.new_uid()).decode()})
                    if path == "/v1/rccl-prepare":
                        uid = base64.b64decode(body["uid"], validate=True) if body.get("uid") else None
                        return self._reply(200, agent.rccl_prepare(uid,
                                                                   int(body["world"]), int(body["rank_base"]),
                                                                   int(body.get("ndev", 1)),
                                                                   int(body.get("max_bytes", 0)),
                                                                   [int(x) for x in body.get("sizes") or []]))
                    if path == "/v1/rccl-gate":
                        uid = base64.b64decode(body["uid"], validate=True)
                        return self._reply(200, agent.rccl_gate(int(body["rank"]), int(body["world"]), uid,
                                                                [int(s) for s in body.get("sizes", [1 << 20])],
                                                                int(body.get("iters", 10)),
                                                                int(body.get("ndev", 1)),
                                                                float(body.get("timeout_s", 600.0)),
                                                                bool(body.get("release_holds", False))))
                    if path == "/v1/rccl-abort":
                        return self._reply(200, agent.rccl_abort(base64.b64decode(body["uid"], validate=True)))
                    if path == "/v1/cleanup":
                        return self._reply(200, agent.cleanup())
                    if path == "/v1/shutdown":
                        # the daemon's main loop (main()) stops the agent and exits; an
                        # embedded agent (no main loop) ignores it
                        agent.shutdown_requested.set()
                        return self._reply(200, {"ok": True})
                except GateAborted as exc:
                    return self._reply(409, {"error": f"GateAborted: {exc}", "aborted": True})
                except _BadRequest as exc:
                    self.close_connection = True  # the body was not read: the stream is out of step
                    return self._reply(exc.code, {"error": str(exc)})
                except (KeyError, TypeError, ValueError, binascii.Error) as exc:
                    # a request this agent cannot take (a missing or malformed field, a value a
                    # step's validation refused): the caller's, not the node's, error
                    return self._reply(400, {"error": f"{type(exc).__name__}: {exc}"})
                except Exception as exc:  # noqa: BLE001
                    return self._reply(500, {"error": f"{type(exc).__name__}: {exc}"})
                return self._reply(404, {"error": "not found"})

        self._server = HTTPServer((host, port), H)
        self._server.daemon_threads = True
        if ssl_context is not None:
            self._server.socket = ssl_context.wrap_socket(self._server.socket, server_side=True,
                                                          do_handshake_on_connect=False)
        # short poll: stop() (server.shutdown) returns within ~20 ms instead of the default 0.5 s
        threading.Thread(target=self._server.serve_forever, kwargs={"poll_interval": 0.02},
                         name=f"agent-{self.name}", daemon=True).start()
        h, p = self._server.server_address[:2]
        return f"{'https' if ssl_context is not None else 'http'}://{h}:{p}"


__all__ = ["AgentHTTPMixin"]
