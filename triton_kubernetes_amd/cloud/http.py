"""Minimal HTTP(S) client on the standard library.

All cloud/Rancher REST traffic goes through :class:`HTTPClient`: persistent
per-host connections (``http.client`` keep-alive, one connection per thread),
JSON helpers, TLS verification (against the system store or a given context, e.g. a
Rancher server's pinned CA, ``rancher/trust.py``; a failure is :class:`TLSVerificationError`,
never retried), and a request hook for signing
(Triton/Manta HTTP signatures, AWS SigV4, bearer tokens).
"""

import http.client
import json
import socket
import ssl
import threading
import time
import urllib.parse
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Optional, Tuple

from ..errors import TKError


class TLSVerificationError(TKError):
    """The server's certificate did not verify against the client's trust roots: never
    retried, and no request (no credential) was sent."""


class HTTPError(TKError):
    def __init__(self, status: int, body: bytes, method: str, url: str):
        self.status = status
        self.body = body
        text = body.decode("utf-8", errors="replace")[:500]
        super().__init__(f"{method} {url}: HTTP {status}: {text}")

    def json(self) -> Any:
        try:
            return json.loads(self.body or b"null")
        except ValueError:
            return None


@dataclass
class Response:
    status: int
    headers: Dict[str, str]
    body: bytes
    elapsed: float = 0.0

    def json(self) -> Any:
        """The body as JSON; a body that is not (a proxy's HTML page, a truncated reply) is an
        error with its first bytes, not a bare ``JSONDecodeError``."""
        try:
            return json.loads(self.body or b"null")
        except ValueError:
            raise TKError(f"expected a JSON response (HTTP {self.status}), got: "
                          f"{bytes(self.body[:120])!r}") from None

    def header(self, name: str, default: str = "") -> str:
        return self.headers.get(name.lower(), default)


Signer = Callable[[str, str, Dict[str, str], bytes], None]
"""``signer(method, url, headers, body)`` mutates ``headers`` in place."""


_CTX_LOCK = threading.Lock()
_CTX: Dict[str, ssl.SSLContext] = {}


def _system_context() -> ssl.SSLContext:
    """One verifying context over the system's trust store per process: building it parses
    the whole CA bundle (~70 ms of CPU), and every new connection of every client had paid
    that.  An SSLContext is safe to share between threads and connections."""
    with _CTX_LOCK:
        ctx = _CTX.get("system")
        if ctx is None:
            ctx = _CTX["system"] = ssl.create_default_context()
        return ctx


def _unverified_context() -> ssl.SSLContext:
    """For the callers that verify by other means (a checksum over what they fetch): no trust
    store is loaded at all."""
    with _CTX_LOCK:
        ctx = _CTX.get("none")
        if ctx is None:
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
            _CTX["none"] = ctx
        return ctx


@dataclass
class HTTPClient:
    base_url: str = ""
    verify_tls: bool = True
    timeout: float = 30.0
    signer: Optional[Signer] = None
    default_headers: Dict[str, str] = field(default_factory=dict)
    retries: int = 2
    retry_backoff: float = 0.2
    # verify against this context's trust roots (e.g. a node-agent CA) instead of the system's
    ssl_context: Optional[ssl.SSLContext] = None
    # appended to a certificate verification failure: what the server was checked against
    tls_hint: str = ""

    def __post_init__(self):
        self._local = threading.local()

    def _ssl_context(self) -> ssl.SSLContext:
        if self.ssl_context is not None:
            return self.ssl_context
        return _system_context() if self.verify_tls else _unverified_context()

    def _conn(self, scheme: str, netloc: str) -> http.client.HTTPConnection:
        pool = getattr(self._local, "pool", None)
        if pool is None:
            pool = self._local.pool = {}
        key = (scheme, netloc)
        conn = pool.get(key)
        if conn is None:
            if scheme == "https":
                conn = http.client.HTTPSConnection(netloc, timeout=self.timeout, context=self._ssl_context())
            else:
                conn = http.client.HTTPConnection(netloc, timeout=self.timeout)
            pool[key] = conn
        if conn.sock is None:
            conn.connect()
            conn.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        return conn

    def _drop(self, scheme: str, netloc: str) -> None:
        pool = getattr(self._local, "pool", {})
        conn = pool.pop((scheme, netloc), None)
        if conn is not None:
            conn.close()

    def url(self, path: str) -> str:
        if path.startswith("http://") or path.startswith("https://"):
            return path
        return self.base_url.rstrip("/") + "/" + path.lstrip("/")

    def request(
        self,
        method: str,
        path: str,
        *,
        params: Optional[Dict[str, Any]] = None,
        json_body: Any = None,
        data: Optional[bytes] = None,
        headers: Optional[Dict[str, str]] = None,
        ok: Tuple[int, ...] = (200, 201, 202, 204),
    ) -> Response:
        url = self.url(path)
        if params:
            url += ("&" if "?" in url else "?") + urllib.parse.urlencode(params, doseq=True)
        hdrs = dict(self.default_headers)
        hdrs.update(headers or {})
        body = data or b""
        if json_body is not None:
            body = json.dumps(json_body).encode()
            hdrs.setdefault("Content-Type", "application/json")
        hdrs.setdefault("Accept", "application/json")
        if self.signer is not None:
            self.signer(method, url, hdrs, body)
        parts = urllib.parse.urlsplit(url)
        target = parts.path or "/"
        if parts.query:
            target += "?" + parts.query
        attempt = 0
        while True:
            t0 = time.perf_counter()
            try:
                conn = self._conn(parts.scheme, parts.netloc)
                conn.request(method, target, body=body if body or method in ("POST", "PUT") else None, headers=hdrs)
                resp = conn.getresponse()
                payload = resp.read()
                out = Response(resp.status, {k.lower(): v for k, v in resp.getheaders()}, payload,
                               time.perf_counter() - t0)
                if resp.getheader("connection", "").lower() == "close":
                    self._drop(parts.scheme, parts.netloc)
                break
            except ssl.SSLCertVerificationError as exc:
                self._drop(parts.scheme, parts.netloc)
                raise TLSVerificationError(
                    f"{method} {url}: TLS: the server's certificate does not verify ({exc})"
                    + (f" against {self.tls_hint}" if self.tls_hint else "")
                    + "; refusing to send the request") from exc
            except (ConnectionError, http.client.HTTPException, OSError) as exc:
                self._drop(parts.scheme, parts.netloc)
                if attempt >= self.retries:
                    raise TKError(f"{method} {url}: {exc}") from exc
                attempt += 1
                time.sleep(self.retry_backoff * attempt)
        if out.status not in ok:
            raise HTTPError(out.status, out.body, method, url)
        return out

    def get_json(self, path: str, **kw) -> Any:
        return self.request("GET", path, **kw).json()

    def post_json(self, path: str, body: Any, **kw) -> Any:
        return self.request("POST", path, json_body=body, **kw).json()

    def put_json(self, path: str, body: Any, **kw) -> Any:
        return self.request("PUT", path, json_body=body, **kw).json()

    def close(self) -> None:
        pool = getattr(self._local, "pool", {})
        for conn in pool.values():
            conn.close()
        pool.clear()
