"""In-process fake S3 (path-style) that verifies SigV4 signatures — for the backup tests."""

import datetime
import http.server
import socket
import threading
import urllib.parse
from typing import Dict, Tuple
from xml.sax.saxutils import escape

from ..utils.httpserver import Server as HTTPServer
from .aws import sigv4_headers


class FakeS3:
    def __init__(self, access_key: str = "AKIDTEST", secret_key: str = "secret", region: str = "us-east-1",
                 page_size: int = 1000):
        self.access_key, self.secret_key, self.region = access_key, secret_key, region
        self.page_size = page_size
        self.objects: Dict[Tuple[str, str], bytes] = {}
        self.encryption: Dict[Tuple[str, str], str] = {}  # x-amz-server-side-encryption per object
        self.buckets = set()
        self.rejected = 0
        self.mu = threading.Lock()
        self._server = HTTPServer(("127.0.0.1", 0), self._handler())
        self._server.daemon_threads = True

    @property
    def url(self) -> str:
        h, p = self._server.server_address[:2]
        return f"http://{h}:{p}"

    def start(self) -> "FakeS3":
        threading.Thread(target=self._server.serve_forever, daemon=True, name="fake-s3").start()
        return self

    def stop(self) -> None:
        self._server.shutdown()
        self._server.server_close()

    def _verify(self, method: str, path: str, headers, body: bytes) -> bool:
        auth = headers.get("Authorization", "")
        amz_date = headers.get("X-Amz-Date", "")
        if not auth.startswith("AWS4-HMAC-SHA256 ") or not amz_date:
            return False
        try:
            now = datetime.datetime.strptime(amz_date, "%Y%m%dT%H%M%SZ")
        except ValueError:
            return False
        # every other x-amz-* header the client signed (e.g. server-side encryption) is part
        # of the signature: a header sent unsigned, or signed with another value, fails
        signed = auth.split("SignedHeaders=", 1)[-1].split(",", 1)[0].split(";")
        extra = {h: headers.get(h, "") for h in signed
                 if h.startswith("x-amz-") and h not in ("x-amz-date", "x-amz-content-sha256", "x-amz-security-token")}
        if any(k.lower().startswith("x-amz-") and k.lower() not in signed for k in headers.keys()):
            return False
        want = sigv4_headers(method, self.url + path, body, self.access_key, self.secret_key, self.region, "s3",
                             now=now, content_sha256=True, extra=extra)
        return want["Authorization"] == auth and headers.get("X-Amz-Content-Sha256") == want["X-Amz-Content-Sha256"]

    def _handler(self):
        fake = self

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def setup(self):
                super().setup()
                self.request.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

            def log_message(self, *args):
                pass

            def _reply(self, code: int, body: bytes = b"", ctype: str = "application/xml"):
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _do(self, method: str):
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n) if n else b""
                if not fake._verify(method, self.path, self.headers, body):
                    with fake.mu:
                        fake.rejected += 1
                    return self._reply(403, b"<Error><Code>SignatureDoesNotMatch</Code></Error>")
                parts = urllib.parse.urlsplit(self.path)
                bucket, _, key = urllib.parse.unquote(parts.path).lstrip("/").partition("/")
                q = dict(urllib.parse.parse_qsl(parts.query, keep_blank_values=True))
                with fake.mu:
                    if method == "PUT":
                        fake.buckets.add(bucket)
                        fake.objects[(bucket, key)] = body
                        fake.encryption[(bucket, key)] = self.headers.get("x-amz-server-side-encryption", "")
                        return self._reply(200)
                    if key:
                        data = fake.objects.get((bucket, key))
                        if data is None:
                            return self._reply(404, b"<Error><Code>NoSuchKey</Code></Error>")
                        return self._reply(200, data, "application/octet-stream")
                    keys = sorted(k for b, k in fake.objects if b == bucket and k.startswith(q.get("prefix", "")))
                    start = int(q.get("continuation-token") or 0)
                    page = keys[start:start + fake.page_size]
                    more = start + fake.page_size < len(keys)
                    xml = "<ListBucketResult>" + "".join(f"<Contents><Key>{escape(k)}</Key></Contents>" for k in page)
                    xml += f"<IsTruncated>{'true' if more else 'false'}</IsTruncated>"
                    if more:
                        xml += f"<NextContinuationToken>{start + fake.page_size}</NextContinuationToken>"
                    xml += "</ListBucketResult>"
                    return self._reply(200, xml.encode())

            def do_PUT(self):
                self._do("PUT")

            def do_GET(self):
                self._do("GET")

        return H
