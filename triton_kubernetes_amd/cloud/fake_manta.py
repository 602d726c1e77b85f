"""In-process fake Manta object store (directories + objects) with HTTP-signature checks.

Used by the Manta backend tests and by the Triton/Manta dry-run configuration
(BASELINE.json config #4).  Every request must carry a valid joyent HTTP
signature for a registered RSA public key (``add_key``).  Like Manta it refuses
to delete a non-empty directory (``DirectoryNotEmpty``), returns an ``ETag`` for
every object, and honours the conditional headers ``If-Match`` /
``If-None-Match`` (``*`` or an etag list) on PUT, GET and DELETE with HTTP 412
``PreconditionFailed``.
"""

import base64
import email.utils
import hashlib
import http.server
import json
import socket
import threading
import time
import urllib.parse
from typing import Dict, Optional, Tuple

from ..utils.sshkeys import PrivateKey, rsa_pkcs1v15_verify
from ..utils.httpserver import Server as HTTPServer
from .triton import parse_signature_header


class FakeManta:
    def __init__(self, account: str = "acct"):
        self.account = account
        self.keys: Dict[str, PrivateKey] = {}  # keyId path -> key (public half used)
        self.dirs = {f"/{account}/stor"}
        self.objects: Dict[str, Tuple[bytes, str, str]] = {}  # path -> (data, content type, etag)
        self._etag_seq = 0
        self.mu = threading.Lock()
        self.requests = 0
        self.rejected = 0
        self._server = HTTPServer(("127.0.0.1", 0), self._handler())
        self._server.daemon_threads = True

    def add_key(self, key: PrivateKey, key_id: Optional[str] = None) -> None:
        self.keys[f"/{self.account}/keys/{key_id or key.fingerprint_md5()}"] = key

    @property
    def url(self) -> str:
        h, p = self._server.server_address[:2]
        return f"http://{h}:{p}"

    def start(self) -> "FakeManta":
        threading.Thread(target=self._server.serve_forever, daemon=True, name="fake-manta").start()
        return self

    def stop(self) -> None:
        self._server.shutdown()
        self._server.server_close()

    def _verify(self, headers) -> bool:
        sig = parse_signature_header(headers.get("Authorization", ""))
        key = self.keys.get(sig.get("keyId", ""))
        date = headers.get("Date", "")
        if key is None or key.kind != "rsa" or not date:
            return False
        try:
            if abs(email.utils.parsedate_to_datetime(date).timestamp() - time.time()) > 300:
                return False
            raw = base64.b64decode(sig.get("signature", ""))
        except (TypeError, ValueError):
            return False
        return rsa_pkcs1v15_verify(key.n, key.e, f"date: {date}".encode(), raw)

    def _handler(self):
        fake = self

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def setup(self):
                super().setup()
                self.request.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

            def log_message(self, *args):
                pass

            def _reply(self, code: int, body: bytes = b"", ctype: str = "application/json", extra=None):
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                for k, v in (extra or {}).items():
                    self.send_header(k, v)
                self.end_headers()
                self.wfile.write(body)

            def _err(self, code: int, name: str):
                self._reply(code, json.dumps({"code": name, "message": name}).encode())

            def _path(self) -> Tuple[str, Dict]:
                parts = urllib.parse.urlsplit(self.path)
                return urllib.parse.unquote(parts.path).rstrip("/"), urllib.parse.parse_qs(parts.query)

            def _precondition_ok(self, path: str) -> bool:
                """If-Match / If-None-Match against the object's current etag (fake.mu held)."""
                cur = fake.objects.get(path)
                etag = cur[2] if cur is not None else None
                im, inm = self.headers.get("If-Match"), self.headers.get("If-None-Match")
                tags = lambda v: {t.strip().strip('"') for t in v.split(",")}  # noqa: E731
                if im is not None and (etag is None or (im.strip() != "*" and etag not in tags(im))):
                    return False
                if inm is not None and etag is not None and (inm.strip() == "*" or etag in tags(inm)):
                    return False
                return True

            def _guard(self) -> bool:
                with fake.mu:
                    fake.requests += 1
                if not fake._verify(self.headers):
                    with fake.mu:
                        fake.rejected += 1
                    self._err(403, "InvalidSignature")
                    return False
                return True

            def do_PUT(self):
                if not self._guard():
                    return
                path, _ = self._path()
                n = int(self.headers.get("Content-Length") or 0)
                data = self.rfile.read(n) if n else b""
                parent = path.rsplit("/", 1)[0]
                with fake.mu:
                    if parent not in fake.dirs:
                        return self._err(404, "DirectoryDoesNotExist")
                    if "type=directory" in self.headers.get("Content-Type", ""):
                        fake.dirs.add(path)
                        return self._reply(204)
                    if not self._precondition_ok(path):
                        return self._err(412, "PreconditionFailed")
                    fake._etag_seq += 1
                    etag = hashlib.md5(data + str(fake._etag_seq).encode()).hexdigest()
                    fake.objects[path] = (data, self.headers.get("Content-Type", ""), etag)
                self._reply(204, extra={"ETag": etag})

            def do_GET(self):
                if not self._guard():
                    return
                path, q = self._path()
                with fake.mu:
                    if path in fake.objects:
                        data, ctype, etag = fake.objects[path]
                        return self._reply(200, data, ctype, {"ETag": etag})
                    if path in fake.dirs:
                        names = sorted({p[len(path) + 1:].split("/", 1)[0] for p in list(fake.dirs) +
                                        list(fake.objects) if p.startswith(path + "/")})
                        marker = (q.get("marker") or [""])[0]
                        limit = int((q.get("limit") or ["1000"])[0])
                        if marker:
                            names = [n for n in names if n >= marker]
                        names = names[:limit]
                        lines = [json.dumps({"name": n, "type": "directory" if f"{path}/{n}" in fake.dirs
                                             else "object"}) for n in names]
                        return self._reply(200, ("\n".join(lines) + "\n").encode(), "application/x-json-stream",
                                           {"Result-Set-Size": str(len(names))})
                self._err(404, "ResourceNotFound")

            def do_DELETE(self):
                if not self._guard():
                    return
                path, _ = self._path()
                with fake.mu:
                    if path in fake.objects:
                        if not self._precondition_ok(path):
                            return self._err(412, "PreconditionFailed")
                        del fake.objects[path]
                    elif path in fake.dirs:
                        if any(p.startswith(path + "/") for p in list(fake.dirs) + list(fake.objects)):
                            return self._err(400, "DirectoryNotEmpty")
                        fake.dirs.discard(path)
                    else:
                        return self._err(404, "ResourceNotFound")
                self._reply(204)

        return H
