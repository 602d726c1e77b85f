"""Triton CloudAPI + Manta clients with HTTP-signature auth.

Replaces ``github.com/joyent/triton-go`` as used by the reference:

* ``network.List``, ``Images().List``, ``Packages().List`` for validation and
  prompt listings (``create/manager_triton.go:153-364``, ``node_triton.go``);
* Manta ``Dir().Put/List/Delete`` and ``Objects().Get/Put/Delete`` for the
  Manta state backend (``backend/manta/backend.go``).

Auth is the joyent HTTP Signature scheme: ``Authorization: Signature
keyId="/<account>/keys/<md5 fingerprint>",algorithm="rsa-sha256",
headers="date",signature="<base64 sig over 'date: <RFC1123 date>'>"``.
"""

import base64
import email.utils
import json
import urllib.parse
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

from ..utils.sshkeys import PrivateKey, load_private_key
from .http import HTTPClient, HTTPError


class HTTPSignatureSigner:
    def __init__(self, account: str, key: PrivateKey, key_id: Optional[str] = None, user: Optional[str] = None):
        self.account = account
        self.key = key
        self.key_id = key_id or key.fingerprint_md5()
        self.user = user

    @classmethod
    def from_path(cls, account: str, key_path: str, key_id: Optional[str] = None) -> "HTTPSignatureSigner":
        return cls(account, load_private_key(key_path), key_id)

    @property
    def key_id_path(self) -> str:
        if self.user:
            return f"/{self.account}/users/{self.user}/keys/{self.key_id}"
        return f"/{self.account}/keys/{self.key_id}"

    def sign_date(self, date: str) -> str:
        sig = self.key.sign(f"date: {date}".encode())
        return base64.b64encode(sig).decode()

    def __call__(self, method: str, url: str, headers: Dict[str, str], body: bytes) -> None:
        date = email.utils.formatdate(usegmt=True)
        headers["Date"] = date
        headers["Authorization"] = (
            f'Signature keyId="{self.key_id_path}",algorithm="{self.key.http_signature_algorithm()}",'
            f'headers="date",signature="{self.sign_date(date)}"'
        )


def parse_signature_header(value: str) -> Dict[str, str]:
    """Parse an ``Authorization: Signature k="v",...`` header (used by fakes)."""
    if not value.startswith("Signature "):
        return {}
    out = {}
    for part in value[len("Signature "):].split(","):
        k, _, v = part.partition("=")
        out[k.strip()] = v.strip().strip('"')
    return out


@dataclass
class Network:
    id: str
    name: str
    public: bool = False


@dataclass
class Image:
    id: str
    name: str
    version: str
    published_at: str = ""
    os: str = ""


@dataclass
class Package:
    id: str
    name: str
    memory: int = 0
    vcpus: int = 0
    disk: int = 0


class TritonCloudAPI:
    def __init__(self, url: str, signer: HTTPSignatureSigner, http: Optional[HTTPClient] = None):
        self.account = signer.account
        self.http = http or HTTPClient(base_url=url, signer=signer)
        if http is not None:
            self.http.signer = signer
            self.http.base_url = url
        self.http.default_headers.setdefault("Accept-Version", "8")

    def networks(self) -> List[Network]:
        data = self.http.get_json(f"/{self.account}/networks")
        return [Network(n.get("id", ""), n.get("name", ""), bool(n.get("public"))) for n in data]

    def images(self) -> List[Image]:
        data = self.http.get_json(f"/{self.account}/images")
        imgs = [Image(i.get("id", ""), i.get("name", ""), i.get("version", ""), i.get("published_at", ""),
                      i.get("os", "")) for i in data]
        # newest first (create/manager_triton.go:271-274)
        imgs.sort(key=lambda i: i.published_at, reverse=True)
        return imgs

    def packages(self) -> List[Package]:
        data = self.http.get_json(f"/{self.account}/packages")
        pkgs = [Package(p.get("id", ""), p.get("name", ""), int(p.get("memory", 0)), int(p.get("vcpus", 0)),
                        int(p.get("disk", 0))) for p in data]
        # increasing memory (create/manager_triton.go:347-350)
        pkgs.sort(key=lambda p: p.memory)
        return pkgs


class MantaClient:
    """The subset of the Manta storage API the state backend needs."""

    def __init__(self, url: str, signer: HTTPSignatureSigner, http: Optional[HTTPClient] = None):
        self.account = signer.account
        self.http = http or HTTPClient(base_url=url, signer=signer)
        if http is not None:
            self.http.signer = signer
            self.http.base_url = url

    def _path(self, path: str) -> str:
        # "/stor/x" -> "/<account>/stor/x"
        return f"/{self.account}/{path.lstrip('/')}"

    def put_directory(self, path: str) -> None:
        self.http.request("PUT", urllib.parse.quote(self._path(path)),
                          headers={"Content-Type": "application/json; type=directory"}, data=b"")

    def list_directory(self, path: str, limit: int = 1000) -> List[Dict[str, Any]]:
        """All entries (paginated with ``marker``; the reference stops at 100)."""
        entries: List[Dict[str, Any]] = []
        marker = None
        while True:
            params: Dict[str, Any] = {"limit": limit}
            if marker:
                params["marker"] = marker
            resp = self.http.request("GET", urllib.parse.quote(self._path(path)), params=params)
            page = [json.loads(line) for line in resp.body.decode().splitlines() if line.strip()]
            if marker and page and page[0].get("name") == marker:
                page = page[1:]
            entries.extend(page)
            if len(page) < limit - (1 if marker else 0) or not page:
                return entries
            marker = page[-1].get("name")

    def get_object(self, path: str) -> Optional[bytes]:
        try:
            return self.http.request("GET", urllib.parse.quote(self._path(path))).body
        except HTTPError as exc:
            if exc.status == 404 or b"ResourceNotFound" in exc.body:
                return None
            raise

    def get_object_etag(self, path: str) -> Tuple[Optional[bytes], Optional[str]]:
        """``(body, etag)``; ``(None, None)`` when the object does not exist."""
        try:
            resp = self.http.request("GET", urllib.parse.quote(self._path(path)))
        except HTTPError as exc:
            if exc.status == 404 or b"ResourceNotFound" in exc.body:
                return None, None
            raise
        return resp.body, resp.header("etag") or None

    def put_object(self, path: str, data: bytes, content_type: str = "application/json",
                   if_match: Optional[str] = None, if_none_match: Optional[str] = None) -> Optional[str]:
        """PUT an object; returns its new ETag.  With ``if_match`` / ``if_none_match``
        (``"*"``: only if absent) the write is conditional: a failed precondition
        (HTTP 412) returns None and changes nothing."""
        headers = {"Content-Type": content_type}
        if if_match is not None:
            headers["If-Match"] = if_match
        if if_none_match is not None:
            headers["If-None-Match"] = if_none_match
        try:
            resp = self.http.request("PUT", urllib.parse.quote(self._path(path)), data=data, headers=headers)
        except HTTPError as exc:
            if exc.status == 412 and (if_match is not None or if_none_match is not None):
                return None
            raise
        return resp.header("etag") or ""

    def delete(self, path: str, missing_ok: bool = True, if_match: Optional[str] = None) -> bool:
        """DELETE; False when ``if_match`` no longer matches (HTTP 412) or the object was absent."""
        headers = {"If-Match": if_match} if if_match is not None else None
        try:
            self.http.request("DELETE", urllib.parse.quote(self._path(path)), headers=headers)
            return True
        except HTTPError as exc:
            if if_match is not None and exc.status == 412:
                return False
            if not (missing_ok and exc.status == 404):
                raise
            return False
