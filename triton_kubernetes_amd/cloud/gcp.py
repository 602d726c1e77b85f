"""GCP Compute listing client (service-account JWT -> OAuth2 token, stdlib only).

Replaces ``google.golang.org/api/compute/v1`` usage of the reference
(``create/manager_gcp.go:93-310``): ``Regions.List``, ``Zones.List`` filtered by
region, ``MachineTypes.List(zone)``, ``Images.List("ubuntu-os-cloud")`` newest
first.  The JWT is RS256-signed with the pure-Python RSA in ``utils.sshkeys``.
"""

import base64
import json
import time
import urllib.parse
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

from ..errors import TKError
from ..utils.sshkeys import parse_private_key
from .http import HTTPClient

SCOPE_COMPUTE_READONLY = "https://www.googleapis.com/auth/compute.readonly"
COMPUTE_API = "https://compute.googleapis.com/compute/v1"


def _b64url(data: bytes) -> str:
    return base64.urlsafe_b64encode(data).decode().rstrip("=")


def load_credentials(path: str) -> Dict[str, Any]:
    try:
        with open(path, "r", encoding="utf-8") as fh:
            return json.load(fh)
    except (OSError, ValueError) as exc:
        raise TKError(f"could not read GCP credentials file '{path}': {exc}") from exc


def project_id_from_credentials(path: str) -> str:
    """``gcp_project_id`` comes from the credentials JSON (``manager_gcp.go:103-110``)."""
    return str(load_credentials(path).get("project_id", ""))


def make_jwt(creds: Dict[str, Any], scope: str, now: Optional[int] = None) -> str:
    now = int(now if now is not None else time.time())
    header = {"alg": "RS256", "typ": "JWT"}
    if creds.get("private_key_id"):
        header["kid"] = creds["private_key_id"]
    claims = {
        "iss": creds["client_email"],
        "scope": scope,
        "aud": creds.get("token_uri", "https://oauth2.googleapis.com/token"),
        "iat": now,
        "exp": now + 3600,
    }
    signing_input = _b64url(json.dumps(header, separators=(",", ":")).encode()) + "." + \
        _b64url(json.dumps(claims, separators=(",", ":")).encode())
    key = parse_private_key(creds["private_key"])
    return signing_input + "." + _b64url(key.sign(signing_input.encode(), "sha256"))


@dataclass
class GCPImage:
    name: str
    self_link: str
    creation_timestamp: str


class ComputeClient:
    def __init__(self, credentials_path: str, http: Optional[HTTPClient] = None, api: str = COMPUTE_API):
        self.creds = load_credentials(credentials_path)
        self.project = str(self.creds.get("project_id", ""))
        self.http = http or HTTPClient()
        self.api = api.rstrip("/")
        self._token: Optional[str] = None
        self._token_exp = 0.0

    def token(self) -> str:
        if self._token and time.time() < self._token_exp - 60:
            return self._token
        assertion = make_jwt(self.creds, SCOPE_COMPUTE_READONLY)
        body = urllib.parse.urlencode({
            "grant_type": "urn:ietf:params:oauth:grant-type:jwt-bearer",
            "assertion": assertion,
        }).encode()
        resp = self.http.request("POST", self.creds.get("token_uri", "https://oauth2.googleapis.com/token"),
                                 data=body, headers={"Content-Type": "application/x-www-form-urlencoded"})
        data = resp.json()
        self._token = data["access_token"]
        self._token_exp = time.time() + float(data.get("expires_in", 3600))
        return self._token

    def _list(self, path: str, params: Optional[Dict[str, str]] = None) -> List[Dict[str, Any]]:
        items: List[Dict[str, Any]] = []
        page = None
        while True:
            q = dict(params or {})
            if page:
                q["pageToken"] = page
            data = self.http.get_json(f"{self.api}/{path}", params=q or None,
                                      headers={"Authorization": f"Bearer {self.token()}"})
            items.extend(data.get("items", []) or [])
            page = data.get("nextPageToken")
            if not page:
                return items

    def regions(self) -> List[str]:
        return [r["name"] for r in self._list(f"projects/{self.project}/regions")]

    def zones(self, region: str) -> List[str]:
        # Zones.List filtered by region (manager_gcp.go:168)
        zones = self._list(f"projects/{self.project}/zones")
        return [z["name"] for z in zones if str(z.get("region", "")).endswith(f"/regions/{region}")]

    def machine_types(self, zone: str) -> List[str]:
        return [m["name"] for m in self._list(f"projects/{self.project}/zones/{zone}/machineTypes")]

    def images(self, image_project: str = "ubuntu-os-cloud") -> List[GCPImage]:
        imgs = [GCPImage(i["name"], i.get("selfLink", ""), i.get("creationTimestamp", ""))
                for i in self._list(f"projects/{image_project}/global/images")]
        imgs.sort(key=lambda i: i.creation_timestamp, reverse=True)
        return imgs
