"""AWS EC2 listing client (Query API + Signature V4, stdlib only).

Replaces the aws-sdk-go calls of the reference: ``DescribeRegions`` (region
validation, issued against us-west-1, ``create/manager_aws.go:106-122``),
``DescribeKeyPairs`` (key picker), ``DescribeImages`` with the Ubuntu name
filter (AMI picker, ``manager_aws.go:426-436``).
"""

import datetime
import hashlib
import hmac
import urllib.parse
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from typing import Dict, List, Optional

from .http import HTTPClient

EC2_API_VERSION = "2016-11-15"
# Ubuntu 22.04 LTS, which the pinned Docker 24.0 installer supports (sizing.py); the
# reference filtered xenial 16.04 for its Docker 17.03 (create/manager_aws.go:426-436)
from ..sizing import AWS_AMI_FILTER as UBUNTU_AMI_FILTER  # noqa: E402


def _sign(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def sigv4_headers(method: str, url: str, body: bytes, access_key: str, secret_key: str, region: str,
                  service: str, now: Optional[datetime.datetime] = None,
                  session_token: Optional[str] = None, content_sha256: bool = False,
                  extra: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """Signature Version 4 headers for one request (AWS general reference algorithm).
    ``extra`` headers (e.g. ``x-amz-server-side-encryption``) are signed and returned."""
    now = now or datetime.datetime.utcnow()
    amz_date = now.strftime("%Y%m%dT%H%M%SZ")
    datestamp = now.strftime("%Y%m%d")
    parts = urllib.parse.urlsplit(url)
    host = parts.netloc
    canonical_uri = urllib.parse.quote(parts.path or "/", safe="/-_.~")
    query = urllib.parse.parse_qsl(parts.query, keep_blank_values=True)
    canonical_query = "&".join(
        f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}" for k, v in sorted(query))
    payload_hash = hashlib.sha256(body).hexdigest()
    headers = {"host": host, "x-amz-date": amz_date}
    if content_sha256:  # required by S3
        headers["x-amz-content-sha256"] = payload_hash
    if session_token:
        headers["x-amz-security-token"] = session_token
    for k, v in (extra or {}).items():
        headers[k.lower()] = str(v).strip()
    signed_headers = ";".join(sorted(headers))
    canonical_headers = "".join(f"{k}:{headers[k]}\n" for k in sorted(headers))
    canonical_request = "\n".join([method, canonical_uri, canonical_query, canonical_headers, signed_headers,
                                   payload_hash])
    scope = f"{datestamp}/{region}/{service}/aws4_request"
    string_to_sign = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope,
                                hashlib.sha256(canonical_request.encode()).hexdigest()])
    k = _sign(("AWS4" + secret_key).encode(), datestamp)
    k = _sign(k, region)
    k = _sign(k, service)
    k = _sign(k, "aws4_request")
    signature = hmac.new(k, string_to_sign.encode(), hashlib.sha256).hexdigest()
    out = {
        "X-Amz-Date": amz_date,
        "Authorization": (f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, "
                          f"SignedHeaders={signed_headers}, Signature={signature}"),
    }
    if session_token:
        out["X-Amz-Security-Token"] = session_token
    if content_sha256:
        out["X-Amz-Content-Sha256"] = payload_hash
    out.update(extra or {})
    return out


@dataclass
class AMI:
    id: str
    name: str
    creation_date: str


def _strip_ns(root: ET.Element) -> ET.Element:
    for el in root.iter():
        if "}" in el.tag:
            el.tag = el.tag.split("}", 1)[1]
    return root


class EC2Client:
    def __init__(self, access_key: str, secret_key: str, region: str = "us-west-1",
                 endpoint: Optional[str] = None, http: Optional[HTTPClient] = None):
        self.access_key, self.secret_key, self.region = access_key, secret_key, region
        self.endpoint = endpoint or f"https://ec2.{region}.amazonaws.com"
        self.http = http or HTTPClient()

    def _call(self, action: str, params: Optional[Dict[str, str]] = None) -> ET.Element:
        q = {"Action": action, "Version": EC2_API_VERSION}
        q.update(params or {})
        url = self.endpoint.rstrip("/") + "/?" + urllib.parse.urlencode(sorted(q.items()))
        hdrs = sigv4_headers("GET", url, b"", self.access_key, self.secret_key, self.region, "ec2")
        resp = self.http.request("GET", url, headers=hdrs)
        return _strip_ns(ET.fromstring(resp.body))

    def regions(self) -> List[str]:
        root = self._call("DescribeRegions")
        return [el.findtext("regionName", "") for el in root.iter("item") if el.find("regionName") is not None]

    def key_pairs(self) -> List[str]:
        root = self._call("DescribeKeyPairs")
        return [el.findtext("keyName", "") for el in root.iter("item") if el.find("keyName") is not None]

    def images(self, name_filter: str = UBUNTU_AMI_FILTER) -> List[AMI]:
        root = self._call("DescribeImages", {"Filter.1.Name": "name", "Filter.1.Value.1": name_filter})
        amis = [AMI(el.findtext("imageId", ""), el.findtext("name", ""), el.findtext("creationDate", ""))
                for el in root.iter("item") if el.find("imageId") is not None]
        amis.sort(key=lambda a: a.creation_date, reverse=True)  # newest first
        return amis

    def for_region(self, region: str) -> "EC2Client":
        return EC2Client(self.access_key, self.secret_key, region, http=self.http)


class S3Client:
    """Minimal S3 object client (path-style URLs, SigV4): put / get / list — used for cluster backups."""

    def __init__(self, access_key: str, secret_key: str, region: str = "us-east-1",
                 endpoint: Optional[str] = None, http: Optional[HTTPClient] = None):
        self.access_key, self.secret_key, self.region = access_key, secret_key, region
        self.endpoint = (endpoint or f"https://s3.{region}.amazonaws.com").rstrip("/")
        self.http = http or HTTPClient()

    def _url(self, bucket: str, key: str = "", query: str = "") -> str:
        path = f"/{bucket}" + (f"/{urllib.parse.quote(key, safe='/-_.~')}" if key else "")
        return self.endpoint + path + (f"?{query}" if query else "")

    def _req(self, method: str, url: str, body: bytes = b"", ok=(200,), extra: Optional[Dict[str, str]] = None):
        hdrs = sigv4_headers(method, url, body, self.access_key, self.secret_key, self.region, "s3",
                             content_sha256=True, extra=extra)
        return self.http.request(method, url, headers=hdrs, data=body if body else None, ok=ok)

    def put_object(self, bucket: str, key: str, data: bytes, encrypt: bool = True) -> None:
        """PUT an object; ``encrypt``: server-side encryption with S3-managed keys (SSE-S3)."""
        self._req("PUT", self._url(bucket, key), data, ok=(200, 201, 204),
                  extra={"x-amz-server-side-encryption": "AES256"} if encrypt else None)

    def get_object(self, bucket: str, key: str) -> bytes:
        return self._req("GET", self._url(bucket, key)).body

    def list_keys(self, bucket: str, prefix: str = "") -> List[str]:
        keys: List[str] = []
        token = ""
        while True:
            q = {"list-type": "2", "prefix": prefix}
            if token:
                q["continuation-token"] = token
            root = _strip_ns(ET.fromstring(self._req("GET", self._url(bucket, query=urllib.parse.urlencode(
                sorted(q.items())))).body))
            keys += [el.findtext("Key", "") for el in root.iter("Contents")]
            token = root.findtext("NextContinuationToken", "") or ""
            if root.findtext("IsTruncated", "false") != "true" or not token:
                return keys
