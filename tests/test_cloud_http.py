"""The stdlib cloud clients against an HTTP-level fake: request shape, auth and pagination.

Triton CloudAPI (HTTP signature), AWS EC2 (SigV4 query API, XML), GCP Compute
(service-account JWT -> token, pageToken pagination) and Azure ARM (client
credentials -> token, api-version).  The providers' own tests use FakeCloud at
the API-object level; these pin the wire protocol under it.
"""

import base64
import datetime
import http.server
import json
import threading
import urllib.parse

import pytest

from triton_kubernetes_amd.cloud.aws import EC2Client, sigv4_headers
from triton_kubernetes_amd.cloud.azure import ARMClient
from triton_kubernetes_amd.cloud.gcp import ComputeClient
from triton_kubernetes_amd.cloud.triton import HTTPSignatureSigner, TritonCloudAPI
from triton_kubernetes_amd.utils.sshkeys import load_private_key, rsa_pkcs1v15_verify

from helpers import make_ssh_key


class Recorder:
    """Routes (method, path) -> fn(query, headers, body) -> (status, body, ctype); records requests."""

    def __init__(self):
        self.routes = {}
        self.requests = []
        rec = self

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _do(self, method):
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n) if n else b""
                parts = urllib.parse.urlsplit(self.path)
                q = dict(urllib.parse.parse_qsl(parts.query, keep_blank_values=True))
                rec.requests.append((method, parts.path, q, dict(self.headers), body, self.path))
                fn = rec.routes.get((method, parts.path))
                status, out, ctype = fn(q, self.headers, body, self.path) if fn else (404, b"{}", "application/json")
                self.send_response(status)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(out)))
                self.end_headers()
                self.wfile.write(out)

            def do_GET(self):
                self._do("GET")

            def do_POST(self):
                self._do("POST")

        self.server = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.server.daemon_threads = True
        threading.Thread(target=self.server.serve_forever, daemon=True).start()
        h, p = self.server.server_address[:2]
        self.url = f"http://{h}:{p}"

    def stop(self):
        self.server.shutdown()
        self.server.server_close()


@pytest.fixture
def rec():
    r = Recorder()
    yield r
    r.stop()


def _json(obj):
    return 200, json.dumps(obj).encode(), "application/json"


def test_triton_cloudapi_signed_and_sorted(rec, tmp_path):
    key = load_private_key(make_ssh_key(tmp_path / "k"))
    rec.routes[("GET", "/acct/networks")] = lambda *a: _json([{"id": "n1", "name": "Joyent-SDC-Public",
                                                                "public": True}])
    rec.routes[("GET", "/acct/images")] = lambda *a: _json([
        {"id": "i1", "name": "ubuntu", "version": "1", "published_at": "2017-01-01T00:00:00Z"},
        {"id": "i2", "name": "ubuntu", "version": "2", "published_at": "2018-01-01T00:00:00Z"}])
    rec.routes[("GET", "/acct/packages")] = lambda *a: _json([{"id": "p2", "name": "big", "memory": 8192},
                                                              {"id": "p1", "name": "small", "memory": 1024}])
    api = TritonCloudAPI(rec.url, HTTPSignatureSigner("acct", key))
    assert [n.name for n in api.networks()] == ["Joyent-SDC-Public"]
    assert [i.version for i in api.images()] == ["2", "1"]  # newest first
    assert [p.name for p in api.packages()] == ["small", "big"]  # by memory
    for _, _, _, headers, _, _ in rec.requests:
        assert headers["Accept-Version"] == "8"
        sig = base64.b64decode(headers["Authorization"].split('signature="')[1].rstrip('"'))
        assert rsa_pkcs1v15_verify(key.n, key.e, f"date: {headers['Date']}".encode(), sig)


def test_ec2_query_api_sigv4(rec):
    xml = {"DescribeRegions": "<DescribeRegionsResponse xmlns='http://ec2.amazonaws.com/doc/2016-11-15/'>"
                              "<regionInfo><item><regionName>us-west-2</regionName></item>"
                              "<item><regionName>eu-west-1</regionName></item></regionInfo></DescribeRegionsResponse>",
           "DescribeKeyPairs": "<r><keySet><item><keyName>ops</keyName></item></keySet></r>",
           "DescribeImages": "<r><imagesSet><item><imageId>ami-1</imageId><name>a</name>"
                             "<creationDate>2017-01-01</creationDate></item><item><imageId>ami-2</imageId>"
                             "<name>b</name><creationDate>2018-01-01</creationDate></item></imagesSet></r>"}
    rec.routes[("GET", "/")] = lambda q, h, b, raw: (200, xml[q["Action"]].encode(), "text/xml")
    ec2 = EC2Client("AKID", "SECRET", "us-west-1", endpoint=rec.url)
    assert ec2.regions() == ["us-west-2", "eu-west-1"]
    assert ec2.key_pairs() == ["ops"]
    assert [a.id for a in ec2.images()] == ["ami-2", "ami-1"]
    _, _, q, headers, body, raw = rec.requests[-1]
    assert q["Filter.1.Name"] == "name" and q["Version"]
    now = datetime.datetime.strptime(headers["X-Amz-Date"], "%Y%m%dT%H%M%SZ")
    want = sigv4_headers("GET", rec.url + raw, b"", "AKID", "SECRET", "us-west-1", "ec2", now=now)
    assert headers["Authorization"] == want["Authorization"]
    assert "/us-west-1/ec2/aws4_request" in headers["Authorization"]


def test_gcp_compute_jwt_token_and_pagination(rec, tmp_path):
    key_path = make_ssh_key(tmp_path / "sa")
    key = load_private_key(key_path)
    creds = tmp_path / "creds.json"
    creds.write_text(json.dumps({"project_id": "proj", "client_email": "sa@proj.iam", "private_key_id": "kid",
                                 "private_key": open(key_path).read(), "token_uri": rec.url + "/token"}))
    tokens = []

    def token(q, h, body, raw):
        form = dict(urllib.parse.parse_qsl(body.decode()))
        assert form["grant_type"] == "urn:ietf:params:oauth:grant-type:jwt-bearer"
        head, claims, sig = form["assertion"].split(".")
        pad = lambda s: s + "=" * (-len(s) % 4)  # noqa: E731
        assert rsa_pkcs1v15_verify(key.n, key.e, f"{head}.{claims}".encode(), base64.urlsafe_b64decode(pad(sig)))
        tokens.append(1)
        return _json({"access_token": "ya29.tok", "expires_in": 3600})

    def zones(q, h, body, raw):
        assert h["Authorization"] == "Bearer ya29.tok"
        if q.get("pageToken") == "p2":
            return _json({"items": [{"name": "us-central1-b", "region": ".../regions/us-central1"}]})
        return _json({"items": [{"name": "us-central1-a", "region": ".../regions/us-central1"},
                                {"name": "europe-west1-b", "region": ".../regions/europe-west1"}],
                      "nextPageToken": "p2"})

    rec.routes[("POST", "/token")] = token
    rec.routes[("GET", "/compute/v1/projects/proj/zones")] = zones
    gce = ComputeClient(str(creds), api=rec.url + "/compute/v1")
    assert gce.zones("us-central1") == ["us-central1-a", "us-central1-b"]  # both pages, filtered
    assert gce.zones("europe-west1") == ["europe-west1-b"]
    assert len(tokens) == 1  # cached across calls


def test_azure_arm_client_credentials(rec):
    def token(q, h, body, raw):
        form = dict(urllib.parse.parse_qsl(body.decode()))
        assert form == {"grant_type": "client_credentials", "client_id": "cid", "client_secret": "sec",
                        "resource": rec.url + "/"}
        return _json({"access_token": "arm-tok", "expires_in": "3600"})

    rec.routes[("POST", "/tenant/oauth2/token")] = token
    rec.routes[("GET", "/subscriptions/sub/locations")] = lambda q, h, b, raw: _json(
        {"value": [{"name": "westus2"}, {"name": "eastus"}]})
    rec.routes[("GET", "/subscriptions/sub/providers/Microsoft.Compute/locations/westus2/vmSizes")] = \
        lambda q, h, b, raw: _json({"value": [{"name": "Standard_A0"}]})
    arm = ARMClient("sub", "cid", "sec", "tenant", endpoints={"login": rec.url, "arm": rec.url})
    assert arm.locations() == ["westus2", "eastus"]
    assert arm.vm_sizes("westus2") == ["Standard_A0"]
    gets = [r for r in rec.requests if r[0] == "GET"]
    assert [r[2]["api-version"] for r in gets] == ["2016-06-01", "2017-12-01"]
    assert all(r[3]["Authorization"] == "Bearer arm-tok" for r in gets)


def test_tls_contexts_are_built_once_per_process():
    """Parsing the system trust store costs ~70 ms of CPU: every client and connection shares
    one verifying context, and the unverified one loads no store at all."""
    import ssl

    from triton_kubernetes_amd.cloud.http import HTTPClient
    from triton_kubernetes_amd.rancher.trust import RancherTrust

    a, b = HTTPClient(base_url="https://a"), HTTPClient(base_url="https://b")
    assert a._ssl_context() is b._ssl_context() is RancherTrust().context()
    assert a._ssl_context().verify_mode == ssl.CERT_REQUIRED and a._ssl_context().check_hostname
    off = HTTPClient(base_url="https://a", verify_tls=False)._ssl_context()
    assert off is not a._ssl_context() and off.verify_mode == ssl.CERT_NONE and not off.check_hostname
    assert off.cert_store_stats()["x509_ca"] == 0
