"""The node agent's HTTP API refuses malformed requests with a 4xx, promptly, and keeps
serving: a length that is not a count (a negative one used to make the handler read until
the client hung up), a body over the limit, a body that is not a JSON object, missing or
malformed fields.  A property test throws generated JSON at ``/v1/plan``: the answer is a
200 (a plan that ran), a 400 or a 403, never a 500."""

import http.client
import json
import tempfile
import time

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from triton_kubernetes_amd.node.agent import NodeAgent
from triton_kubernetes_amd.node import agent_http

TOKEN = "robust-token-0123456789"


@pytest.fixture(scope="module")
def agent():
    a = NodeAgent(name="robust", mode="sim", token=TOKEN, root=tempfile.mkdtemp())
    url = a.serve()
    yield a, url.split("//")[1]
    a.stop()


def _raw(netloc, path, body=b"", length=None, token=TOKEN):
    conn = http.client.HTTPConnection(netloc, timeout=10)
    conn.putrequest("POST", path)
    conn.putheader("X-TK-Agent-Token", token)
    conn.putheader("Content-Length", str(len(body)) if length is None else length)
    conn.endheaders()
    if body:
        conn.send(body)
    resp = conn.getresponse()
    out = resp.status, json.loads(resp.read() or b"{}")
    conn.close()
    return out


@pytest.mark.parametrize("path,body,length,code", [
    ("/v1/plan", b"", "-5", 400),
    ("/v1/plan", b"", "abc", 400),
    ("/v1/plan", b"", str(agent_http.MAX_BODY + 1), 413),
    ("/v1/plan", b"[]", None, 400),
    ("/v1/plan", b"not json", None, 400),
    ("/v1/plan", b"{}", None, 400),
    ("/v1/plan", b'{"plan": {"hostname": 3}}', None, 400),
    ("/v1/rccl-prepare", b'{"world": "x", "rank_base": 0}', None, 400),
    ("/v1/rccl-abort", b'{"uid": "%%%"}', None, 400),
    ("/v1/nothing", b"{}", None, 404),
])
def test_malformed_requests_get_a_4xx_promptly(agent, path, body, length, code):
    _, netloc = agent
    t0 = time.monotonic()
    status, doc = _raw(netloc, path, body, length)
    assert status == code and "error" in doc, (status, doc)
    assert time.monotonic() - t0 < 5.0
    assert _get_info(netloc) == 200  # still serving


def _get_info(netloc):
    conn = http.client.HTTPConnection(netloc, timeout=10)
    conn.request("GET", "/v1/info", headers={"X-TK-Agent-Token": TOKEN})
    status = conn.getresponse().status
    conn.close()
    return status


JSON = st.recursive(st.none() | st.booleans() | st.integers(-5, 5) | st.text(max_size=8),
                    lambda kids: st.lists(kids, max_size=3) | st.dictionaries(st.text(max_size=8), kids, max_size=3),
                    max_leaves=10)


@settings(max_examples=80, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(st.one_of(JSON, st.dictionaries(st.just("plan"), JSON, min_size=1)))
def test_generated_plan_bodies_never_get_a_500(agent, body):
    _, netloc = agent
    status, doc = _raw(netloc, "/v1/plan", json.dumps(body).encode())
    assert status in (200, 400, 403), (status, doc)
