"""Node-agent security (``node/security.py``, VERDICT r2 "secure the node agent").

* plain HTTP is refused off loopback (server and client side);
* each node has its own token, derived from the manager secret: node A's token is
  refused by node B;
* an agent image outside the node's allow-list is refused before any step runs;
* the client trusts only the manager's CA;
* the whole create path (DirectExecutor -> agents -> readiness gate) runs over TLS with
  per-node tokens from the backend-held PKI.
"""

import json
import os
import subprocess
import sys

import pytest

from triton_kubernetes_amd.backend import LocalBackend, MemoryBackend
from triton_kubernetes_amd.cloud.http import HTTPClient, HTTPError
from triton_kubernetes_amd.errors import ExecutorError, TKError
from triton_kubernetes_amd.node.agent import NodeAgent
from triton_kubernetes_amd.node.plan import build_host_plan
from triton_kubernetes_amd.node.security import (AgentPKI, AgentPolicy, agent_address, load_pki, read_credentials,
                                                 PKI_BLOB)
from triton_kubernetes_amd.parallel.transport import AgentTransport, HostRef
from triton_kubernetes_amd.versions import AGENT_IMAGE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = {"hostname": "w-1", "rancher_host_labels": {"worker": "true"}}


@pytest.fixture(scope="module")
def pki():
    return AgentPKI.create("mgr")


def _agent(pki, tmp_path, address, images=(AGENT_IMAGE,), servers=()):
    d = str(tmp_path / f"creds-{address}")
    pki.issue(address, list(images), servers=list(servers)).write(d)
    creds = read_credentials(d)
    agent = NodeAgent(name=address, mode="sim", token=creds["token"], root=str(tmp_path / address),
                      policy=creds["policy"])
    url = agent.serve(address, ssl_context=creds["ssl_context"])
    return agent, url


def test_credentials_files_and_token_derivation(pki, tmp_path):
    creds = pki.issue("10.0.0.5", [AGENT_IMAGE])
    files = creds.write(str(tmp_path / "c"))
    assert sorted(os.path.basename(f) for f in files) == sorted(
        ["agent-token", "agent.crt", "agent.key", "ca.crt", "agent-policy.json"])
    assert all(os.stat(f).st_mode & 0o077 == 0 for f in files)
    assert creds.token == pki.node_token("agent+https://10.0.0.5:7946") == pki.node_token("10.0.0.5")
    assert pki.node_token("10.0.0.6") != creds.token
    assert AgentPKI.create("mgr").node_token("10.0.0.5") != creds.token  # another manager's secret
    # the certificate names the node's address
    out = subprocess.run(["openssl", "x509", "-noout", "-ext", "subjectAltName"], input=creds.cert_pem,
                         capture_output=True, text=True).stdout
    assert "IP Address:10.0.0.5" in out
    assert agent_address("agent+https://[::1]:7946") == "::1"


def test_plain_http_refused_off_loopback(pki):
    agent = NodeAgent(name="x", mode="sim", token="t" * 20)
    with pytest.raises(ValueError, match="refusing to serve plain HTTP on 10.1.2.3"):
        agent.serve("10.1.2.3", 0)
    # the daemon: --insecure-local only on loopback; no credentials and no flag -> refused
    for argv, msg in ((["--listen", "10.1.2.3:7946", "--insecure-local"], "loopback only"),
                      (["--listen", "10.1.2.3:7946"], "--credentials DIR is required")):
        p = subprocess.run([sys.executable, "-m", "triton_kubernetes_amd.node.agent", *argv], capture_output=True,
                           text=True, cwd=ROOT, timeout=60)
        assert p.returncode == 2 and msg in p.stderr, p.stderr
    # the client side, with the manager's PKI: an http:// agent off loopback is refused
    with pytest.raises(ExecutorError, match="refusing plain HTTP"):
        AgentTransport(pki=pki).post(HostRef("agent+http://10.1.2.3:7946"), "/v1/info", {})


def test_other_nodes_token_refused(pki, tmp_path):
    a, url_a = _agent(pki, tmp_path, "127.1.9.2")
    b, url_b = _agent(pki, tmp_path, "127.1.9.3")
    try:
        assert url_b.startswith("https://127.1.9.3:")
        ctx = pki.client_context()
        good = HTTPClient(base_url=url_b, ssl_context=ctx, default_headers={"X-TK-Agent-Token": b.token})
        assert good.get_json("/v1/info")["name"] == "127.1.9.3"
        stolen = HTTPClient(base_url=url_b, ssl_context=ctx, retries=0,
                            default_headers={"X-TK-Agent-Token": a.token})
        with pytest.raises(HTTPError) as exc:
            stolen.get_json("/v1/info")
        assert exc.value.status == 401
        # the CLI's transport derives each node's own token: both work
        tr = AgentTransport(pki=pki)
        for url in (url_a, url_b):
            assert tr._client(HostRef("agent+" + url)).get_json("/v1/info")["pending_gates"] == 0
    finally:
        a.stop()
        b.stop()


def test_unlisted_image_refused_before_any_step(pki, tmp_path):
    agent, url = _agent(pki, tmp_path, "127.1.9.4", images=["rancher/rancher-agent@sha256:" + "ab" * 32])
    try:
        tr = AgentTransport(pki=pki)
        plan = build_host_plan(dict(WORKER, k8s_distribution="rke1", rancher_agent_image="evil/agent:latest"),
                               "https://r", "tok", "sum")
        with pytest.raises(HTTPError) as exc:
            tr.run_plan(HostRef("agent+" + url), plan)
        assert exc.value.status == 403 and "allow-list" in exc.value.body.decode()
        # the tag of the pinned repository is not the pinned digest either
        plan2 = build_host_plan(dict(WORKER, k8s_distribution="rke1", rancher_agent_image="rancher/rancher-agent:v2.8.5"),
                                "https://r", "t", "s")
        with pytest.raises(HTTPError):
            tr.run_plan(HostRef("agent+" + url), plan2)
        assert agent.history == []  # nothing ran
    finally:
        agent.stop()


def test_rke2_join_only_through_an_allowed_server(pki, tmp_path):
    """An RKE2 plan runs the installer of its Rancher server: a server outside the node's
    allow-list (a plan pointing the node at someone else's installer) is refused with 403
    before any step; the listed server passes (scheme/host/port compared)."""
    from triton_kubernetes_amd.rancher.fake import FakeRancher

    with FakeRancher.for_manager("mgr", "tk-admin-pw-0123") as rancher:
        agent, url = _agent(pki, tmp_path, "127.1.9.7", servers=[rancher.url + "/"])
        try:
            tr = AgentTransport(pki=pki)
            evil = build_host_plan(WORKER, "https://198.51.100.7", "tok", "sum")
            with pytest.raises(HTTPError) as exc:
                tr.run_plan(HostRef("agent+" + url), evil)
            assert exc.value.status == 403 and "198.51.100.7" in exc.value.body.decode()
            assert agent.history == []
            # the listed server: the plan runs (here the token is unknown to Rancher, so the
            # registration itself fails -- after the installer was fetched from the server)
            res = tr.run_plan(HostRef("agent+" + url), build_host_plan(WORKER, rancher.url, "tok", "sum"))
            assert [s["name"] for s in res["steps"]] == ["firewall", "hostname", "agent"]
            assert not res["ok"] and "401" in res["error"]
        finally:
            agent.stop()
    assert AgentPolicy(servers=["https://r.example"]).allows_server("https://R.example:443/x")
    assert not AgentPolicy(servers=["https://r.example"]).allows_server("http://r.example")
    assert not AgentPolicy().allows_server("http://127.0.0.1:9")
    assert AgentPolicy(loopback_servers=True).allows_server("http://127.0.0.1:9")
    with pytest.raises(TKError):
        AgentPolicy.from_json({"images": [], "servers": ["ftp://x"]})


def test_rke1_plan_to_a_foreign_server_refused(pki, tmp_path):
    """an RKE1 plan with the allow-listed image but a Rancher server the
    node does not list was run (``docker run --privileged ... --server <theirs>``): a
    token holder could hand the node to a Rancher they control.  Both distributions now
    need an allowed server, and a node enrolled for RKE2 refuses RKE1 plans outright."""
    def agent_with(address, **kw):
        d = str(tmp_path / f"creds-{address}")
        pki.issue(address, [AGENT_IMAGE], servers=["https://rancher.example"], **kw).write(d)
        creds = read_credentials(d)
        a = NodeAgent(name=address, mode="sim", token=creds["token"], root=str(tmp_path / address),
                      policy=creds["policy"])
        return a, a.serve(address, ssl_context=creds["ssl_context"])

    tr = AgentTransport(pki=pki)
    any_dist, url = agent_with("127.1.9.8")
    rke2_only, url2 = agent_with("127.1.9.9", distributions=["rke2"])
    try:
        foreign = build_host_plan(dict(WORKER, k8s_distribution="rke1", rancher_agent_image=AGENT_IMAGE),
                                  "https://203.0.113.9", "tok", "sum")
        with pytest.raises(HTTPError) as exc:
            tr.run_plan(HostRef("agent+" + url), foreign)
        assert exc.value.status == 403 and "203.0.113.9" in exc.value.body.decode()
        rke1 = build_host_plan(dict(WORKER, k8s_distribution="rke1", rancher_agent_image=AGENT_IMAGE),
                               "https://rancher.example", "tok", "sum")
        assert any_dist.refusals(rke1) == []  # enrolled for either: listed image and server pass
        with pytest.raises(HTTPError) as exc:
            tr.run_plan(HostRef("agent+" + url2), rke1)
        assert exc.value.status == 403 and "distribution 'rke1'" in exc.value.body.decode()
        assert any_dist.history == [] and rke2_only.history == []
        assert AgentPolicy.from_json(rke2_only.policy.to_json()).distributions == ["rke2"]
        with pytest.raises(TKError):
            AgentPolicy.from_json({"images": [AGENT_IMAGE], "distributions": ["k3s"]})
    finally:
        any_dist.stop()
        rke2_only.stop()


def test_client_trusts_only_the_managers_ca(pki, tmp_path):
    other = AgentPKI.create("someone-else")
    agent, url = _agent(other, tmp_path, "127.1.9.5")
    try:
        c = HTTPClient(base_url=url, ssl_context=pki.client_context(), retries=0,
                       default_headers={"X-TK-Agent-Token": other.node_token("127.1.9.5")})
        with pytest.raises(TKError, match="CERTIFICATE_VERIFY_FAILED"):
            c.get_json("/v1/info")
    finally:
        agent.stop()


def test_stalled_tls_client_does_not_block_others(pki, tmp_path):
    """A client that connects and never handshakes must not block the accept loop."""
    import socket

    agent, url = _agent(pki, tmp_path, "127.1.9.6")
    try:
        host, port = url[len("https://"):].rsplit(":", 1)
        stall = socket.create_connection((host, int(port)))
        c = HTTPClient(base_url=url, ssl_context=pki.client_context(), timeout=5, retries=0,
                       default_headers={"X-TK-Agent-Token": agent.token})
        assert c.get_json("/v1/info")["name"] == "127.1.9.6"
        stall.close()
    finally:
        agent.stop()


def test_pki_lives_in_the_backend_and_is_stable(tmp_path):
    be = LocalBackend(str(tmp_path / "s"))
    p1 = load_pki(be, "mgr")
    assert os.stat(os.path.join(be.root, "mgr", PKI_BLOB)).st_mode & 0o077 == 0
    p2 = load_pki(be, "mgr")
    assert p1.node_token("10.0.0.1") == p2.node_token("10.0.0.1") and p1.ca_cert == p2.ca_cert
    assert load_pki(MemoryBackend(), "x", create=False) is None
    assert AgentPolicy.from_json({"images": ["a:1"]}).allows("a:1")
    with pytest.raises(TKError):
        AgentPolicy.from_json({"images": "a:1"})


def test_create_cluster_over_tls_with_per_node_tokens(tmp_path):
    """The DirectExecutor and the readiness gate reach TLS agents with tokens derived from
    the manager's backend-held PKI (no shared agent_token anywhere)."""
    from triton_kubernetes_amd import workflows as wf
    from triton_kubernetes_amd.node.labels import synthetic_topology
    from triton_kubernetes_amd.rancher.fake import FakeRancher

    from helpers import make_ctx, output

    be = LocalBackend(str(tmp_path / "state"))
    with FakeRancher.for_manager("mgr", "tk-admin-pw-0123") as rancher:
        wf.new_manager(make_ctx({"executor": "direct", "manager_cloud_provider": "baremetal", "name": "mgr",
                                 "rancher_admin_password": "tk-admin-pw-0123", "rancher_bootstrap_password": rancher.bootstrap_password, "host": "rancher+" + rancher.url,
                                 "ssh_user": "u", "bastion_host": "", "key_path": "k"}), be)
        assert be.read_blob("mgr", PKI_BLOB)  # created with the manager (inside its apply lock)
        pki = load_pki(be, "mgr")
        agents = []
        try:
            urls = []
            for i, addr in enumerate(("127.1.8.2", "127.1.8.3")):
                d = str(tmp_path / f"c{i}")
                pki.issue(addr, [AGENT_IMAGE], servers=[rancher.url]).write(d)
                creds = read_credentials(d)
                ag = NodeAgent(name=addr, mode="sim", devices=list(range(8)) if i else [], token=creds["token"],
                               root=str(tmp_path / f"r{i}"), policy=creds["policy"],
                               topology_override=synthetic_topology(8) if i else None,
                               burnin_override=(lambda dev, level: {"ok": True, "simulated": True, "level": level})
                               if i else None)
                agents.append(ag)
                urls.append("agent+" + ag.serve(addr, ssl_context=creds["ssl_context"]))
            ctx = make_ctx({"executor": "direct", "cluster_manager": "mgr", "cluster_cloud_provider": "baremetal",
                            "name": "tls", "k8s_version": "v1.28.10-rancher1-1", "k8s_network_provider": "flannel",
                            "wait": True, "rccl_gate": True, "gpu_addons": True, "nodes": [
                                {"rancher_host_label": "control", "node_count": 1, "hostname": "cp", "ssh_user": "u",
                                 "bastion_host": "", "key_path": "k", "hosts": [urls[0]]},
                                {"rancher_host_label": "etcd", "node_count": 1, "hostname": "etcd", "ssh_user": "u",
                                 "bastion_host": "", "key_path": "k", "hosts": [urls[0]]},
                                {"rancher_host_label": "worker", "node_count": 1, "hostname": "gpu", "ssh_user": "u",
                                 "bastion_host": "", "key_path": "k", "hosts": [urls[1]], "gpu": "mi355x",
                                 "gpu_count": 8}]})
            wf.new_cluster(ctx, be)
            assert "rccl_gate" in output(ctx)
            assert all(url.startswith("agent+https://") for url in urls)
            assert agents[1].history and agents[1].history[-1]["ok"]
        finally:
            for ag in agents:
                ag.stop()


def test_pki_created_inside_the_workflow_lock(tmp_path):
    """The executor creates the PKI while the workflow holds the manager lock: the local
    backend's lock is re-entrant within a thread (no self-deadlock)."""
    import threading
    import time

    be = LocalBackend(str(tmp_path / "s"))
    with be.lock("mgr", timeout=2):
        t0 = time.monotonic()
        pki = load_pki(be, "mgr")
        assert time.monotonic() - t0 < 1.5 and pki is not None
    got = []

    def other():
        with be.lock("mgr", timeout=2):
            got.append(True)

    with be.lock("mgr"):
        t = threading.Thread(target=other)
        t.start()
        time.sleep(0.2)
        assert got == []  # another thread still waits
    t.join()
    assert got == [True]


def test_cli_credentials_node(tmp_path, monkeypatch):
    """``triton-kubernetes credentials node``: the node's files, signed by the manager's CA,
    with the manager's agent image as the allow-list."""
    from triton_kubernetes_amd.cli.main import run
    from triton_kubernetes_amd.state import State
    import io

    home = tmp_path / "home"
    be = LocalBackend(str(home / ".triton-kubernetes"))
    st = State("mgr")
    st.set_manager({"source": "x", "name": "mgr", "rancher_agent_image": "rancher/rancher-agent@sha256:" + "cd" * 32})
    be.persist_state(st)
    monkeypatch.setenv("HOME", str(home))
    monkeypatch.setenv("TRITON_KUBERNETES_HOME", be.root)
    out = io.StringIO()
    cfg = tmp_path / "c.yaml"
    cfg.write_text(f"backend_provider: local\ncluster_manager: mgr\nagent_address: 10.2.3.4\n"
                   f"credentials_dir: {tmp_path / 'creds'}\n")
    rc = run(["--non-interactive", "--config", str(cfg), "credentials", "node"], out=out)
    assert rc == 0, out.getvalue()
    policy = json.loads((tmp_path / "creds" / "agent-policy.json").read_text())
    # no manager state yet: no Rancher server to allow (RKE2 joins refused, and said so)
    assert policy == {"images": ["rancher/rancher-agent@sha256:" + "cd" * 32], "servers": [], "distributions": ["rke2"]}
    assert "cannot join RKE2 clusters" in out.getvalue()
    pki = load_pki(be, "mgr", create=False)
    assert (tmp_path / "creds" / "agent-token").read_text().strip() == pki.node_token("10.2.3.4")
    assert (tmp_path / "creds" / "ca.crt").read_text() == pki.ca_cert
    # once the manager is applied, its rancher_url is the allowed server
    be.write_tfstate("mgr", json.dumps({"version": 4, "outputs": {
        "cluster-manager__rancher_url": {"value": "https://10.9.8.7"}}}).encode())
    rc = run(["--non-interactive", "--config", str(cfg), "credentials", "node"], out=io.StringIO())
    assert rc == 0
    policy = json.loads((tmp_path / "creds" / "agent-policy.json").read_text())
    assert policy["servers"] == ["https://10.9.8.7"]


@pytest.mark.parametrize("extra,msg", [
    (["--devices", "a,b"], "argument --devices"), (["--devices", "0,0"], "given twice"),
    (["--devices", "-1"], "argument --devices"), (["--listen", "nohost"], "argument --listen"),
    (["--listen", "127.0.0.1:99999"], "argument --listen"), (["--synthetic-gpus", "-3"], "argument --synthetic-gpus"),
    (["--token-file", "/nonexistent/token"], "--token-file /nonexistent/token"),
    (["--credentials", "/nonexistent/creds"], "--credentials /nonexistent/creds"),
])
def test_agent_command_line_refusals_are_argparse_errors(tmp_path, capsys, extra, msg):
    """What systemd hands the daemon and it cannot use ends in one usage line and exit 2,
    not a traceback from the middle of the start-up (an RCCL error for `--devices 0,0`)."""
    from triton_kubernetes_amd.node import agent as agent_mod

    argv = ["--mode", "sim", "--root", str(tmp_path)] + (["--insecure-local"] if "--credentials" not in extra else [])
    with pytest.raises(SystemExit) as exc:
        agent_mod.main(argv + extra)
    assert exc.value.code == 2
    err = capsys.readouterr().err
    assert msg in err and "Traceback" not in err, err
