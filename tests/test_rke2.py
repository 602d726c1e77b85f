"""RKE2 custom clusters (the default) next to RKE1 (reference-era documents), end to end.

Rancher v2.10 provisions RKE2 through ``provisioning.cattle.io/v1`` ``Cluster`` objects whose
nodes join by running the server's ``system-agent-install.sh``; the reference's flow (v3
cluster + ``docker run rancher/rancher-agent``, ``create/cluster.go``,
``terraform/modules/files/install_rancher_agent.sh.tpl``) is kept as RKE1.  Every create
path is exercised on both: the DirectExecutor with node agents, the Terraform modules
(document -> module inputs -> planned expressions, preconditions, rendered host scripts),
the CLI's prompts and ``migrate manager``.
"""

import json
import subprocess
import tempfile

import pytest

from triton_kubernetes_amd import versions
from triton_kubernetes_amd.backend import LocalBackend
from triton_kubernetes_amd.errors import ConfigError
from triton_kubernetes_amd.models import baremetal
from triton_kubernetes_amd.models.common import base_cluster_config
from triton_kubernetes_amd.node.agent import NodeAgent
from triton_kubernetes_amd.node.labels import synthetic_topology
from triton_kubernetes_amd.rancher.fake import FakeRancher
from triton_kubernetes_amd.state import State
from triton_kubernetes_amd.terraform import catalog
from triton_kubernetes_amd.terraform.plan import plan_module
from triton_kubernetes_amd.workflows import delete_cluster, new_cluster, new_manager

from helpers import assert_blocks_match_modules, make_ctx, output

TOKEN = "rke2-test-token-0123"
VERSION = {"rke2": "v1.30.10+rke2r1", "rke1": "v1.30.10-rancher1-1"}


@pytest.fixture
def env(tmp_path):
    fake = FakeRancher.for_manager("mgr", "s3cret-passw0rd").start()
    agents = []

    def agent(name, gpus=0):
        a = NodeAgent(name=name, mode="sim", devices=list(range(gpus)), token=TOKEN, root=tempfile.mkdtemp(),
                      topology_override=synthetic_topology(gpus) if gpus else None,
                      burnin_override=lambda d, lvl: {"ok": True})
        agents.append(a)
        return "agent+" + a.serve()

    backend = LocalBackend(str(tmp_path / "state"))
    base = {"executor": "direct", "agent_token": TOKEN}
    new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr",
                              rancher_admin_password="s3cret-passw0rd", rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="ubuntu",
                              bastion_host="", key_path="k")), backend)
    yield fake, agent, backend, base
    for a in agents:
        a.stop()
    fake.stop()


def _nodes(cp, workers):
    common = {"ssh_user": "u", "bastion_host": "", "key_path": "k"}
    return [dict(common, rancher_host_label="control", node_count=1, hostname="cp", hosts=[cp]),
            dict(common, rancher_host_label="etcd", node_count=1, hostname="etcd", hosts=[cp]),
            dict(common, rancher_host_label="worker", node_count=len(workers), hostname="gpu", hosts=workers,
                 gpu="mi355x", gpu_count=8)]


@pytest.mark.parametrize("dist", ["rke2", "rke1"])
def test_bare_metal_and_mi355x_create_on_both_distributions(env, dist):
    fake, agent, backend, base = env
    cp, workers = agent("cp"), [agent("w1", gpus=8), agent("w2", gpus=8)]
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="dev",
                        k8s_version=VERSION[dist], k8s_network_provider="calico", gpu_addons=True, wait=True,
                        rccl_gate=True, nodes=_nodes(cp, workers)))
    new_cluster(ctx, backend)
    out = output(ctx)
    assert "cluster ready in" in out and "rccl_gate" in out
    st = backend.state("mgr")
    assert st.get("module.cluster_baremetal_dev.k8s_distribution") == dist
    # the nodes carry the cluster's distribution by value (how they join)
    assert {st.module(k)["k8s_distribution"] for k in st.nodes("cluster_baremetal_dev").values()} == {dist}
    (cid,) = list(fake.state.clusters)
    if dist == "rke2":
        obj = fake.state.v2_clusters["fleet-default/dev"]
        assert obj["spec"]["kubernetesVersion"] == VERSION["rke2"] and obj["status"]["clusterName"] == cid
        assert obj["spec"]["rkeConfig"]["machineGlobalConfig"]["cni"] == "calico"
        assert cid.startswith("c-m-")
    else:
        assert fake.state.v2_clusters == {}
        assert fake.state.clusters[cid]["rancherKubernetesEngineConfig"]["kubernetesVersion"] == VERSION["rke1"]
    kinds = {n["hostname"]: n["agentKind"] for n in fake.state.nodes.values()}
    assert set(kinds) == {"cp-1", "etcd-1", "gpu-1", "gpu-2"}
    assert set(kinds.values()) == {"system-agent" if dist == "rke2" else "rancher-agent"}
    nodes = {n["metadata"]["name"]: n for n in fake.k8s_nodes(cid)}
    assert nodes["gpu-1"]["status"]["allocatable"]["amd.com/gpu"] == "8"
    assert nodes["gpu-2"]["metadata"]["labels"]["amd.com/gpu.product-name"] == "MI355X"
    # what the GPU node ran: RKE2 has no container-runtime or docker-login step
    tf = json.loads(backend.read_tfstate("mgr"))
    assert tf["module_state"]["addons_baremetal_dev"]["status"] == "ok"
    delete_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_name="dev", rancher_cleanup=True)), backend)
    assert fake.state.clusters == {} and fake.state.v2_clusters == {}


def test_rke2_node_plan_never_touches_docker(env):
    fake, agent, backend, base = env
    cp, w = agent("cp"), agent("w1", gpus=8)
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="dev", k8s_version="v1.31",
                        k8s_network_provider="canal", gpu_addons=False, wait=False, nodes=_nodes(cp, [w])))
    new_cluster(ctx, backend)
    st = backend.state("mgr")
    # a bare minor: the default distribution's pinned release
    assert st.get("module.cluster_baremetal_dev.k8s_distribution") == versions.DEFAULT_DISTRIBUTION == "rke2"
    assert st.get("module.cluster_baremetal_dev.k8s_version") == versions.DEFAULT_K8S_VERSION
    (obj,) = fake.state.v2_clusters.values()
    assert obj["spec"]["kubernetesVersion"] == versions.DEFAULT_K8S_VERSION
    report = ctx.extras["last_apply"]
    for key, run in report.runs.items():
        if key.startswith("node_"):
            names = [s["name"] for s in run.detail["steps"]]
            assert "runtime" not in names and "registry_login" not in names and names[-1] == "agent", names


@pytest.mark.parametrize("dist", ["rke2", "rke1"])
def test_terraform_documents_plan_and_render_per_distribution(dist):
    """The Terraform path: the document's blocks satisfy the modules (validations,
    preconditions, every expression), and the host modules render the right join."""
    st = State("mgr")
    baremetal.new_manager(make_ctx({"name": "mgr", "rancher_admin_password": "long-enough-pw-1", "host": "10.0.0.1",
                                    "ssh_user": "u", "bastion_host": "", "key_path": "k"}), st, "mgr")
    settings = {"name": "dev", "k8s_distribution": dist, "k8s_version": VERSION[dist][:5],
                "k8s_network_provider": "canal"}
    baremetal.new_cluster(make_ctx(settings), None, st)
    assert st.get("module.cluster_baremetal_dev.k8s_version") == versions.normalize_k8s_version(VERSION[dist][:5],
                                                                                                 dist)
    for label, gpu in (("control", "none"), ("worker", "mi355x")):
        baremetal.new_node(make_ctx({"rancher_host_label": label, "node_count": 1, "hostname": label, "gpu": gpu,
                                     "hosts": ["10.0.0.9"], "ssh_user": "u", "bastion_host": "", "key_path": "k",
                                     "gpu_count": 8}), "mgr", "cluster_baremetal_dev", None, st)
    assert_blocks_match_modules(st)
    for key in st.nodes("cluster_baremetal_dev").values():
        block = st.module(key)
        assert block["k8s_distribution"] == dist
        mod = catalog.module_from_source(block["source"]).local_dir
        inputs = dict(block, rancher_cluster_registration_token="tok", rancher_cluster_ca_checksum="ab" * 32,
                      rancher_api_url="https://rancher.example")
        planned = plan_module(mod, inputs, check_files=False)
        assert planned.ok, planned.errors
        (script,) = [t for name, texts in planned.rendered.items() if name.endswith(".sh.tftpl")
                     and ("agent" in name or "mi355x" in name) for t in texts]
        assert subprocess.run(["bash", "-n"], input=script, capture_output=True, text=True).returncode == 0
        if dist == "rke2":
            assert "https://rancher.example/system-agent-install.sh" in script
            assert "--node-name" in script and "docker run" not in script and "get.docker.com" not in script
        else:
            assert "docker run -d --privileged" in script and "system-agent-install" not in script
        if "mi355x" in block["source"]:
            assert " $labels" in script  # the GPU labels travel on the join command


def test_cluster_module_preconditions_catch_mixed_documents():
    mod = catalog.CATALOG["bare-metal-rancher-k8s"].local_dir
    base = {"name": "c", "rancher_api_url": "${module.m.url}", "rancher_access_key": "${module.m.a}",
            "rancher_secret_key": "${module.m.s}"}
    assert plan_module(mod, base).ok  # defaults: RKE2 release, canal
    mixed = plan_module(mod, dict(base, k8s_distribution="rke1"))  # RKE1 with the RKE2 default release
    assert any("precondition failed: k8s_version must be a release of k8s_distribution" in e for e in mixed.errors)
    cni = plan_module(mod, dict(base, k8s_network_provider="weave"))
    assert any("is not a CNI of k8s_distribution" in e for e in cni.errors)
    assert plan_module(mod, dict(base, k8s_distribution="rke1", k8s_version="v1.29.14-rancher1-1",
                                 k8s_network_provider="weave")).ok


def test_interactive_create_asks_for_the_distribution():
    ctx = make_ctx({"name": "dev", "k8s_network_provider": "calico"}, answers=[1, "v1.29", "", ""],
                   non_interactive=False)
    cfg = base_cluster_config(ctx, "terraform/modules/bare-metal-rancher-k8s")
    assert cfg["k8s_distribution"] == "rke1" and cfg["k8s_version"] == "v1.29.14-rancher1-1"
    asked = [label for _, label in ctx.prompter.asked]
    assert asked[:2] == ["Kubernetes Distribution", "Kubernetes Version"]
    # a release string names its distribution: no question
    ctx = make_ctx({"name": "dev", "k8s_version": "v1.31.6+rke2r1", "k8s_network_provider": "cilium"},
                   answers=["", ""], non_interactive=False)
    assert base_cluster_config(ctx, "terraform/modules/bare-metal-rancher-k8s")["k8s_distribution"] == "rke2"
    assert "Kubernetes Distribution" not in [label for _, label in ctx.prompter.asked]
    with pytest.raises(ConfigError, match="not a RKE1 network provider"):
        base_cluster_config(make_ctx({"name": "dev", "k8s_distribution": "rke1", "k8s_version": "v1.29",
                                      "k8s_network_provider": "cilium"}),
                            "terraform/modules/bare-metal-rancher-k8s")


def test_migrated_reference_documents_stay_rke1():
    """A reference-era document (RKE1 clusters, Terraform 0.11 module sources) is migrated
    with k8s_distribution rke1 on its cluster and node blocks."""
    from triton_kubernetes_amd.workflows.migrate import plan_migration

    ref = "github.com/joyent/triton-kubernetes//terraform/modules/{}?ref=master"
    doc = {"module": {
        "cluster-manager": {"source": ref.format("bare-metal-rancher"), "name": "mgr", "host": "10.0.0.1",
                            "rancher_admin_password": "long-enough-pw-1"},
        "cluster_baremetal_dev": {"source": ref.format("bare-metal-rancher-k8s"), "name": "dev",
                                  "rancher_api_url": "${module.cluster-manager.rancher_url}",
                                  "rancher_access_key": "${module.cluster-manager.rancher_access_key}",
                                  "rancher_secret_key": "${module.cluster-manager.rancher_secret_key}",
                                  "k8s_version": "v1.30.10-rancher1-1", "k8s_network_provider": "calico"},
        "node_baremetal_dev_w-1": {"source": ref.format("bare-metal-rancher-k8s-host"), "hostname": "w-1",
                                   "host": "10.0.0.2", "rancher_api_url": "${module.cluster-manager.rancher_url}",
                                   "rancher_cluster_registration_token":
                                       "${module.cluster_baremetal_dev.rancher_cluster_registration_token}",
                                   "rancher_cluster_ca_checksum":
                                       "${module.cluster_baremetal_dev.rancher_cluster_ca_checksum}",
                                   "rancher_host_labels": {"worker": "true"}, "ssh_user": "u", "key_path": "k"}}}
    blocks, errors, warnings = plan_migration(make_ctx({}), doc)
    assert not errors, errors
    assert blocks["cluster_baremetal_dev"]["k8s_distribution"] == "rke1"
    assert blocks["node_baremetal_dev_w-1"]["k8s_distribution"] == "rke1"
    assert "k8s_distribution" not in blocks["cluster-manager"]
    assert any("k8s_distribution set to rke1" in w for w in warnings)
    assert not [w for w in warnings if "precondition" in w], warnings


def test_direct_executor_refuses_a_name_of_the_other_distribution(env):
    fake, agent, backend, base = env
    from triton_kubernetes_amd.rancher.client import RancherClient

    mgr = json.loads(backend.read_tfstate("mgr"))["module_outputs"]["cluster-manager"]
    client = RancherClient(mgr["rancher_url"], mgr["rancher_access_key"], mgr["rancher_secret_key"])
    client.ensure_cluster("taken", distribution="rke1")
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="taken",
                        k8s_version="v1.31", k8s_network_provider="canal",
                        nodes=_nodes(agent("cp"), [agent("w", gpus=8)])))
    with pytest.raises(Exception, match="already exists as an RKE1 cluster"):
        new_cluster(ctx, backend)
    assert fake.state.v2_clusters == {}


def test_exec_mode_agent_runs_the_servers_installer(tmp_path, monkeypatch):
    """``exec`` mode (the production agent): the RKE2 join downloads the allowed server's
    system-agent-install.sh and runs it with a fixed argv (no shell text from the plan)."""
    from triton_kubernetes_amd.node.plan import build_host_plan
    from triton_kubernetes_amd.parallel.transport import AgentTransport, HostRef

    bindir = tmp_path / "bin"
    bindir.mkdir()
    log = tmp_path / "calls.log"
    stub = bindir / "hostnamectl"
    stub.write_text(f'#!/bin/sh\necho "hostnamectl $*" >> {log}\n')
    stub.chmod(0o755)
    monkeypatch.setenv("PATH", f"{bindir}:/usr/bin:/bin")
    monkeypatch.setenv("TK_FAKE_SYSTEM_AGENT_LOG", str(log))
    with FakeRancher() as fake:
        cid, token, checksum = fake.registration()
        agent = NodeAgent(name="x", mode="exec", token=TOKEN, root=str(tmp_path / "root"))
        url = agent.serve()
        try:
            plan = build_host_plan({"hostname": "w-1", "rancher_host_labels": {"worker": "true"}}, fake.url,
                                   token, checksum)
            res = AgentTransport(token=TOKEN).run_plan(HostRef("agent+" + url), plan)
            # the installer verified the CA checksum and registered the node as a system agent
            (node,) = fake.state.cluster_nodes[cid].values()
            assert node["hostname"] == "w-1" and node["agentKind"] == "system-agent" and node["roles"]["worker"]
            # a wrong checksum stops the installer before it registers anything
            bad = build_host_plan({"hostname": "w-2", "rancher_host_labels": {"worker": "true"}}, fake.url, token,
                                  "0" * 64)
            res_bad = AgentTransport(token=TOKEN).run_plan(HostRef("agent+" + url), bad)
            assert not res_bad["ok"] and "does not match --ca-checksum" in res_bad["error"]
            assert len(fake.state.cluster_nodes[cid]) == 1
        finally:
            agent.stop()
    assert res["ok"], res
    calls = log.read_text()
    assert "hostnamectl set-hostname w-1" in calls
    assert (f"system-agent-install --server {fake.url} --label cattle.io/os=linux --token {token} "
            f"--ca-checksum {checksum} --node-name w-1 --worker") in calls


def test_exec_join_without_a_ca_checksum(tmp_path, monkeypatch):
    """A server with a publicly trusted certificate reports no CA and no checksum: the
    agent joins without --ca-checksum instead of refusing the empty value."""
    from triton_kubernetes_amd.node.plan import build_host_plan
    from triton_kubernetes_amd.parallel.transport import AgentTransport, HostRef

    bindir = tmp_path / "bin"
    bindir.mkdir()
    log = tmp_path / "calls.log"
    (bindir / "hostnamectl").write_text(f'#!/bin/sh\necho "hostnamectl $*" >> {log}\n')
    (bindir / "hostnamectl").chmod(0o755)
    monkeypatch.setenv("PATH", f"{bindir}:/usr/bin:/bin")
    monkeypatch.setenv("TK_FAKE_SYSTEM_AGENT_LOG", str(log))
    with FakeRancher() as fake:
        cid, token, _ = fake.registration()
        agent = NodeAgent(name="x", mode="exec", token=TOKEN, root=str(tmp_path / "root"))
        url = agent.serve()
        try:
            plan = build_host_plan({"hostname": "w-1", "rancher_host_labels": {"worker": "true"}}, fake.url,
                                   token, "")
            res = AgentTransport(token=TOKEN).run_plan(HostRef("agent+" + url), plan)
        finally:
            agent.stop()
        assert [n["hostname"] for n in fake.state.cluster_nodes[cid].values()] == ["w-1"]
    assert res["ok"], res
    calls = log.read_text()
    assert f"--token {token} --node-name w-1 --worker" in calls and "--ca-checksum" not in calls


def _https_rancher(tmp_path, cacerts_body: bytes):
    """A TLS server standing in for Rancher's installer endpoints, its certificate for
    127.0.0.1 signed by a CA whose PEM ``/cacerts`` serves (or ``cacerts_body``)."""
    import http.server
    import threading

    from triton_kubernetes_amd.k8s.tls import issue, make_ca
    from triton_kubernetes_amd.node.security import server_context

    ca = make_ca("rancher-test-ca")
    cert = issue(ca, "127.0.0.1", ["127.0.0.1"])
    body = cacerts_body if cacerts_body is not None else ca.cert_pem.encode()

    class H(http.server.BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_GET(self):
            data = body if self.path == "/cacerts" else b"#!/bin/sh\necho installed\n"
            self.send_response(200)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    srv.socket = server_context(cert.cert_pem, cert.key_pem).wrap_socket(srv.socket, server_side=True)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv, f"https://127.0.0.1:{srv.server_address[1]}", body


@pytest.mark.parametrize("tamper", [False, True])
def test_installer_fetched_over_tls_pinned_by_the_ca_checksum(tmp_path, tamper):
    """The RKE2 join trusts the installer only over TLS verified against the CA whose
    sha256 is the cluster's --ca-checksum (agent and shell paths alike)."""
    import hashlib

    from triton_kubernetes_amd.node.plan import BootstrapPlan, build_host_plan

    srv, url, pem = _https_rancher(tmp_path, None)
    try:
        checksum = hashlib.sha256(pem).hexdigest() if not tamper else "0" * 64
        agent = NodeAgent(name="x", mode="sim", token=TOKEN, root=str(tmp_path / "r"))
        plan = BootstrapPlan("w-1", "worker", url, "tok", checksum, distribution="rke2")
        if tamper:
            with pytest.raises(RuntimeError, match="does not match the cluster's CA checksum"):
                agent._fetch_installer(plan)
        else:
            assert agent._fetch_installer(plan).startswith(b"#!/bin/sh")
        agent.stop()
        # the rendered shell step: real curl against the TLS server, sudo stubbed
        bindir = tmp_path / "bin"
        bindir.mkdir()
        log = tmp_path / "sudo.log"
        # drains stdin like the real command would (a step's stdin is /dev/null; `printf | sudo
        # tee` must not see its reader exit early: SIGPIPE under pipefail failed the step)
        (bindir / "sudo").write_text(f'#!/bin/sh\necho "$*" >> {log}\ncat >/dev/null 2>&1 || true\n')
        (bindir / "sudo").chmod(0o755)
        shell_plan = build_host_plan({"hostname": "w-1", "rancher_host_labels": {"worker": "true"}}, url, "tok",
                                     checksum)
        from triton_kubernetes_amd.parallel.transport import HostRef, LocalTransport

        res = LocalTransport(env={"PATH": f"{bindir}:/usr/bin:/bin"}).run_plan(HostRef("local"), shell_plan)
        ran = log.exists() and "--server" in log.read_text()
        assert res["ok"] is (not tamper) and ran is (not tamper), res
    finally:
        srv.shutdown()
