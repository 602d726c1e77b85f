"""DirectExecutor end to end against the fake Rancher and sim-mode node agents.

The executor path is the one ``bench.py`` times; here the GPU steps use a
synthetic 8xMI355X topology and a stubbed burn-in so the test runs on CPU.
"""

import json
import tempfile

import pytest

from triton_kubernetes_amd.backend import LocalBackend
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.executor.direct import DirectExecutor, module_deps, resolve
from triton_kubernetes_amd.node.agent import NodeAgent
from triton_kubernetes_amd.node.labels import synthetic_topology
from triton_kubernetes_amd.parallel.transport import AgentTransport, RecordingTransport, TransportRouter
from triton_kubernetes_amd.rancher.client import RancherClient
from triton_kubernetes_amd.rancher.fake import FakeRancher
from triton_kubernetes_amd.workflows import delete_cluster, delete_node, get_cluster, get_manager, new_cluster
from triton_kubernetes_amd.workflows import new_manager, new_node

from helpers import make_ctx, output

TOKEN = "test-token-123456"


@pytest.fixture
def env(tmp_path):
    fake = FakeRancher.for_manager("mgr", "s3cret-passw0rd").start()
    agents = []

    def agent(name, gpus=0, fail_burnin=False):
        a = NodeAgent(name=name, mode="sim", devices=list(range(gpus)), token=TOKEN, root=tempfile.mkdtemp(),
                      topology_override=synthetic_topology(gpus) if gpus else None,
                      burnin_override=lambda d, l: {"ok": not fail_burnin, "failures": ["hbm"] if fail_burnin else []})
        agents.append(a)
        return "agent+" + a.serve()

    backend = LocalBackend(str(tmp_path / "state"))
    base = {"executor": "direct", "agent_token": TOKEN}
    yield fake, agent, backend, base
    for a in agents:
        a.stop()
    fake.stop()


def _manager(fake, backend, base):
    new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr", rancher_admin_password="s3cret-passw0rd",
                              rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="ubuntu", bastion_host="", key_path="k")),
                backend)


def _nodes(cp, workers, gpu=True, count=8):
    return [
        {"rancher_host_label": "control", "node_count": 1, "hostname": "cp", "ssh_user": "u", "bastion_host": "",
         "key_path": "k", "hosts": [cp]},
        {"rancher_host_label": "etcd", "node_count": 1, "hostname": "etcd", "ssh_user": "u", "bastion_host": "",
         "key_path": "k", "hosts": [cp]},
        {"rancher_host_label": "worker", "node_count": len(workers), "hostname": "gpu", "ssh_user": "u",
         "bastion_host": "", "key_path": "k", "hosts": workers, **({"gpu": "mi355x", "gpu_count": count}
                                                                    if gpu else {})},
    ]


def test_full_bringup_with_gpu_addons_and_wait(env):
    fake, agent, backend, base = env
    _manager(fake, backend, base)
    assert fake.state.admin_password == "s3cret-passw0rd"  # S3: password changed
    cp = agent("cp")
    workers = [agent(f"w{i}", gpus=8) for i in range(3)]
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="dev",
                        k8s_version="v1.28.10-rancher1-1", k8s_network_provider="calico", gpu_addons=True, wait=True,
                        nodes=_nodes(cp, workers)))
    new_cluster(ctx, backend)
    out = output(ctx)
    assert "3 nodes added: gpu-1, gpu-2, gpu-3" in out
    assert "cluster ready in" in out and "gpus_allocatable" in out
    cid = list(fake.state.clusters)[0]
    nodes = {n["metadata"]["name"]: n for n in fake.k8s_nodes(cid)}
    assert nodes["gpu-1"]["status"]["allocatable"]["amd.com/gpu"] == "8"
    labels = nodes["gpu-2"]["metadata"]["labels"]
    assert labels["amd.com/gpu.product-name"] == "MI355X"
    assert labels["amd.com/xgmi.fully-connected"] == "true" and labels["amd.com/xgmi.links-per-gpu"] == "7"
    assert fake.state.clusters[cid]["rancherKubernetesEngineConfig"]["network"]["plugin"] == "calico"
    tf = json.loads(backend.read_tfstate("mgr"))
    assert tf["module_state"]["addons_baremetal_dev"]["status"] == "ok"
    assert json.loads(tf["module_outputs"]["node_baremetal_dev_gpu-1"]["gpu_node_labels"])["amd.com/gpu.count"] == "8"

    # get manager / cluster work without terraform (tfstate written by the executor)
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_name="dev"))
    get_cluster(ctx, backend)
    assert f"rancher_cluster_id = {cid}" in output(ctx)
    ctx = make_ctx(dict(base, cluster_manager="mgr"))
    get_manager(ctx, backend)
    assert f"rancher_url = {fake.url}" in output(ctx)

    # re-apply on `create node`: only the new node runs, the rest is skipped
    w4 = agent("w4", gpus=8)
    new_node(make_ctx(dict(base, cluster_manager="mgr", cluster_name="dev", rancher_host_label="worker",
                           node_count=1, hostname="gpu", ssh_user="u", bastion_host="", key_path="k", hosts=[w4],
                           gpu="mi355x")), backend)
    tf2 = json.loads(backend.read_tfstate("mgr"))
    assert tf2["module_state"]["node_baremetal_dev_gpu-4"]["status"] == "ok"
    assert tf2["module_state"]["node_baremetal_dev_gpu-1"]["applied_at"] == \
        tf["module_state"]["node_baremetal_dev_gpu-1"]["applied_at"]

    cid = next(iter(fake.state.clusters))
    assert any(n["hostname"] == "gpu-4" for n in fake.state.cluster_nodes[cid].values())
    dn = make_ctx(dict(base, cluster_manager="mgr", cluster_name="dev", hostname="gpu-4", rancher_cleanup=True))
    delete_node(dn, backend)
    assert "node_baremetal_dev_gpu-4" not in json.loads(backend.read_tfstate("mgr"))["module_outputs"]
    # Q7 extension: the node's Rancher object is gone too (and with it the k8s node)
    assert not any(n["hostname"] == "gpu-4" for n in fake.state.cluster_nodes[cid].values())
    assert "gpu-4" not in {n["metadata"]["name"] for n in fake.k8s_nodes(cid)}
    assert "Removed Rancher node" in output(dn)
    delete_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_name="dev", rancher_cleanup=True)), backend)
    assert backend.state("mgr").clusters() == {}
    assert fake.state.clusters == {}  # Q7 extension: Rancher object removed


def test_failed_node_blocks_addons_and_resume(env):
    fake, agent, backend, base = env
    _manager(fake, backend, base)
    cp = agent("cp")
    good, bad = agent("good", gpus=8), agent("bad", gpus=8, fail_burnin=True)
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="dev",
                        k8s_version="v1.28.10-rancher1-1", k8s_network_provider="flannel", gpu_addons=True,
                        nodes=_nodes(cp, [good, bad])))
    with pytest.raises(TKError) as exc:
        new_cluster(ctx, backend)
    assert "gpu_burnin" in str(exc.value) and "hbm" in str(exc.value)
    tf = json.loads(backend.read_tfstate("mgr"))
    assert tf["module_state"]["node_baremetal_dev_gpu-2"]["status"] == "failed"
    assert tf["module_state"]["node_baremetal_dev_gpu-1"]["status"] == "ok"
    assert "addons_baremetal_dev" not in tf["module_state"]  # blocked, never started
    assert "cluster_baremetal_dev" in backend.state("mgr").clusters().values()  # persisted for resume


def test_dag_and_interpolation_helpers():
    cfg = {"a": "${module.cluster-manager.rancher_url}/x", "b": ["${module.cluster_b_c.rancher_cluster_id}"],
           "c": {"d": 1}}
    assert module_deps(cfg) == {"cluster-manager", "cluster_b_c"}
    out = resolve(cfg, {"cluster-manager": {"rancher_url": "https://r"}, "cluster_b_c": {"rancher_cluster_id": "c-1"}})
    assert out == {"a": "https://r/x", "b": ["c-1"], "c": {"d": 1}}
    with pytest.raises(TKError):
        resolve(cfg, {})


def test_unsupported_module_and_parallel_fanout(env):
    fake, agent, backend, base = env
    from triton_kubernetes_amd.state import State

    st = State("x")
    st.add_cluster("aws", "c", {"source": "g//terraform/modules/aws-rancher-k8s?ref=m", "name": "c"})
    with pytest.raises(TKError) as exc:
        DirectExecutor(transport=RecordingTransport()).apply(st, backend)
    assert "does not implement module" in str(exc.value)

    # 40 hosts with a 0.2 s bootstrap each: concurrent fan-out, not Terraform's waves of 10
    _manager(fake, backend, base)
    client = RancherClient(fake.url)
    rec = RecordingTransport(delay=0.2)
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="wide",
                        k8s_version="v1.28.10-rancher1-1", k8s_network_provider="flannel",
                        nodes=[{"rancher_host_label": "worker", "node_count": 40, "hostname": "w", "ssh_user": "u",
                                "bastion_host": "", "key_path": "k", "hosts": [f"10.1.0.{i}" for i in range(40)]}]))
    ctx.extras["transport"] = TransportRouter(ssh=rec, agent=AgentTransport(token=TOKEN))
    import time

    t0 = time.time()
    new_cluster(ctx, backend)
    assert len(rec.plans) == 40
    assert time.time() - t0 < 5.0, "node bootstrap must fan out concurrently (one by one: 8 s)"
    assert client.ping()


def test_pipelined_rccl_gate_through_agents(env):
    """wait + rccl_gate: the gate's communicators are prepared with the apply and run after readiness."""
    fake, agent, backend, base = env
    _manager(fake, backend, base)
    cp = agent("cp")
    workers = [agent(f"w{i}", gpus=8) for i in range(3)]
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="gate",
                        k8s_version="v1.28.10-rancher1-1", k8s_network_provider="calico", gpu_addons=True, wait=True,
                        rccl_gate=True, nodes=_nodes(cp, workers)))
    from triton_kubernetes_amd.utils.trace import TRACER

    TRACER.reset()
    new_cluster(ctx, backend)
    spans = TRACER.report()["spans"]
    gates = [s for s in spans if s["name"] == "node.rccl_gate"]
    assert len(gates) == 3 and all(s["attrs"]["pipelined"] for s in gates)
    assert sorted(s["attrs"]["rank"] for s in gates) == [0, 8, 16]
    assert {s["attrs"]["world"] for s in gates} == {24}
    prep = [s for s in spans if s["name"] == "gate.prepare"]
    assert len(prep) == 1
    assert "rccl_gate" in output(ctx)


def test_gate_released_when_apply_fails(env):
    fake, agent, backend, base = env
    _manager(fake, backend, base)
    cp = agent("cp")
    good = agent("good", gpus=8)
    bad = agent("bad", gpus=8, fail_burnin=True)
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="fail",
                        k8s_version="v1.28.10-rancher1-1", k8s_network_provider="calico", gpu_addons=True, wait=True,
                        rccl_gate=True, nodes=_nodes(cp, [good, bad])))
    with pytest.raises(TKError):
        new_cluster(ctx, backend)
    # the prepared communicators were released on every agent
    from triton_kubernetes_amd.cloud.http import HTTPClient

    for h in (good, bad):
        info = HTTPClient(base_url=h[len("agent+"):]).request("GET", "/v1/info",
                                                             headers={"X-TK-Agent-Token": TOKEN}).json()
        assert info["pending_gates"] == 0


def test_host_retry_recovers_flaky_node(env):
    fake, agent, backend, base = env
    _manager(fake, backend, base)
    calls = {"n": 0}
    a = NodeAgent(name="flaky", mode="sim", devices=list(range(8)), token=TOKEN, root=tempfile.mkdtemp(),
                  topology_override=synthetic_topology(8))

    def burn(dev, level):
        calls["n"] += 1
        return {"ok": calls["n"] > 8, "failures": ["hbm"] if calls["n"] <= 8 else []}  # first pass fails

    a.burnin_override = burn
    url = "agent+" + a.serve()
    try:
        cp = agent("cp")
        events = []
        ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="retry",
                            k8s_version="v1.28.10-rancher1-1", k8s_network_provider="calico", host_retries=2,
                            host_retry_backoff="0.01", nodes=_nodes(cp, [url])))
        new_cluster(ctx, backend)
        tf = json.loads(backend.read_tfstate("mgr"))
        assert tf["module_state"]["node_baremetal_retry_gpu-1"]["status"] == "ok"
        assert calls["n"] == 16  # 8 GPUs failed once, then 8 passed
        # without retries the same flake fails the apply
        calls["n"] = 0
        ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="noretry",
                            k8s_version="v1.28.10-rancher1-1", k8s_network_provider="calico",
                            nodes=_nodes(cp, [url])))
        with pytest.raises(TKError):
            new_cluster(ctx, backend)
        del events
    finally:
        a.stop()


# --- create cost independent of the clusters already on the manager -------------------------------------


def _plain_tfstate(doc):
    from triton_kubernetes_amd.executor.tfstate import derived_outputs

    full = dict(doc)
    full["outputs"] = derived_outputs(doc["module_outputs"])
    return json.dumps(full, indent=2, sort_keys=True).encode()


def test_tfstate_codec_bytes_and_reuse():
    from triton_kubernetes_amd.executor.tfstate import TfstateCodec

    codec = TfstateCodec()
    doc = {"version": 4, "serial": 1, "lineage": "l", "resources": [], "terraform_version": "t",
           "module_outputs": {}, "module_state": {}}
    assert codec.dumps("m", doc) == _plain_tfstate(doc)
    for i in range(30):
        key = f"node_baremetal_c{i // 5}_h-{i}"
        doc["module_outputs"][key] = {"gpu_node_labels": json.dumps({"amd.com/gpu<&>": i}), "z": "é "}
        doc["module_state"][key] = {"hash": f"{i:016x}", "status": "ok", "applied_at": 1.5 + i, "source": None}
        if i % 7 == 0:
            assert codec.dumps("m", doc) == _plain_tfstate(doc)
    # replaced (not edited) entries and removed ones are picked up
    doc["module_state"]["node_baremetal_c0_h-0"] = {"hash": "x", "status": "failed", "error": "boom"}
    doc["module_outputs"]["node_baremetal_c0_h-1"] = {"gpu_node_labels": "{}"}
    doc["module_outputs"].pop("node_baremetal_c0_h-2")
    doc["module_state"].pop("node_baremetal_c0_h-3")
    raw = codec.dumps("m", doc)
    assert raw == _plain_tfstate(doc)
    # a load of the bytes just saved reuses the document (no "outputs": derived on save) ...
    again = codec.load("m", raw)
    assert again["module_state"] == doc["module_state"] and "outputs" not in again
    again["module_state"]["new"] = {"hash": "n", "status": "ok"}
    assert "new" not in doc["module_state"]  # the copy's sections are its own
    # ... and other bytes are parsed
    other = codec.load("m", _plain_tfstate(dict(doc, serial=99)))
    assert other["serial"] == 99 and other["module_outputs"] == doc["module_outputs"]
    assert codec.load("m", b"not json") is None and codec.load("m", b'{"version": 4}') is None


def test_fingerprint_matches_hash_and_deps():
    from triton_kubernetes_amd.executor.direct import config_hash, fingerprint

    cfgs = [{}, {"a": "${module.cluster-manager.rancher_url}", "q": "say \"${module.x_y.z}\" \\ é"},
            {"n": [1, {"m": "${module.node_b_c_h.out}x${module.cluster_b_c.id}"}], "u": None, "f": 1.5}]
    for cfg in cfgs:
        assert fingerprint(cfg) == (config_hash(cfg), module_deps(cfg))


def test_fake_rancher_settles_clusters(env):
    fake, agent, backend, base = env
    _manager(fake, backend, base)
    for name in ("one", "two"):  # a host is a node of one cluster at a time: its own hosts each
        new_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name=name,
                                  k8s_version="v1.28.10-rancher1-1", k8s_network_provider="flannel", wait=True,
                                  nodes=_nodes(agent(f"{name}-cp"), [agent(f"{name}-w", gpus=8)]))), backend)
    # a settled cluster is no longer walked by the simulation; each cluster lists its own nodes
    assert fake.state.unsettled == set()
    cids = {c["name"]: c["id"] for c in fake.state.clusters.values()}
    assert {n["metadata"]["name"] for n in fake.k8s_nodes(cids["two"])} == {"cp-1", "etcd-1", "gpu-1"}
    user, _, secret = RancherClient(fake.url).login("admin", "s3cret-passw0rd").partition(":")
    client = RancherClient(fake.url, user, secret)
    assert {n["clusterId"] for n in client.nodes(cids["one"])} == {cids["one"]}


def test_tfstate_codec_foreign_shapes_fall_back_to_plain_encoding():
    from triton_kubernetes_amd.executor.tfstate import TfstateCodec

    codec = TfstateCodec()
    # module_outputs entries that are not objects, or non-string keys: plain json.dumps
    odd = {"version": 4, "serial": 1, "module_outputs": {"m": "not-a-dict"}, "module_state": {"m": {"status": "ok"}}}
    assert json.loads(codec.dumps("x", odd)) == odd
    assert codec.load("x", codec.dumps("x", odd)) is not None  # parsed, not served from the cache
    keyed = {"version": 4, "module_outputs": {}, "module_state": {1: {"status": "ok"}}}
    assert json.loads(codec.dumps("y", keyed))["module_state"] == {"1": {"status": "ok"}}
    codec.forget("x")
    codec.forget("never-saved")


def test_fake_rancher_node_delete_keeps_cluster_index(env):
    fake, agent, backend, base = env
    _manager(fake, backend, base)
    cp = agent("cp")
    new_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="dev",
                              k8s_version="v1.28.10-rancher1-1", k8s_network_provider="flannel", wait=True,
                              nodes=_nodes(cp, [agent("w", gpus=8)]))), backend)
    cid = next(iter(fake.state.clusters))
    user, _, secret = RancherClient(fake.url).login("admin", "s3cret-passw0rd").partition(":")
    client = RancherClient(fake.url, user, secret)
    gpu = next(n for n in client.nodes(cid) if n["hostname"] == "gpu-1")
    client.http.request("DELETE", f"/v3/nodes/{gpu['id']}", ok=(200,))
    assert {n["metadata"]["name"] for n in fake.k8s_nodes(cid)} == {"cp-1", "etcd-1"}
    assert gpu["id"] not in fake.state.nodes and gpu["id"] not in fake.state.cluster_nodes[cid]


def test_direct_executor_refuses_what_terraform_would(env):
    """A document edited by hand (or written by another tool) with a value a module's
    validation refuses: `terraform plan` would stop with "Invalid value for variable", and
    the DirectExecutor stops the same way, before it touches a host."""
    fake, agent, backend, base = env
    _manager(fake, backend, base)
    rec = RecordingTransport()
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="c1",
                        k8s_version="v1.28.10-rancher1-1", k8s_network_provider="flannel",
                        nodes=[{"rancher_host_label": "worker", "node_count": 1, "hostname": "g", "ssh_user": "u",
                                "bastion_host": "", "key_path": "k", "hosts": ["10.1.0.1"], "gpu": "mi355x",
                                "gpu_count": 8}]))
    ctx.extras["transport"] = TransportRouter(ssh=rec, agent=AgentTransport(token=TOKEN))
    new_cluster(ctx, backend)
    st = backend.state("mgr")
    key = next(k for k, m in st.modules().items() if "mi355x-rancher-k8s-host" in str(m.get("source")))
    mod = dict(st.module(key))
    mod["rccl_env"] = dict(mod.get("rccl_env") or {}, NCCL_NET_PLUGIN="/tmp/evil.so")
    st.set_module(key, mod)
    plans_before = len(rec.plans)
    with pytest.raises(TKError, match="rccl_env"):
        DirectExecutor(transport=TransportRouter(ssh=rec, agent=AgentTransport(token=TOKEN))).apply(st, backend)
    assert len(rec.plans) == plans_before


def test_apply_after_upgrade_accepts_pre_r4_module_hashes(env):
    """module hashes persisted before the hash covered the module's identity (it
    covered the source string the module was applied from) still match: the first apply
    after an upgrade re-runs no module -- no host bootstrap on nodes in service."""
    from triton_kubernetes_amd.executor.direct import fingerprint

    fake, agent, backend, base = env
    _manager(fake, backend, base)
    cp = agent("cp")
    workers = [agent("w0", gpus=8)]
    new_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_name="dev", cluster_cloud_provider="baremetal",
                              name="dev", k8s_version="v1.28.10-rancher1-1", k8s_network_provider="calico",
                              nodes=_nodes(cp, workers))), backend)
    state_doc = {"module": backend.state("mgr").modules()}
    tf = json.loads(backend.read_tfstate("mgr"))
    # rewrite the tfstate as round 3 wrote it: sources at an absolute install path, hashes over them
    old_root = "/usr/lib/python3/dist-packages/triton_kubernetes_amd/terraform/modules"
    for key, entry in tf["module_state"].items():
        cfg = state_doc["module"][key]
        name = cfg["source"].split("?")[0].rstrip("/").rsplit("/", 1)[-1]
        legacy_src = f"{old_root}/{name}"
        entry["source"] = legacy_src
        entry["hash"] = fingerprint(dict(cfg, source=legacy_src))[0]
    from triton_kubernetes_amd.executor.tfstate import CODEC

    backend.write_tfstate("mgr", CODEC.dumps("mgr", tf))
    before = {k: v["applied_at"] for k, v in tf["module_state"].items()}

    ex = DirectExecutor(transport=TransportRouter(agent=AgentTransport(token=TOKEN)))
    report = ex.apply_report(backend.state("mgr"), backend)
    assert report.ok and {r.status for r in report.runs.values()} == {"skipped"}
    after = json.loads(backend.read_tfstate("mgr"))["module_state"]
    assert {k: v["applied_at"] for k, v in after.items()} == before
    # stored in today's form: the next apply matches directly
    assert all(after[k]["hash"] == report.runs[k].hash for k in after)

    # a changed config is still re-applied (the legacy form is not a blanket pass)
    st = backend.state("mgr")
    for key in list(after):
        tf2 = json.loads(backend.read_tfstate("mgr"))
        e = tf2["module_state"][key]
        e["hash"] = "0" * 16
        backend.write_tfstate("mgr", CODEC.dumps("mgr", tf2))
        break
    rep2 = ex.apply_report(st, backend)
    assert rep2.runs[key].status == "ok"
