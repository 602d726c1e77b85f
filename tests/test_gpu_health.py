"""MI355X GPU health policy (``node/health.py``, ``tk_topo.cpp:render_health``).

Fixture sysfs trees (``test_partitions.make_tree``) get RAS counters
(``ras/*_err_count``: ``ue: N`` / ``ce: N``) and the driver's bad-page records
(``ras/gpu_vram_bad_pages``: ``0x<page> : 0x<size> : R|P|F``); the native labeller and
the Python spec must return the same verdict and labels.
"""

import json
import os
import subprocess

import pytest

from test_partitions import make_tree, native_ok  # noqa: F401 - fixture
from triton_kubernetes_amd.errors import ConfigError
from triton_kubernetes_amd.node import health
from triton_kubernetes_amd.node.labels import labels_from_topology
from triton_kubernetes_amd.ops import topo
from triton_kubernetes_amd.ops.native import executable


def _ras(root, minor, ue=0, ce=0, bad=None, block="umc"):
    ras = os.path.join(root, f"sys/class/drm/renderD{minor}/device/ras")
    os.makedirs(ras, exist_ok=True)
    with open(os.path.join(ras, f"{block}_err_count"), "w") as fh:
        fh.write(f"ue: {ue}\nce: {ce}\n")
    if bad is None:
        return
    with open(os.path.join(ras, "gpu_vram_bad_pages"), "w") as fh:
        for k, st in enumerate(bad):
            fh.write(f"0x{0x1000 + k:08x} : 0x00001000 : {st}\n")


def healthy_tree(root, compute="SPX", memory="NPS1"):
    make_tree(root, compute=compute, memory=memory)
    parts = {"SPX": 1, "CPX": 8}[compute]
    for g in range(8):
        _ras(root, 128 + g * parts, bad=())
    return root


def _both(root, max_ue=0, max_bad=-1):
    native = topo.native_health("sysfs", root, max_ue, max_bad)
    python = health.evaluate(topo.native_topology("sysfs", root), max_ue, max_bad)
    assert native == python
    return native


def test_healthy_node(tmp_path, native_ok):
    root = healthy_tree(str(tmp_path))
    v = _both(root)
    assert v["status"] == "healthy" and v["reasons"] == [] and len(v["gpus"]) == 8
    # 294896 MiB of HBM: the driver's default threshold is one page per 100 MiB
    assert v["gpus"][0]["bad_page_limit"] == 2949 and v["max_bad_pages"] == "auto"
    labels = topo.native_labels("sysfs", root)
    assert labels == labels_from_topology(topo.native_topology("sysfs", root))
    assert labels["amd.com/gpu.ecc-uncorrectable"] == "0" and labels["amd.com/gpu.bad-pages"] == "0"


def test_uncorrectable_errors_and_retired_pages(tmp_path, native_ok):
    root = healthy_tree(str(tmp_path))
    _ras(root, 131, ue=2, ce=7)
    _ras(root, 133, ce=40, bad=["R"] * 5 + ["P"] * 2)
    _ras(root, 133, ue=0, ce=1, block="gfx")  # another RAS block: counters add up
    v = _both(root, max_ue=0, max_bad=6)
    assert v["status"] == "unhealthy" and v["unhealthy_gpus"] == 2
    assert v["reasons"] == ["GPU 3 (0000:35:00.0): 2 uncorrectable ECC errors (max 0)",
                            "GPU 5 (0000:55:00.0): 7 retired VRAM pages (max 6)"]
    g5 = v["gpus"][5]
    assert g5["ecc_correctable"] == 41 and g5["bad_pages"] == 7 and g5["bad_pages_pending"] == 2
    # the same pages under the driver's own threshold, and UE errors allowed up to 2
    assert _both(root, max_ue=2, max_bad=-1)["status"] == "healthy"
    labels = topo.native_labels("sysfs", root)
    assert labels["amd.com/gpu.ecc-uncorrectable"] == "2" and labels["amd.com/gpu.bad-pages"] == "7"
    assert labels == labels_from_topology(topo.native_topology("sysfs", root))


def test_labeller_cli_health(tmp_path, native_ok):
    root = healthy_tree(str(tmp_path))
    exe = executable("amdgpu-topo-labeller")
    ok = subprocess.run([exe, "--health", "--source", "sysfs", "--sysfs-root", root], capture_output=True, text=True)
    assert ok.returncode == 0 and json.loads(ok.stdout)["status"] == "healthy"
    _ras(root, 128, ue=1)
    bad = subprocess.run([exe, "--health", "--source", "sysfs", "--sysfs-root", root, "--max-bad-pages", "auto"],
                         capture_output=True, text=True)
    assert bad.returncode == 3 and json.loads(bad.stdout)["reasons"][0].startswith("GPU 0 (0000:05:00.0): 1 ")
    lab = subprocess.run([exe, "--health", "--labels", "--source", "sysfs", "--sysfs-root", root],
                         capture_output=True, text=True)
    assert lab.returncode == 3
    assert lab.stdout.splitlines() == ["amd.com/gpu.health=unhealthy", "amd.com/gpu.unhealthy-count=1"]
    assert dict(ln.split("=") for ln in lab.stdout.splitlines()) == health.health_labels(json.loads(bad.stdout))


def test_partitions_count_a_gpu_once(tmp_path, native_ok):
    """CPX: eight logical GPUs per physical one.  Counters on the PCI function (sysfs) or
    repeated on every partition (as amd_smi reports them) are one GPU's, counted once."""
    root = healthy_tree(str(tmp_path), compute="CPX", memory="NPS2")
    _ras(root, 128 + 8 * 2, ue=3, bad=["R"])
    v = _both(root)
    assert len(v["gpus"]) == 8 and v["unhealthy_gpus"] == 1
    assert v["reasons"] == ["GPU 2 (0000:25:00.0): 3 uncorrectable ECC errors (max 0)"]
    doc = topo.native_topology("sysfs", root)
    for g in doc["gpus"]:  # amd_smi-style: every partition reports its device's counters
        if g["bdf"] == "0000:25:00.0":
            g.update(ecc_uncorrectable=3, ecc_correctable=0, bad_pages=1, bad_pages_pending=0)
    assert health.evaluate(doc) == v
    assert labels_from_topology(doc)["amd.com/gpu.ecc-uncorrectable"] == "3"


def test_aca_counters(tmp_path, native_ok):
    """MI300/MI350-series drivers report per-block counts as ras/aca_<block> ("ue: N", "ce: N",
    "de: N"); when the legacy <block>_err_count files are there too, only ACA counts."""
    root = healthy_tree(str(tmp_path))
    ras = os.path.join(root, "sys/class/drm/renderD130/device/ras")
    for block, ue in (("umc", 1), ("gfx", 0), ("xgmi_wafl", 2)):
        with open(os.path.join(ras, f"aca_{block}"), "w") as fh:
            fh.write(f"ue: {ue}\nce: 3\nde: 0\n")
    _ras(root, 130, ue=9, ce=9)  # legacy view of the same errors: not counted again
    v = _both(root)
    assert v["reasons"] == ["GPU 2 (0000:25:00.0): 3 uncorrectable ECC errors (max 0)"]
    assert v["gpus"][2]["ecc_correctable"] == 9


def test_no_ras_reported_is_not_judged(native_ok, tmp_path):
    root = make_tree(str(tmp_path))  # no ras directories at all
    v = _both(root)
    assert v["status"] == "healthy" and "ecc_uncorrectable" not in v["gpus"][0]
    assert "amd.com/gpu.bad-pages" not in topo.native_labels("sysfs", root)


def test_policy_settings():
    assert health.policy_of({}) == "fail" and health.policy_of({"gpu_health": "TAINT"}) == "taint"
    with pytest.raises(ConfigError, match="gpu_health must be one of fail, taint, off"):
        health.policy_of({"gpu_health": "warn"})
    assert health.limits_of({}) == (0, -1)
    assert health.limits_of({"gpu_max_uncorrectable_ecc": "3", "gpu_max_retired_pages": "auto"}) == (3, -1)
    assert health.limits_of({"gpu_max_retired_pages": "64"}) == (0, 64)
    with pytest.raises(ConfigError, match="gpu_max_retired_pages must be a non-negative integer or auto"):
        health.limits_of({"gpu_max_retired_pages": "-5"})
    with pytest.raises(ConfigError, match="gpu_max_uncorrectable_ecc must be a non-negative integer"):
        health.limits_of({"gpu_max_uncorrectable_ecc": "x"})
    assert health.taint_flag() == "amd.com/gpu-health=unhealthy:NoSchedule"
    assert health.has_health_taint({"spec": {"taints": [dict(health.HEALTH_TAINT)]}})
    assert not health.has_health_taint({"spec": {}})


# --- bring-up: shell step (SSH / Terraform path) --------------------------------------------


def _run_health_step(tmp_path, root, cfg_extra):
    """The rendered gpu_health step against a fixture tree: the real labeller behind a
    wrapper that points it at the tree; /etc and sudo redirected into tmp_path."""
    from triton_kubernetes_amd.node.plan import TOOLS_DIR, build_host_plan

    cfg = dict({"hostname": "g", "rancher_host_labels": {"worker": "true"}, "gpu_count": 8, "gpu_burnin": "off"},
               **cfg_extra)
    plan = build_host_plan(cfg, "https://r", "t", "s", mi355x=True)
    step = next(s for s in plan.steps if s.name == "gpu_health")
    tools, etc = tmp_path / "tools", tmp_path / "etc"
    tools.mkdir(exist_ok=True)
    (etc / "triton-kubernetes").mkdir(parents=True, exist_ok=True)
    wrapper = tools / "amdgpu-topo-labeller"
    wrapper.write_text(f'#!/bin/sh\nexec {executable("amdgpu-topo-labeller")} --source sysfs --sysfs-root {root} "$@"\n')
    wrapper.chmod(0o755)
    body = step.shell.replace(TOOLS_DIR, str(tools)).replace("/etc/", f"{etc}/").replace("sudo ", "")
    p = subprocess.run(["bash", "-c", "set -euo pipefail\nf() {\n" + body + "\n}\nf"], capture_output=True, text=True)
    files = {n: (etc / "triton-kubernetes" / n).read_text() for n in os.listdir(etc / "triton-kubernetes")}
    return p, files, step


@pytest.mark.parametrize("policy", ["fail", "taint"])
def test_shell_health_step(tmp_path, native_ok, policy):
    root = healthy_tree(str(tmp_path / "tree"))
    p, files, step = _run_health_step(tmp_path, root, {"gpu_health": policy})
    assert p.returncode == 0, p.stderr
    assert json.loads(files["gpu-health.json"])["status"] == "healthy" and "gpu-taints" not in files
    assert "amd.com/gpu.health=healthy" in files["gpu-burnin-labels"]
    assert step.params == {"policy": policy, "max_uncorrectable": 0, "max_bad_pages": -1}
    _ras(root, 130, ue=4)
    p, files, _ = _run_health_step(tmp_path, root, {"gpu_health": policy})
    assert "amd.com/gpu.health=unhealthy" in files["gpu-burnin-labels"]
    if policy == "fail":
        assert p.returncode == 1 and "GPU 2 (0000:25:00.0): 4 uncorrectable ECC errors (max 0)" in p.stderr
    else:
        assert p.returncode == 0 and files["gpu-taints"].strip() == "amd.com/gpu-health=unhealthy:NoSchedule"
    # limits raised past the counters: healthy again
    p, files, _ = _run_health_step(tmp_path, root, {"gpu_health": policy, "gpu_max_uncorrectable_ecc": 4})
    assert p.returncode == 0 and json.loads(files["gpu-health.json"])["status"] == "healthy"


def test_join_carries_the_taint_file():
    from triton_kubernetes_amd.node.plan import TAINT_FILE, build_host_plan

    cfg = {"hostname": "g", "rancher_host_labels": {"worker": "true"}, "gpu_count": 8, "gpu_health": "taint"}
    for dist in ("rke2", "rke1"):
        plan = build_host_plan(dict(cfg, k8s_distribution=dist), "https://r", "t", "s", mi355x=True)
        join = plan.steps[-1].shell
        assert f'sed "s/^/ --taints /" {TAINT_FILE}' in join, dist


def test_terraform_host_script_renders_the_policy():
    """The MI355X Terraform module's host script, rendered by the planner from module inputs."""
    from triton_kubernetes_amd.terraform import plan as tfplan
    from triton_kubernetes_amd.terraform.catalog import MODULES_DIR

    path = os.path.join(MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host", "files", "install_mi355x_node.sh.tftpl")
    base = {"hostname": "g", "docker_engine_install_url": "u", "docker_install_sha256": "", "rancher_api_url": "https://r",
            "rancher_cluster_registration_token": "t", "rancher_cluster_ca_checksum": "c", "rancher_node_role": "worker",
            "k8s_distribution": "rke2", "rancher_agent_image": "i", "rancher_registry": "", "rancher_registry_username": "",
            "rancher_registry_password": "", "gpu_count": 8, "gpu_burnin": "quick", "rccl_env_file": "", "rccl_min_busbw": "0",
            "gpu_link_min_frac": "0.5", "gpu_link_min_gbps": "38", "gpu_compute_partition": "spx",
            "gpu_memory_partition": "nps1", "gpu_partitions": 1, "rccl_slim": "off",
            "gpu_max_uncorrectable_ecc": "0", "gpu_max_retired_pages": "auto", "gpu_host_tuning": "warn",
            "gpu_metrics_textfile": ""}
    fail = tfplan._f_templatefile(path, dict(base, gpu_health="fail"))
    taint = tfplan._f_templatefile(path, dict(base, gpu_health="taint"))
    off = tfplan._f_templatefile(path, dict(base, gpu_health="off"))
    assert "--health --max-uncorrectable 0 --max-bad-pages auto" in fail and "exit 1 ;;" in fail
    assert "amd.com/gpu-health=unhealthy:NoSchedule" in taint and "amd.com/gpu-health" not in fail
    assert "--health" not in off
    for script in (fail, taint, off):
        assert subprocess.run(["bash", "-n"], input=script, text=True).returncode == 0


# --- bring-up end to end: agents, fake Rancher, readiness --------------------------------------


def _sick_topology(ngpu=8):
    from triton_kubernetes_amd.node.labels import synthetic_topology

    doc = synthetic_topology(ngpu)
    for g in doc["gpus"]:
        g.update(ecc_uncorrectable=0, ecc_correctable=0, bad_pages=0, bad_pages_pending=0, vram_mb=294896)
    doc["gpus"][1]["ecc_uncorrectable"] = 2
    return doc


def _create(tmp_path, policy):
    import tempfile

    from helpers import make_ctx
    from triton_kubernetes_amd import versions
    from triton_kubernetes_amd.backend import LocalBackend
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.labels import synthetic_topology
    from triton_kubernetes_amd.rancher.fake import FakeRancher
    from triton_kubernetes_amd.workflows import new_cluster, new_manager

    token = "health-token-123456"
    fake = FakeRancher.for_manager("mgr", "s3cret-passw0rd").start()
    agents = []

    def agent(name, topology=None):
        a = NodeAgent(name=name, mode="sim", devices=list(range(8)) if topology else [], token=token,
                      root=tempfile.mkdtemp(), topology_override=topology, burnin_override=lambda d, lvl: {"ok": True})
        agents.append(a)
        return "agent+" + a.serve()

    backend = LocalBackend(str(tmp_path / "state"))
    base = {"executor": "direct", "agent_token": token}
    new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr", rancher_admin_password="s3cret-passw0rd",
                              rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="ubuntu", bastion_host="", key_path="k")), backend)
    cp = agent("cp")
    healthy, sick = agent("w0", synthetic_topology(8)), agent("w1", _sick_topology())
    nodes = [{"rancher_host_label": "control", "node_count": 1, "hostname": "cp", "ssh_user": "u", "bastion_host": "",
              "key_path": "k", "hosts": [cp]},
             {"rancher_host_label": "etcd", "node_count": 1, "hostname": "etcd", "ssh_user": "u", "bastion_host": "",
              "key_path": "k", "hosts": [cp]},
             {"rancher_host_label": "worker", "node_count": 2, "hostname": "gpu", "ssh_user": "u", "bastion_host": "",
              "key_path": "k", "hosts": [healthy, sick], "gpu": "mi355x", "gpu_count": 8, "gpu_health": policy}]
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="dev",
                        k8s_version=versions.DEFAULT_K8S_VERSION, k8s_network_provider="calico", gpu_addons=True,
                        wait=True, rccl_gate=True, nodes=nodes))
    return fake, agents, backend, ctx, new_cluster


def test_taint_policy_joins_the_sick_node_outside_gpu_scheduling(tmp_path):
    fake, agents, backend, ctx, new_cluster = _create(tmp_path, "taint")
    try:
        new_cluster(ctx, backend)
        rep = ctx.extras["last_readiness"]
        assert rep.gpu_unhealthy == ["gpu-2"]
        # the gate ran over the healthy node's 8 GPUs only
        assert rep.rccl["ok"] and rep.rccl["world"] == 8 and rep.rccl["nodes"] == 1
        cid = list(fake.state.clusters)[0]
        k8s = {n["metadata"]["name"]: n for n in fake.k8s_nodes(cid)}
        sick = k8s["gpu-2"]
        assert health.has_health_taint(sick) and sick["metadata"]["labels"]["amd.com/gpu.health"] == "unhealthy"
        # the device plugin does not tolerate the taint: no amd.com/gpu on the sick node
        assert "amd.com/gpu" not in sick["status"]["allocatable"]
        assert k8s["gpu-1"]["status"]["allocatable"]["amd.com/gpu"] == "8"
        assert k8s["gpu-1"]["metadata"]["labels"]["amd.com/gpu.health"] == "healthy"
        assert "health taint" in ctx.out.getvalue()
    finally:
        for a in agents:
            a.stop()
        fake.stop()


def test_fail_policy_stops_the_create_with_the_reason(tmp_path):
    fake, agents, backend, ctx, new_cluster = _create(tmp_path, "fail")
    try:
        with pytest.raises(Exception, match=r"unhealthy GPUs \(gpu_health = fail\): GPU 1: 2 uncorrectable ECC"):
            new_cluster(ctx, backend)
    finally:
        for a in agents:
            a.stop()
        fake.stop()


# --- day 2: health cluster -----------------------------------------------------------------


def test_health_cluster_reconciles_the_taint(tmp_path):
    from triton_kubernetes_amd.cli.main import dispatch
    from triton_kubernetes_amd.node.labels import synthetic_topology
    from triton_kubernetes_amd.workflows.health import cluster_health

    from helpers import make_ctx

    fake, agents, backend, ctx, new_cluster = _create(tmp_path, "taint")
    try:
        new_cluster(ctx, backend)
        cid = list(fake.state.clusters)[0]
        w0, w1 = agents[1], agents[2]
        # report only: nothing changes in the cluster
        base = {"agent_token": "health-token-123456", "cluster_manager": "mgr", "cluster_name": "dev"}
        report = make_ctx(base)
        verdicts = {v["node"]: v for v in cluster_health(report, backend)}
        assert verdicts["gpu-1"]["status"] == "healthy" and verdicts["gpu-2"]["status"] == "unhealthy"
        assert "taint" not in verdicts["gpu-1"] and "unhealthy: 1 (gpu-2)" in report.out.getvalue()
        # the sick GPU is replaced; the other node logs an uncorrectable error
        w1.topology_override = synthetic_topology(8)
        w0.topology_override = _sick_topology()
        # labels only: the counters and verdict labels move, no taint changes
        relabel = make_ctx(dict(base, health_labels=True))
        cluster_health(relabel, backend)
        k8s = {n["metadata"]["name"]: n for n in fake.k8s_nodes(cid)}
        assert k8s["gpu-1"]["metadata"]["labels"]["amd.com/gpu.health"] == "unhealthy"
        assert not health.has_health_taint(k8s["gpu-1"]) and health.has_health_taint(k8s["gpu-2"])
        assert k8s["gpu-2"]["metadata"]["labels"]["amd.com/gpu.health"] == "healthy"
        fence = make_ctx(dict(base, health_taint=True))
        assert dispatch(fence, backend, "health", "cluster") == 0
        k8s = {n["metadata"]["name"]: n for n in fake.k8s_nodes(cid)}
        assert health.has_health_taint(k8s["gpu-1"]) and not health.has_health_taint(k8s["gpu-2"])
        assert k8s["gpu-1"]["metadata"]["labels"]["amd.com/gpu.health"] == "unhealthy"
        assert k8s["gpu-2"]["metadata"]["labels"]["amd.com/gpu.health"] == "healthy"
        # the RAS counters labels are refreshed from the same verdict
        sick_labels = health.ras_labels(health.physical_gpus(_sick_topology()))
        assert sick_labels["amd.com/gpu.ecc-uncorrectable"] != "0"
        for k, v in sick_labels.items():
            assert k8s["gpu-1"]["metadata"]["labels"][k] == v, k
        assert k8s["gpu-1"]["metadata"]["labels"]["amd.com/gpu.unhealthy-count"] == "1"
        assert k8s["gpu-2"]["metadata"]["labels"]["amd.com/gpu.unhealthy-count"] == "0"
        assert k8s["gpu-2"]["metadata"]["labels"]["amd.com/gpu.ecc-uncorrectable"] == "0"
        # NoSchedule keeps new pods off but does not evict the running device plugin;
        # the healed node's plugin pod schedules now that the taint is gone
        assert k8s["gpu-1"]["status"]["allocatable"]["amd.com/gpu"] == "8"
        assert k8s["gpu-2"]["status"]["allocatable"]["amd.com/gpu"] == "8"
        lines = [json.loads(ln) for ln in fence.out.getvalue().splitlines() if ln.startswith("{")]
        assert {d["node"]: d["taint"] for d in lines} == {"gpu-1": "tainted", "gpu-2": "untainted"}
        # idempotent
        again = make_ctx(dict(base, health_taint=True))
        cluster_health(again, backend)
        assert '"taint": "unchanged"' in again.out.getvalue() and "tainted" not in again.out.getvalue()
        # NoExecute: the taint's effect changes and the pods running there are evicted --
        # the device plugin too, so the sick node stops advertising GPUs
        evict = make_ctx(dict(base, health_taint=True, health_taint_effect="noexecute"))
        cluster_health(evict, backend)
        assert '"taint": "tainted NoExecute"' in evict.out.getvalue()
        k8s = {n["metadata"]["name"]: n for n in fake.k8s_nodes(cid)}
        assert [t["effect"] for t in k8s["gpu-1"]["spec"]["taints"] if t["key"] == health.HEALTH_TAINT["key"]] == \
            ["NoExecute"]
        assert k8s["gpu-1"]["status"]["allocatable"].get("amd.com/gpu", "0") == "0"
        assert k8s["gpu-2"]["status"]["allocatable"]["amd.com/gpu"] == "8"
        with pytest.raises(ConfigError, match="health_taint_effect must be one of NoSchedule, NoExecute"):
            cluster_health(make_ctx(dict(base, health_taint=True, health_taint_effect="PreferNoSchedule")), backend)
        # a limit given here overrides the node modules'
        lenient = make_ctx(dict(base, gpu_max_uncorrectable_ecc=5))
        assert all(v["status"] == "healthy" for v in cluster_health(lenient, backend))
    finally:
        for a in agents:
            a.stop()
        fake.stop()


def test_health_taint_keeps_a_taint_added_meanwhile(tmp_path):
    """spec.taints is replaced whole, so fencing a node from a node list read
    earlier dropped a taint added since (the node-lifecycle controller's unreachable taint).
    The patch now carries the node's resourceVersion; the API server answers 409 on a stale
    one (the fake refuses it too) and the node is read again."""
    from triton_kubernetes_amd.cloud.http import HTTPError
    from triton_kubernetes_amd.rancher.client import RancherClient
    from triton_kubernetes_amd.workflows.health import _reconcile

    fake, agents, backend, ctx, new_cluster = _create(tmp_path, "taint")
    try:
        new_cluster(ctx, backend)
        cid = list(fake.state.clusters)[0]
        outs = json.loads(backend.read_tfstate("mgr"))["module_outputs"]["cluster-manager"]
        client = RancherClient(fake.url, outs["rancher_access_key"], outs["rancher_secret_key"])
        stale = next(n for n in client.k8s_nodes(cid) if n["metadata"]["name"] == "gpu-1")
        unreachable = {"key": "node.kubernetes.io/unreachable", "effect": "NoExecute"}
        client.patch_node(cid, "gpu-1", {"spec": {"taints": list(stale["spec"]["taints"]) + [unreachable]}})
        # the fake refuses a patch against the old resourceVersion, as the API server does
        with pytest.raises(HTTPError) as exc:
            client.patch_node(cid, "gpu-1", {"metadata": {"resourceVersion": stale["metadata"]["resourceVersion"]},
                                            "spec": {"taints": []}})
        assert exc.value.status == 409
        verdict = {"status": "unhealthy", "gpus": [], "unhealthy_gpus": 1}
        assert _reconcile(client, cid, stale, verdict) == "tainted"
        node = next(n for n in client.k8s_nodes(cid) if n["metadata"]["name"] == "gpu-1")
        keys = [t["key"] for t in node["spec"]["taints"]]
        assert "node.kubernetes.io/unreachable" in keys and health.HEALTH_TAINT["key"] in keys
    finally:
        for a in agents:
            a.stop()
        fake.stop()


def test_health_probe_over_the_host_transport(tmp_path, native_ok):
    """SSH / Terraform nodes: the labeller runs on the node; exit 3 is a verdict, not an error."""
    from triton_kubernetes_amd.parallel.transport import LocalTransport
    from triton_kubernetes_amd.workflows.health import _probe

    from helpers import make_ctx

    root = healthy_tree(str(tmp_path / "tree"))
    _ras(root, 129, ue=1)
    tools = tmp_path / "tools"
    tools.mkdir()
    (tools / "amdgpu-topo-labeller").write_text(
        f'#!/bin/sh\nexec {executable("amdgpu-topo-labeller")} --source sysfs --sysfs-root {root} "$@"\n')
    (tools / "amdgpu-topo-labeller").chmod(0o755)
    ctx = make_ctx({"node_tools_dir": str(tools)})
    ctx.extras["transport"] = LocalTransport()
    v = _probe(ctx, None, "gpu-9", {"host": "local", "gpu_max_retired_pages": "auto"})
    assert v["node"] == "gpu-9" and v["status"] == "unhealthy"
    assert v["reasons"] == ["GPU 1 (0000:15:00.0): 1 uncorrectable ECC errors (max 0)"]
    assert _probe(ctx, None, "gpu-9", {"host": "local", "gpu_max_uncorrectable_ecc": "1"})["status"] == "healthy"


# --- on the MI355X ---------------------------------------------------------------------------


@pytest.mark.gpu
def test_health_on_the_box():
    """The box's own RAS counters: both collectors, the native verdict and the Python spec."""
    exe = executable("amdgpu-topo-labeller")
    docs = {}
    for source in ("sysfs", "amdsmi"):
        p = subprocess.run([exe, "--health", "--source", source], capture_output=True, text=True, timeout=120)
        print(source, p.returncode, p.stdout[:1500], p.stderr[-500:])
        assert p.returncode in (0, 3), p.stderr
        docs[source] = json.loads(p.stdout)
    sysfs, smi = docs["sysfs"], docs["amdsmi"]
    assert len(sysfs["gpus"]) == len(smi["gpus"]) >= 1
    assert sysfs["status"] == smi["status"]
    for a, b in zip(sysfs["gpus"], smi["gpus"]):
        assert a["bdf"] == b["bdf"]
        if "ecc_uncorrectable" in a and "ecc_uncorrectable" in b:
            assert a["ecc_uncorrectable"] == b["ecc_uncorrectable"]
        if "pcie_max_width" in a and "pcie_max_width" in b:  # both collectors see the same link
            assert (a["pcie_width"], a["pcie_max_width"]) == (b["pcie_width"], b["pcie_max_width"])
    assert topo.native_health("sysfs") == health.evaluate(topo.native_topology("sysfs"))


@pytest.mark.gpu
def test_gpu_health_cli_on_the_box(capsys):
    from triton_kubernetes_amd.ops.cli import main

    for source in ("sysfs", "amdsmi"):
        rc = main(["health", "--source", source])
        doc = json.loads(capsys.readouterr().out)
        assert rc in (0, 3) and (rc == 0) == (doc["status"] == "healthy")
        assert doc["gpus"] and doc["gpus"][0]["bad_page_limit"] > 0


def test_get_nodes_shows_gpu_state(tmp_path):
    """``get nodes``: the cluster's nodes through Rancher's Kubernetes API, with the MI355X
    columns (GPUs allocatable / counted, product, partition, burn-in, xGMI, health)."""
    from triton_kubernetes_amd import versions
    from triton_kubernetes_amd.cli.main import dispatch

    from helpers import make_ctx

    fake, agents, backend, ctx, new_cluster = _create(tmp_path, "taint")
    try:
        new_cluster(ctx, backend)
        base = {"agent_token": "health-token-123456", "cluster_manager": "mgr", "cluster_name": "dev"}
        table = make_ctx(base)
        assert dispatch(table, backend, "get", "nodes") == 0
        lines = [ln for ln in table.out.getvalue().splitlines() if ln and not ln.startswith("get nodes")]
        assert lines[0].split() == ["NAME", "READY", "ROLES", "VERSION", "GPUS", "PRODUCT", "PARTITION", "BURN-IN",
                                    "XGMI", "PCIE", "UE/PAGES", "HEALTH"]
        rows = {ln.split()[0]: ln.split() for ln in lines[1:]}
        assert set(rows) == {"cp-1", "etcd-1", "gpu-1", "gpu-2"}
        assert rows["gpu-1"][3] == versions.DEFAULT_K8S_VERSION
        assert rows["gpu-1"][4:] == ["8/8", "MI355X", "spx/nps1", "passed(full)", "mesh", "x16", "0/0", "healthy"]
        assert rows["gpu-2"][4] == "0/8" and rows["gpu-2"][-1] == "unhealthy,tainted"
        assert rows["gpu-2"][-2] == "2/0"
        assert rows["cp-1"][1] == "Ready" and rows["cp-1"][4] == "-"
        js = make_ctx(dict(base, output="json"))
        dispatch(js, backend, "get", "nodes")
        docs = [json.loads(ln) for ln in js.out.getvalue().splitlines() if ln.startswith("{")]
        assert {d["NAME"]: d["GPUS"] for d in docs}["gpu-1"] == "8/8"
    finally:
        for a in agents:
            a.stop()
        fake.stop()


def test_degraded_pcie_link(tmp_path, native_ok):
    """A GPU whose PCIe link trained narrower than the device supports is unhealthy (the
    speed is not judged: power management lowers it at idle); the narrowest link is a label."""
    root = healthy_tree(str(tmp_path))
    dev = os.path.join(root, "sys/class/drm/renderD134/device")
    for attr, val in (("current_link_width", "8"), ("current_link_speed", "16.0 GT/s PCIe")):
        with open(os.path.join(dev, attr), "w") as fh:
            fh.write(val + "\n")
    doc = topo.native_topology("sysfs", root)
    g6 = doc["gpus"][6]
    assert (g6["pcie_width"], g6["pcie_max_width"], g6["pcie_speed_gts"], g6["pcie_max_speed_gts"]) == (8, 16, 16.0, 32.0)
    v = _both(root)
    assert v["reasons"] == ["GPU 6 (0000:65:00.0): PCIe link trained at x8, the device supports x16"]
    labels = topo.native_labels("sysfs", root)
    assert labels["amd.com/gpu.pcie-width"] == "8" and labels == labels_from_topology(doc)
    # a lower link speed alone (idle power management) is not a problem
    with open(os.path.join(dev, "current_link_width"), "w") as fh:
        fh.write("16\n")
    assert _both(root)["status"] == "healthy"


def test_vbios_label(tmp_path, native_ok):
    """One VBIOS on every GPU is a label; GPUs flashed apart read ``mixed`` (both labellers)."""
    root = healthy_tree(str(tmp_path), compute="CPX")
    labels = topo.native_labels("sysfs", root)
    assert labels["amd.com/gpu.vbios"] == "113-M355-01-1K1-020F" and labels["amd.com/rocm.version"] == "7.2.0-43"
    assert topo.native_topology("sysfs", root)["rocm"] == {"version": "7.2.0-43"}
    assert labels["amd.com/gpu.power-cap"] == "1400"
    assert labels == labels_from_topology(topo.native_topology("sysfs", root))
    with open(os.path.join(root, "sys/class/drm/renderD136/device/vbios_version"), "w") as fh:
        fh.write("113-M355-01-1K1-021F\n")
    doc = topo.native_topology("sysfs", root)
    assert {g.get("vbios_version") for g in doc["gpus"]} == {"113-M355-01-1K1-020F", "113-M355-01-1K1-021F", None}
    labels = topo.native_labels("sysfs", root)
    assert labels["amd.com/gpu.vbios"] == "mixed" and labels == labels_from_topology(doc)
    # one GPU capped at 1000 W: the label is the lowest cap (both labellers)
    with open(os.path.join(root, "sys/class/drm/renderD136/device/hwmon/hwmon3/power1_cap"), "w") as fh:
        fh.write("1000000000\n")
    doc = topo.native_topology("sysfs", root)
    assert doc["gpus"][8]["power_cap_w"] == 1000 and doc["gpus"][8]["power_cap_default_w"] == 1400
    labels = topo.native_labels("sysfs", root)
    assert labels["amd.com/gpu.power-cap"] == "1000" and labels == labels_from_topology(doc)


def test_readiness_reports_gpu_nodes_that_differ(tmp_path):
    """Two MI355X nodes flashed with different VBIOS: the cluster is ready, and the report
    and the CLI warn about it (``readiness/waiter.py:gpu_mismatch``)."""
    from triton_kubernetes_amd.readiness.waiter import gpu_mismatch

    fake, agents, backend, ctx, new_cluster = _create(tmp_path, "off")
    try:
        for agent, vb in ((agents[1], "113-M355-01-1K1-020F"), (agents[2], "113-M355-01-1K1-021F")):
            for g in agent.topology_override["gpus"]:
                g["vbios_version"] = vb
        new_cluster(ctx, backend)
        rep = ctx.extras["last_readiness"]
        assert rep.gpu_mismatch == {"amd.com/gpu.vbios": {"113-M355-01-1K1-020F": ["gpu-1"],
                                                          "113-M355-01-1K1-021F": ["gpu-2"]}}
        assert "warning: MI355X nodes differ in amd.com/gpu.vbios" in ctx.out.getvalue()
        assert rep.rccl["ok"]  # a warning, not a failed readiness
        from triton_kubernetes_amd.cli.main import dispatch

        from helpers import make_ctx

        table = make_ctx({"agent_token": "health-token-123456", "cluster_manager": "mgr", "cluster_name": "dev"})
        dispatch(table, backend, "get", "nodes")
        assert ("warning: MI355X nodes differ in amd.com/gpu.vbios: 113-M355-01-1K1-020F: gpu-1; "
                "113-M355-01-1K1-021F: gpu-2") in table.out.getvalue()
    finally:
        for a in agents:
            a.stop()
        fake.stop()
    # non-GPU nodes are not compared; a label one node lacks reads "-"
    assert gpu_mismatch({"cp": {"amd.com/gpu.present": "false"},
                         "a": {"amd.com/gpu.present": "true", "amd.com/gpu.vram": "288G"},
                         "b": {"amd.com/gpu.present": "true"}}) == {"amd.com/gpu.vram": {"288G": ["a"], "-": ["b"]}}


def test_thousands_of_retired_pages_are_counted(tmp_path, native_ok):
    """A bad-page file far larger than any read buffer: every record counts (3000 > 2949,
    the driver's threshold for 288 GiB)."""
    root = healthy_tree(str(tmp_path))
    _ras(root, 133, bad=["R"] * 2990 + ["P"] * 10)
    v = _both(root)
    g5 = v["gpus"][5]
    assert (g5["bad_pages"], g5["bad_pages_pending"], g5["bad_page_limit"]) == (3000, 10, 2949)
    assert v["reasons"] == ["GPU 5 (0000:55:00.0): 3000 retired VRAM pages (max 2949)"]


@pytest.mark.parametrize("argv,needle", [
    (["health", "--max-bad-pages", "lots"], "gpu_max_retired_pages"),
    (["metrics", "--max-bad-pages", "-3"], "gpu_max_retired_pages"),
    (["health", "--max-bad-pages", "1.5"], "gpu_max_retired_pages"),
    (["gemm", "--size", "100"], "multiples of 256"),
])
def test_tk_gpu_refusals_are_one_line(capsys, argv, needle):
    """`tk-gpu` (ops/cli.py) refuses what it cannot use with one line and exit 2, not a
    traceback."""
    from triton_kubernetes_amd.ops.cli import main

    assert main(argv) == 2
    err = capsys.readouterr().err
    assert err.startswith("tk-gpu: ") and needle in err and "Traceback" not in err


def test_tk_gpu_health_without_gpus_is_not_healthy(tmp_path, monkeypatch, capsys, native_ok):
    """A node where the collector finds no GPU (status 2) gets exit 2 from `tk-gpu health`
    and `metrics`, as from `amdgpu-topo-labeller --health` / `--prom`, not a healthy verdict
    over zero GPUs."""
    from triton_kubernetes_amd.ops import cli, topo

    empty = topo.native_topology("sysfs", str(tmp_path))
    assert empty["status"] == 2
    monkeypatch.setattr(topo, "native_topology", lambda source="sysfs", sysfs_root="": dict(empty))
    for cmd in ("health", "metrics"):
        assert cli.main([cmd]) == 2
        assert "GPU collector failed (status 2)" in capsys.readouterr().err


@pytest.mark.parametrize("argv", [["hbm", "--gib", "-4"], ["hbm", "--gib", "nan"], ["hbm", "--blocks-per-cu", "0"],
                                  ["mfma", "--iters", "0"], ["gemm", "--reps", "0"], ["gemm", "--size", "-256"],
                                  ["links", "--mib", "0"], ["links", "--min-frac", "-0.5"], ["burnin", "--device", "-1"],
                                  ["rccl-local", "--ngpus", "-2"], ["health", "--max-uncorrectable", "x"],
                                  ["health", "--max-uncorrectable", "-1"]])
def test_tk_gpu_sizes_and_counts_are_checked_before_the_gpu(argv, capsys):
    """A negative size reached the native probes as a huge unsigned byte count; argparse
    now refuses it (exit 2) before any GPU call."""
    from triton_kubernetes_amd.ops.cli import main

    with pytest.raises(SystemExit) as exc:
        main(argv)
    assert exc.value.code == 2 and "error: argument --" in capsys.readouterr().err
