"""Prometheus metrics of an MI355X node (``node/metrics.py``, ``amdgpu-topo-labeller --prom``).

* the native ``--prom`` text equals the Python rendering of the native health verdict on
  fixture sysfs trees (healthy, sick, partitioned, degraded PCIe link);
* the text parses with ``prometheus_client``'s own parser (an independent check of the
  exposition format);
* the node agent serves it at ``GET /metrics`` with Prometheus' bearer authorization.
"""

import json
import os
import subprocess

import pytest

from test_gpu_health import _ras, healthy_tree
from test_partitions import native_ok  # noqa: F401 - fixture
from triton_kubernetes_amd.node import metrics
from triton_kubernetes_amd.node.agent import NodeAgent
from triton_kubernetes_amd.node.labels import synthetic_topology
from triton_kubernetes_amd.ops import topo
from triton_kubernetes_amd.ops.native import executable

parser = pytest.importorskip("prometheus_client.parser")


def _native_prom(root, node="gpu-1", *extra):
    p = subprocess.run([executable("amdgpu-topo-labeller"), "--prom", "--node", node, "--source", "sysfs",
                        "--sysfs-root", root, *extra], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    return p.stdout


def _samples(text):
    out = {}
    for fam in parser.text_string_to_metric_families(text):
        for s in fam.samples:
            out[(s.name, tuple(sorted(s.labels.items())))] = s.value
    return out


def test_native_prom_matches_python(tmp_path, native_ok):
    root = healthy_tree(str(tmp_path))
    _ras(root, 131, ue=2, ce=7)
    _ras(root, 133, ce=40, bad=["R"] * 5 + ["P"] * 2)
    dev = os.path.join(root, "sys/class/drm/renderD134/device")
    with open(os.path.join(dev, "current_link_width"), "w") as fh:
        fh.write("8\n")
    text = _native_prom(root, "gpu-1", "--max-bad-pages", "6")
    assert text == metrics.gpu_metrics(topo.native_health("sysfs", root, 0, 6), "gpu-1")
    s = _samples(text)
    who = lambda i, bdf: (("bdf", bdf), ("gpu", str(i)), ("node", "gpu-1"))  # noqa: E731
    assert s[("tk_gpu_healthy", who(0, "0000:05:00.0"))] == 1
    assert s[("tk_gpu_healthy", who(3, "0000:35:00.0"))] == 0
    assert s[("tk_gpu_ecc_uncorrectable_errors", who(3, "0000:35:00.0"))] == 2
    assert s[("tk_gpu_ecc_correctable_errors", who(5, "0000:55:00.0"))] == 40
    assert s[("tk_gpu_retired_pages", who(5, "0000:55:00.0"))] == 7
    assert s[("tk_gpu_retired_pages_pending", who(5, "0000:55:00.0"))] == 2
    assert s[("tk_gpu_retired_pages_limit", who(5, "0000:55:00.0"))] == 6
    assert s[("tk_gpu_pcie_link_width", who(6, "0000:65:00.0"))] == 8
    assert s[("tk_gpu_pcie_link_max_width", who(6, "0000:65:00.0"))] == 16
    assert s[("tk_node_unhealthy_gpus", (("node", "gpu-1"),))] == 3


def test_partitions_are_one_gpu_each(tmp_path, native_ok):
    root = healthy_tree(str(tmp_path), compute="CPX")  # 8 partitions per GPU
    text = _native_prom(root, 'odd"name')
    assert text == metrics.gpu_metrics(topo.native_health("sysfs", root), 'odd"name')
    weird = 'a\\b\nc"d'  # backslash, newline, quote: escaped alike by both
    assert _native_prom(root, weird) == metrics.gpu_metrics(topo.native_health("sysfs", root), weird)
    assert dict(next(k for k in _samples(_native_prom(root, weird)) if k[0] == "tk_node_unhealthy_gpus")[1])["node"] == weird
    healthy = [k for k in _samples(text) if k[0] == "tk_gpu_healthy"]
    assert len(healthy) == 8 and dict(healthy[0][1])["node"] == 'odd"name'


def test_no_ras_reported_no_counter_samples(tmp_path, native_ok):
    from test_partitions import make_tree

    root = make_tree(str(tmp_path))  # no ras/ directory, links at x16
    text = _native_prom(root)
    assert text == metrics.gpu_metrics(topo.native_health("sysfs", root), "gpu-1")
    names = {k[0] for k in _samples(text)}
    assert "tk_gpu_ecc_uncorrectable_errors" not in names and "tk_gpu_retired_pages" not in names
    assert {"tk_gpu_healthy", "tk_gpu_pcie_link_width", "tk_node_unhealthy_gpus"} <= names


def test_bringup_metrics_of_a_plan():
    plan = {"ok": True, "ms": 2081.5, "steps": [
        {"name": "gpu_preflight", "ok": True, "ms": 12.0, "detail": {"gpus": 8}},
        {"name": "gpu_burnin", "ok": True, "ms": 900.25, "detail": {
            "0": {"ok": True, "hbm": {"read_gbps": 6500.5}, "mfma": {"bf16": {"tflops": 2100.0}},
                  "gemm": {"tflops": 1800.0, "verified": True}, "memtest": {"bytes": 1 << 30}}}},
        {"name": "gpu_links", "ok": True, "ms": 300.0,
         "detail": {"labels": {"amd.com/xgmi.p2p-min-gbps": "48", "amd.com/xgmi.p2p-median-gbps": "51"}}},
        {"name": "rccl_local", "ok": True, "ms": 500.0, "detail": {"peak_busbw_gbps": 301.5}},
        {"name": "agent", "ok": False, "ms": 1.0, "detail": "boom"}]}
    s = _samples(metrics.bringup_metrics(plan, "n1", "sim"))
    assert s[("tk_agent_info", (("mode", "sim"), ("node", "n1")))] == 1
    assert s[("tk_bringup_duration_seconds", (("node", "n1"),))] == pytest.approx(2.0815)
    assert s[("tk_bringup_step_success", (("node", "n1"), ("step", "agent")))] == 0
    assert s[("tk_bringup_step_duration_seconds", (("node", "n1"), ("step", "gpu_burnin")))] == pytest.approx(0.90025)
    burn = lambda check, metric: ("tk_gpu_burnin", (("check", check), ("gpu", "0"), ("metric", metric),  # noqa: E731
                                                    ("node", "n1")))
    assert s[burn("hbm", "read_gbps")] == 6500.5 and s[burn("mfma", "bf16.tflops")] == 2100
    assert s[burn("memtest", "bytes")] == 1 << 30 and burn("gemm", "verified") not in s  # numbers only
    assert s[("tk_xgmi_p2p_min_gbps", (("node", "n1"),))] == 48
    assert s[("tk_rccl_local_busbw_gbps", (("node", "n1"),))] == 301.5
    # before any plan: the agent's info only
    assert set(k[0] for k in _samples(metrics.bringup_metrics(None, "n1"))) == {"tk_agent_info"}


def test_agent_serves_metrics_with_bearer_auth(tmp_path):
    from triton_kubernetes_amd.cloud.http import HTTPClient
    from triton_kubernetes_amd.node.plan import build_host_plan

    from test_node import GPU_WORKER

    sick = synthetic_topology(8)
    sick["gpus"][2]["ecc_uncorrectable"] = 3
    agent = NodeAgent("gpu-7", "sim", devices=list(range(8)), root=str(tmp_path), token="sekrit-token",
                      topology_override=sick, burnin_override=lambda d, lvl: {"ok": True, "hbm": {"read_gbps": 6400.0}})
    plan = build_host_plan(dict(GPU_WORKER, gpu_health="taint", gpu_max_uncorrectable_ecc=5), "http://127.0.0.1:9",
                           "tok", "sum", mi355x=True)
    plan.steps = [s for s in plan.steps if s.action != "agent"]
    assert agent.run_plan(plan)["ok"]
    url = agent.serve()
    try:
        http = HTTPClient(base_url=url)
        with pytest.raises(Exception, match="401"):
            http.request("GET", "/metrics", headers={"Authorization": "Bearer wrong"})
        resp = http.request("GET", "/metrics", headers={"Authorization": "Bearer sekrit-token"})
        assert resp.header("Content-Type").startswith("text/plain; version=0.0.4")
        s = _samples(resp.body.decode())
    finally:
        agent.stop()
    assert s[("tk_bringup_success", (("node", "gpu-7"),))] == 1
    burn = ("tk_gpu_burnin", (("check", "hbm"), ("gpu", "3"), ("metric", "read_gbps"), ("node", "gpu-7")))
    assert s[burn] == 6400
    # judged with the limits the node was brought up with (5 uncorrectable allowed)
    gpu2 = [v for k, v in s.items() if k[0] == "tk_gpu_ecc_uncorrectable_errors" and ("gpu", "2") in k[1]]
    assert gpu2 == [3] and s[("tk_node_unhealthy_gpus", (("node", "gpu-7"),))] == 0
    assert s[("tk_agent_gpu_collect_success", (("node", "gpu-7"),))] == 1
    info = next(dict(k[1]) for k in s if k[0] == "tk_node_gpu_info")
    assert info["product"] == "MI355X" and info["compute_partition"] == "spx" and info["node"] == "gpu-7"
    # a GPU read that fails costs the GPU families, not the endpoint
    agent.topology_override = {"gpus": [{"bdf": "x", "bad_pages": "garbled"}]}
    s = _samples(agent.metrics())
    assert s[("tk_agent_gpu_collect_success", (("node", "gpu-7"),))] == 0 and s[("tk_bringup_success", (("node", "gpu-7"),))] == 1
    assert not any(k[0].startswith("tk_gpu_healthy") for k in s)


def _run_textfile_script(tmp_path, root, systemd: bool):
    """The rendered script with the host's paths moved under tmp_path: sudo and systemctl
    are shims, the labeller reads the fixture tree."""
    from triton_kubernetes_amd.node.metrics import textfile_script

    bin_dir, tools = tmp_path / "bin", tmp_path / "tools"
    bin_dir.mkdir()
    tools.mkdir()
    (bin_dir / "sudo").write_text('#!/bin/sh\nexec "$@"\n')
    (bin_dir / "systemctl").write_text(f'#!/bin/sh\necho "$@" >> {tmp_path}/systemctl.log\n')
    (tools / "amdgpu-topo-labeller").write_text(
        f'#!/bin/sh\nexec {executable("amdgpu-topo-labeller")} --source sysfs --sysfs-root {root} --node gpu-1 "$@"\n')
    for f in (bin_dir / "sudo", bin_dir / "systemctl", tools / "amdgpu-topo-labeller"):
        f.chmod(0o755)
    (tmp_path / "units").mkdir()
    if systemd:
        (tmp_path / "run-systemd").mkdir()
    script = textfile_script(str(tools), str(tmp_path / "textfile"), "0", "auto")
    script = (script.replace("/etc/systemd/system", str(tmp_path / "units"))
              .replace("/run/systemd/system", str(tmp_path / "run-systemd")))
    env = dict(os.environ, PATH=f"{bin_dir}:{os.environ['PATH']}")
    p = subprocess.run(["bash", "-e", "-c", script], capture_output=True, text=True, env=env, timeout=60)
    assert p.returncode == 0, p.stderr
    return p


@pytest.mark.parametrize("systemd", [True, False])
def test_textfile_collector_script(tmp_path, native_ok, systemd):
    root = healthy_tree(str(tmp_path / "host"))
    _ras(root, 131, ue=1)
    p = _run_textfile_script(tmp_path, root, systemd)
    text = (tmp_path / "textfile" / "tk_gpu.prom").read_text()
    assert text == metrics.gpu_metrics(topo.native_health("sysfs", root), "gpu-1")
    assert not (tmp_path / "textfile" / "tk_gpu.prom.tmp").exists()
    assert _samples(text)[("tk_node_unhealthy_gpus", (("node", "gpu-1"),))] == 1
    units = sorted(os.listdir(tmp_path / "units"))
    if systemd:
        assert units == ["tk-gpu-metrics.service", "tk-gpu-metrics.timer"]
        svc = (tmp_path / "units" / "tk-gpu-metrics.service").read_text()
        assert "amdgpu-topo-labeller --prom --max-uncorrectable 0 --max-bad-pages auto" in svc
        assert "OnUnitActiveSec=60s" in (tmp_path / "units" / "tk-gpu-metrics.timer").read_text()
        assert "enable --now tk-gpu-metrics.timer" in (tmp_path / "systemctl.log").read_text()
    else:
        assert units == [] and "written once" in p.stderr


def test_textfile_setting_in_both_delivery_paths(tmp_path):
    """``gpu_metrics_textfile``: a gpu_metrics step in the host plan, the same script in the
    Terraform module's host script; off by default; validated."""
    from triton_kubernetes_amd.errors import ConfigError
    from triton_kubernetes_amd.node.plan import build_host_plan
    from triton_kubernetes_amd.terraform import plan as tfplan
    from triton_kubernetes_amd.terraform.catalog import MODULES_DIR

    from test_node import GPU_WORKER

    names = [s.name for s in build_host_plan(GPU_WORKER, "https://r", "t", "c", mi355x=True).steps]
    assert "gpu_metrics" not in names
    plan = build_host_plan(dict(GPU_WORKER, gpu_metrics_textfile="/var/lib/node_exporter/textfile/"),
                           "https://r", "t", "c", mi355x=True)
    names = [s.name for s in plan.steps]
    assert names.index("gpu_metrics") == names.index("gpu_health") + 1
    step = next(s for s in plan.steps if s.name == "gpu_metrics")
    assert step.params["dir"] == "/var/lib/node_exporter/textfile"
    for bad in ("relative/dir", "/tmp/x y", "/a/../etc", "/x;rm -rf /"):
        with pytest.raises(ConfigError, match="gpu_metrics_textfile"):
            metrics.textfile_dir_of({"gpu_metrics_textfile": bad})
    path = os.path.join(MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host", "files", "install_mi355x_node.sh.tftpl")
    base = {"hostname": "g", "docker_engine_install_url": "u", "docker_install_sha256": "", "rancher_api_url": "https://r",
            "rancher_cluster_registration_token": "t", "rancher_cluster_ca_checksum": "c", "rancher_node_role": "worker",
            "k8s_distribution": "rke2", "rancher_agent_image": "i", "rancher_registry": "", "rancher_registry_username": "",
            "rancher_registry_password": "", "gpu_count": 8, "gpu_burnin": "quick", "rccl_env_file": "", "rccl_min_busbw": "0",
            "gpu_link_min_frac": "0.5", "gpu_link_min_gbps": "38", "gpu_compute_partition": "spx",
            "gpu_memory_partition": "nps1", "gpu_partitions": 1, "rccl_slim": "off", "gpu_health": "fail",
            "gpu_max_uncorrectable_ecc": "2", "gpu_max_retired_pages": "auto", "gpu_host_tuning": "warn"}
    off = tfplan._f_templatefile(path, dict(base, gpu_metrics_textfile=""))
    on = tfplan._f_templatefile(path, dict(base, gpu_metrics_textfile="/var/lib/node_exporter/textfile"))
    assert "tk-gpu-metrics" not in off
    want = metrics.textfile_script("/opt/triton-kubernetes/bin", "/var/lib/node_exporter/textfile", "2", "auto")
    assert want in on
    assert subprocess.run(["bash", "-n"], input=on, text=True).returncode == 0


@pytest.mark.gpu
def test_gpu_metrics_cli_on_the_box(capsys):
    from triton_kubernetes_amd.ops.cli import main

    for source in ("sysfs", "amdsmi"):
        assert main(["metrics", "--node", "box", "--source", source]) == 0
        text = capsys.readouterr().out
        s = _samples(text)
        assert s[("tk_node_unhealthy_gpus", (("node", "box"),))] >= 0 and "tk_gpu_healthy" in text


@pytest.mark.gpu
def test_prom_on_the_box():
    """Both collectors' --prom text on the MI355X equals the Python rendering of that
    collector's verdict, and parses."""
    for source in ("sysfs", "amdsmi"):
        p = subprocess.run([executable("amdgpu-topo-labeller"), "--prom", "--node", "box", "--source", source],
                           capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stderr
        print(source, p.stdout)
        # amd_smi runs in the labeller executable (a child process), never in this one
        v = subprocess.run([executable("amdgpu-topo-labeller"), "--health", "--source", source],
                           capture_output=True, text=True, timeout=120)
        assert v.returncode in (0, 3), v.stderr
        assert p.stdout == metrics.gpu_metrics(json.loads(v.stdout), "box")
        s = _samples(p.stdout)
        assert s[("tk_node_unhealthy_gpus", (("node", "box"),))] >= 0
        assert any(k[0] == "tk_gpu_pcie_link_width" for k in s)


def test_scrape_config_for_agent_nodes(tmp_path):
    """``get scrape-config``: one job per agent node (its own token, the manager's agent CA),
    secrets in files (0600), and the jobs actually scrape the agents' /metrics over TLS."""
    import ssl
    import stat

    import yaml

    from test_direct_executor import _manager, _nodes
    from triton_kubernetes_amd import versions
    from triton_kubernetes_amd.backend import LocalBackend
    from triton_kubernetes_amd.cli.main import dispatch
    from triton_kubernetes_amd.cloud.http import HTTPClient
    from triton_kubernetes_amd.node.security import load_pki, read_credentials
    from triton_kubernetes_amd.rancher.fake import FakeRancher
    from triton_kubernetes_amd.workflows import new_cluster

    from helpers import make_ctx, output

    fake = FakeRancher.for_manager("mgr", "s3cret-passw0rd").start()
    backend = LocalBackend(str(tmp_path / "state"))
    base = {"executor": "direct"}
    agents = []

    def agent(name, addr, gpus=0):
        d = tmp_path / f"creds-{name}"
        pki.issue(addr, [versions.AGENT_IMAGE], servers=[fake.url]).write(str(d))
        creds = read_credentials(str(d))
        a = NodeAgent(name=name, mode="sim", devices=list(range(gpus)), token=creds["token"], root=str(tmp_path / name),
                      topology_override=synthetic_topology(gpus) if gpus else None,
                      burnin_override=lambda d, lvl: {"ok": True})
        agents.append(a)
        return "agent+" + a.serve(addr, ssl_context=creds["ssl_context"])

    try:
        _manager(fake, backend, base)
        pki = load_pki(backend, "mgr")
        cp = agent("cp", "127.0.0.1")
        workers = [agent("w0", "127.0.0.2", 8), agent("w1", "127.0.0.3", 8)]
        new_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="dev",
                                  k8s_version="v1.28.10-rancher1-1", k8s_network_provider="calico",
                                  nodes=_nodes(cp, workers))), backend)
        ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_name="dev",
                            metrics_secrets_dir=str(tmp_path / "prom")))
        assert dispatch(ctx, backend, "get", "scrape-config") == 0
        lines = output(ctx).splitlines()
        assert lines[0] == "get scrape-config called"  # the reference's breadcrumb, then the YAML
        jobs = yaml.safe_load("\n".join(lines[1:]))
        to_file = make_ctx(dict(base, cluster_manager="mgr", cluster_name="dev",
                                metrics_secrets_dir=str(tmp_path / "prom"), scrape_config_file=str(tmp_path / "s.yml")))
        dispatch(to_file, backend, "get", "scrape-config")
        assert yaml.safe_load((tmp_path / "s.yml").read_text()) == jobs
        assert [j["job_name"] for j in jobs] == ["tk-dev-gpu-1", "tk-dev-gpu-2"]
        secrets = sorted(os.listdir(tmp_path / "prom"))
        assert secrets == ["mgr-agent-ca.pem", "mgr-dev-gpu-1.token", "mgr-dev-gpu-2.token"]
        for f in secrets:
            assert stat.S_IMODE(os.stat(tmp_path / "prom" / f).st_mode) == 0o600
        assert "tka1." not in output(ctx)  # no secret printed
        # scrape as Prometheus would: https, the CA file, server_name, the token file
        for job, node in zip(jobs, ("w0", "w1")):
            tls = ssl.create_default_context(cafile=job["tls_config"]["ca_file"])
            target = job["static_configs"][0]["targets"][0]
            with open(job["authorization"]["credentials_file"], encoding="utf-8") as fh:
                token = fh.read()
            resp = HTTPClient(base_url=f"https://{target}", ssl_context=tls).request(
                "GET", "/metrics", headers={"Authorization": f"Bearer {token}"})
            s = _samples(resp.body.decode())
            assert s[("tk_bringup_success", (("node", node),))] == 1
            assert any(k[0] == "tk_gpu_healthy" for k in s)
            # the scrape token is read-only -- the monitoring stack that holds it
            # reads /metrics and /v1/health, but cannot post plans, shut down or run RCCL
            assert token.startswith("tkm1.") and "tka1." not in token
            client = HTTPClient(base_url=f"https://{target}", ssl_context=tls, retries=0)
            assert client.request("GET", "/v1/health", headers={"Authorization": f"Bearer {token}"}).status == 200
            for path in ("/v1/plan", "/v1/shutdown", "/v1/cleanup", "/v1/rccl-uid", "/v1/rccl-abort"):
                with pytest.raises(Exception, match="401"):
                    client.request("POST", path, json_body={}, headers={"X-TK-Agent-Token": token})
            with pytest.raises(Exception, match="401"):
                client.request("GET", "/v1/info", headers={"Authorization": f"Bearer {token}"})
        # an SSH / Terraform node with the textfile collector: a node_exporter job
        st = backend.state("mgr")
        key = st.nodes("cluster_baremetal_dev")["gpu-1"]
        st.set_module(key, dict(st.module(key), host="10.0.0.9", gpu_metrics_textfile="/var/lib/node_exporter"))
        backend.persist_state(st)
        mixed = make_ctx(dict(base, cluster_manager="mgr", cluster_name="dev", node_exporter_port="9101",
                              metrics_secrets_dir=str(tmp_path / "prom2"), scrape_config_file=str(tmp_path / "m.yml")))
        dispatch(mixed, backend, "get", "scrape-config")
        got = yaml.safe_load((tmp_path / "m.yml").read_text())
        assert [j["job_name"] for j in got] == ["tk-dev-gpu-2", "tk-dev-node-exporter"]
        assert got[1]["static_configs"] == [{"targets": ["10.0.0.9:9101"], "labels": {"cluster": "dev", "tk_node": "gpu-1"}}]
        # another node's token is refused
        with open(jobs[0]["authorization"]["credentials_file"], encoding="utf-8") as fh:
            wrong = fh.read()
        tls = ssl.create_default_context(cafile=jobs[1]["tls_config"]["ca_file"])
        with pytest.raises(Exception, match="401"):
            HTTPClient(base_url=f"https://{jobs[1]['static_configs'][0]['targets'][0]}", ssl_context=tls).request(
                "GET", "/metrics", headers={"Authorization": f"Bearer {wrong}"})
    finally:
        for a in agents:
            a.stop()
        fake.stop()


def test_long_node_name_is_not_truncated(tmp_path, native_ok):
    """Label values longer than any fixed buffer (an escaped 253-byte host name) render whole."""
    from test_partitions import make_tree

    root = make_tree(str(tmp_path))
    node = ("n" * 120 + '"\\\\') * 2  # escaping doubles the quotes and backslashes
    text = _native_prom(root, node)
    assert text == metrics.gpu_metrics(topo.native_health("sysfs", root), node)
    assert dict(next(k for k in _samples(text) if k[0] == "tk_node_unhealthy_gpus")[1])["node"] == node


def test_alert_rules_use_exported_metrics(tmp_path):
    """``get alert-rules``: valid rule-file YAML whose expressions use only metric families
    this framework exports."""
    import re

    import yaml

    from triton_kubernetes_amd.backend import MemoryBackend
    from triton_kubernetes_amd.cli.main import dispatch
    from triton_kubernetes_amd.workflows.scrape import ALERTS

    from helpers import make_ctx

    ctx = make_ctx({"alert_rules_file": str(tmp_path / "rules.yml")})
    assert dispatch(ctx, MemoryBackend(), "get", "alert-rules") == 0
    doc = yaml.safe_load((tmp_path / "rules.yml").read_text())
    rules = doc["groups"][0]["rules"]
    assert [r["alert"] for r in rules] == [a["alert"] for a in ALERTS]
    exported = {n for n, _, _ in metrics.GPU_FAMILIES + metrics.BRINGUP_FAMILIES}
    for r in rules:
        used = set(re.findall(r"\btk_[a-z_]+\b", r["expr"]))
        assert used and used <= exported, (r["alert"], used - exported)
        assert r["labels"]["severity"] in ("warning", "critical")
