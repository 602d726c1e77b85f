"""`userdata node`: cloud-init delivery of a node's bootstrap plan (RCCL env via write_files)."""

import subprocess

import pytest
import yaml

from triton_kubernetes_amd.backend import LocalBackend
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.node.plan import build_host_plan, render_cloud_init
from triton_kubernetes_amd.rancher.fake import FakeRancher
from triton_kubernetes_amd.workflows import new_cluster, new_manager
from triton_kubernetes_amd.workflows.userdata import node_userdata

from helpers import make_ctx, output


def test_render_cloud_init_document():
    plan = build_host_plan({"hostname": "g1", "rancher_host_labels": {"worker": "true"}, "gpu_count": 8},
                           "https://r", "tok", "sum", mi355x=True)
    text = render_cloud_init(plan, {"NCCL_SOCKET_IFNAME": "eth0"})
    assert text.startswith("#cloud-config\n")
    doc = yaml.safe_load(text)
    assert doc["hostname"] == "g1"
    files = {f["path"]: f for f in doc["write_files"]}
    assert files["/etc/rccl/rccl.env"]["content"].strip().endswith('NCCL_SOCKET_IFNAME="eth0"')
    script = files["/opt/triton-kubernetes/bootstrap.sh"]
    assert script["permissions"] == "0755"
    assert subprocess.run(["bash", "-n"], input=script["content"], text=True).returncode == 0
    assert "bootstrap.sh" in doc["runcmd"][0][2]


def test_userdata_node_from_applied_cluster(tmp_path):
    fake = FakeRancher.for_manager("mgr", "tk-admin-pw-0123").start()
    try:
        backend = LocalBackend(str(tmp_path / "state"))
        base = {"executor": "direct"}
        new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr", rancher_admin_password="tk-admin-pw-0123",
                                  rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="u", bastion_host="", key_path="k")), backend)
        new_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="pxe",
                                  k8s_version="v1.28.10-rancher1-1", k8s_network_provider="calico")), backend)
        # the node is only recorded (its delivery will be cloud-init): persist without applying the host
        from triton_kubernetes_amd.models import baremetal

        st = backend.state("mgr")
        baremetal.new_node(make_ctx({"rancher_host_label": "worker", "node_count": 1, "hostname": "gpu",
                                     "ssh_user": "u", "bastion_host": "", "key_path": "k", "hosts": ["10.9.0.1"],
                                     "gpu": "mi355x", "rccl_env": {"NCCL_IB_HCA": "mlx5_0"},
                                     "gpu_metrics_textfile": "/var/lib/node_exporter/textfile"}),
                           "mgr", "cluster_baremetal_pxe", None, st)
        backend.persist_state(st)
        ctx = make_ctx({"cluster_manager": "mgr", "cluster_name": "pxe", "hostname": "gpu-1"})
        text = node_userdata(ctx, backend)
        assert output(ctx) == text
        doc = yaml.safe_load(text)
        files = {f["path"]: f["content"] for f in doc["write_files"]}
        cid = list(fake.state.clusters)[0]
        token = next(t for t, r in fake.state.reg_tokens.items() if r["clusterId"] == cid)
        assert f"--token {token}" in files["/opt/triton-kubernetes/bootstrap.sh"]
        assert 'NCCL_IB_HCA="mlx5_0"' in files["/etc/rccl/rccl.env"]
        assert "gpu_burnin" in files["/opt/triton-kubernetes/bootstrap.sh"]
        # the node_exporter textfile timer travels with the cloud-init delivery too
        assert "tk-gpu-metrics.timer" in files["/opt/triton-kubernetes/bootstrap.sh"]
        with pytest.raises(TKError, match="A node named 'nope', does not exist."):
            node_userdata(make_ctx({"cluster_manager": "mgr", "cluster_name": "pxe", "hostname": "nope"}), backend)
    finally:
        fake.stop()
