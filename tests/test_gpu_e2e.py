"""End-to-end MI355X bring-up on the real GPU (``pytest -m gpu``).

A bare-metal ``create cluster`` through the DirectExecutor whose worker agent
runs the native GPU steps for real: amd_smi topology labels, quick burn-in
(HBM/MFMA/memtest kernels), then the readiness waiter's RCCL gate.
"""

import json
import tempfile

import pytest

pytestmark = pytest.mark.gpu


def test_real_gpu_bringup(tmp_path):
    from triton_kubernetes_amd.backend import LocalBackend
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.parallel.transport import AgentTransport
    from triton_kubernetes_amd.rancher.fake import FakeRancher
    from triton_kubernetes_amd.workflows import new_cluster, new_manager

    from helpers import make_ctx, output

    token = "gpu-e2e-token-1234"
    fake = FakeRancher().start()
    cp = NodeAgent(name="cp", mode="sim", token=token, root=tempfile.mkdtemp())
    w = NodeAgent(name="w0", mode="sim", devices=[0], token=token, root=tempfile.mkdtemp())
    cp_url, w_url = cp.serve(), w.serve()
    backend = LocalBackend(str(tmp_path / "state"))
    base = {"executor": "direct", "agent_token": token}
    try:
        new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr", rancher_admin_password="p",
                                  host="rancher+" + fake.url, ssh_user="u", bastion_host="", key_path="k")), backend)
        ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="gpu",
                            k8s_version="v1.9.5-rancher1-1", k8s_network_provider="flannel", gpu_addons=True,
                            wait=True, rccl_gate=True, nodes=[
                                {"rancher_host_label": "control", "node_count": 1, "hostname": "cp", "ssh_user": "u",
                                 "bastion_host": "", "key_path": "k", "hosts": ["agent+" + cp_url]},
                                {"rancher_host_label": "etcd", "node_count": 1, "hostname": "etcd", "ssh_user": "u",
                                 "bastion_host": "", "key_path": "k", "hosts": ["agent+" + cp_url]},
                                {"rancher_host_label": "worker", "node_count": 1, "hostname": "mi355x",
                                 "ssh_user": "u", "bastion_host": "", "key_path": "k", "hosts": ["agent+" + w_url],
                                 "gpu": "mi355x", "gpu_count": 1},
                            ]))
        ctx.extras["agent_transport"] = AgentTransport(token=token)
        new_cluster(ctx, backend)
        assert "rccl_gate" in output(ctx)
        labels = w.last_labels
        print(json.dumps(labels, indent=1))
        assert labels["amd.com/gpu.present"] == "true"
        assert labels["amd.com/gpu.target"] == "gfx950"
        assert labels["amd.com/gpu.product-name"].startswith("MI355")
        hist = w.history[-1]
        burn = [s for s in hist["steps"] if s["name"] == "gpu_burnin"][0]
        assert burn["ok"] and burn["detail"]["0"]["ok"], burn
    finally:
        w.stop()
        cp.stop()
        fake.stop()
