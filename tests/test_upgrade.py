"""``upgrade cluster`` (``workflows/upgrade.py``) against the fake Rancher: RKE2 through the
provisioning object, RKE1 through the v3 cluster, one minor at a time, the document
updated, the rollout and readiness waited for."""

import pytest

from test_direct_executor import _manager, _nodes, env  # noqa: F401 - fixture
from triton_kubernetes_amd.cli.main import dispatch
from triton_kubernetes_amd.errors import ConfigError
from triton_kubernetes_amd.workflows import new_cluster
from triton_kubernetes_amd.workflows.upgrade import check_upgrade

from helpers import make_ctx, output


def _cluster(fake, agent, backend, base, version):
    _manager(fake, backend, base)
    cp = agent("cp")
    workers = [agent("w0", gpus=8)]
    new_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="dev",
                              k8s_version=version, k8s_network_provider="calico", gpu_addons=True, wait=True,
                              nodes=_nodes(cp, workers))), backend)
    return next(iter(fake.state.clusters))


def test_check_upgrade_rules():
    check_upgrade("v1.29.14+rke2r1", "v1.30.10+rke2r1")
    check_upgrade("v1.30.2+rke2r1", "v1.30.10+rke2r1")  # patch
    with pytest.raises(ConfigError, match="one minor at a time: the cluster runs v1.29, so the next release is v1.30"):
        check_upgrade("v1.29.14+rke2r1", "v1.31.6+rke2r1")
    with pytest.raises(ConfigError, match="cannot downgrade"):
        check_upgrade("v1.30.10+rke2r1", "v1.29.14+rke2r1")
    with pytest.raises(ConfigError, match="cannot change distribution"):
        check_upgrade("v1.29.14+rke2r1", "v1.30.10-rancher1-1")


def test_upgrade_rke2_cluster(env):  # noqa: F811 - fixture
    fake, agent, backend, base = env
    cid = _cluster(fake, agent, backend, base, "v1.29.14+rke2r1")
    assert cid.startswith("c-m-")
    fake.state.upgrade_seconds = 0.2
    sel = dict(base, cluster_manager="mgr", cluster_name="dev")
    with pytest.raises(ConfigError, match="one minor at a time"):
        dispatch(make_ctx(dict(sel, k8s_version="v1.31")), backend, "upgrade", "cluster")
    ctx = make_ctx(dict(sel, k8s_version="v1.30"))  # a minor: the server's release of it
    assert dispatch(ctx, backend, "upgrade", "cluster") == 0
    out = output(ctx)
    assert "v1.29.14+rke2r1 -> v1.30.10+rke2r1 requested" in out and "cluster 'dev' runs v1.30.10+rke2r1" in out
    assert "cluster ready in" in out  # the readiness waiter ran after the rollout
    assert fake.state.v2_clusters["fleet-default/dev"]["spec"]["kubernetesVersion"] == "v1.30.10+rke2r1"
    nodes = fake.k8s_nodes(cid)
    assert {n["status"]["nodeInfo"]["kubeletVersion"] for n in nodes} == {"v1.30.10+rke2r1"}
    assert next(n for n in nodes if n["metadata"]["name"] == "gpu-1")["status"]["allocatable"]["amd.com/gpu"] == "8"
    # the document describes the running cluster
    assert backend.state("mgr").module("cluster_baremetal_dev")["k8s_version"] == "v1.30.10+rke2r1"
    # again: nothing to do
    again = make_ctx(dict(sel, k8s_version="v1.30.10+rke2r1"))
    dispatch(again, backend, "upgrade", "cluster")
    assert "already runs v1.30.10+rke2r1" in output(again) and fake.state.upgrades == 1
    with pytest.raises(ConfigError, match="is an RKE1 release"):
        dispatch(make_ctx(dict(sel, k8s_version="v1.31.6-rancher1-1")), backend, "upgrade", "cluster")


def test_upgrade_rke1_cluster(env):  # noqa: F811 - fixture
    fake, agent, backend, base = env
    cid = _cluster(fake, agent, backend, base, "v1.28.15-rancher1-1")
    assert not cid.startswith("c-m-")
    # Rancher reports an RKE1 cluster's upstream version, not the RKE1 release string
    assert fake.state.clusters[cid]["version"]["gitVersion"] == "v1.28.15"
    fake.state.upgrade_seconds = 0.2
    sel = dict(base, cluster_manager="mgr", cluster_name="dev")
    ctx = make_ctx(dict(sel, k8s_version="v1.29.14-rancher1-1", wait_timeout=60))
    assert dispatch(ctx, backend, "upgrade", "cluster") == 0  # the wait used to time out here
    assert "cluster 'dev' runs v1.29.14-rancher1-1" in output(ctx)
    assert fake.state.clusters[cid]["rancherKubernetesEngineConfig"]["kubernetesVersion"] == "v1.29.14-rancher1-1"
    assert fake.state.clusters[cid]["state"] == "active"
    nodes = fake.k8s_nodes(cid)
    assert {n["status"]["nodeInfo"]["kubeletVersion"] for n in nodes} == {"v1.29.14"}
    assert backend.state("mgr").module("cluster_baremetal_dev")["k8s_version"] == "v1.29.14-rancher1-1"
    again = make_ctx(dict(sel, k8s_version="v1.29.14-rancher1-1"))
    dispatch(again, backend, "upgrade", "cluster")
    assert "already runs v1.29.14" in output(again) and fake.state.upgrades == 1
