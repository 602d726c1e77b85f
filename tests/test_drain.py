"""``destroy node`` with ``drain: true`` (``workflows/drain.py``) against the fake Rancher:
cordon, evictions through the Eviction API honouring disruption budgets (429), DaemonSet
pods kept, and a drain that cannot finish failing the destroy before anything is destroyed."""

import json

import pytest

from test_direct_executor import _manager, _nodes, env  # noqa: F401 - fixture
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.rancher.client import RancherClient
from triton_kubernetes_amd.rancher.fake import FakeRancher
from triton_kubernetes_amd.workflows import delete_node, new_cluster

from helpers import make_ctx, output


def _pod(name, node, ns="default", daemonset=False, refusals=None, owner="Job"):
    meta = {"name": name, "namespace": ns}
    if daemonset:
        meta["ownerReferences"] = [{"kind": "DaemonSet", "name": "amdgpu-device-plugin"}]
    elif owner:
        meta["ownerReferences"] = [{"kind": owner, "name": f"{name}-owner"}]
    if refusals is not None:
        meta["annotations"] = {FakeRancher.PDB_ANNOTATION: str(refusals)}
    return {"apiVersion": "v1", "kind": "Pod", "metadata": meta,
            "spec": {"nodeName": node, "containers": [{"name": "c", "image": "busybox:1.36"}]}}


def _cluster(fake, agent, backend, base):
    _manager(fake, backend, base)
    cp = agent("cp")
    workers = [agent(f"w{i}", gpus=8) for i in range(2)]
    new_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="dev",
                              k8s_version="v1.28.10-rancher1-1", k8s_network_provider="calico",
                              nodes=_nodes(cp, workers))), backend)
    return next(iter(fake.state.clusters))


def _post(fake, cid, pod):
    st = fake.state
    key = f"{cid}|/api/v1/namespaces/{pod['metadata']['namespace']}/pods|{pod['metadata']['name']}"
    with st.mu:  # bound pods as the scheduler leaves them (the fake has no scheduler for pods)
        st.objects[key] = json.loads(json.dumps(pod))
        st.cluster_objects.setdefault(cid, {})[key] = None


def _pods_on(fake, cid, node):
    return sorted(o["metadata"]["name"] for k, o in fake.state.objects.items()
                  if k.startswith(f"{cid}|/api/v1/namespaces/") and "/pods|" in k
                  and (o.get("spec") or {}).get("nodeName") == node)


def test_drain_evicts_then_destroys(env):  # noqa: F811 - fixture
    fake, agent, backend, base = env
    cid = _cluster(fake, agent, backend, base)
    _post(fake, cid, _pod("train-0", "gpu-2", ns="ml"))
    _post(fake, cid, _pod("serve-0", "gpu-2", ns="ml", refusals=2))  # its budget refuses twice
    _post(fake, cid, _pod("plugin-x", "gpu-2", ns="kube-system", daemonset=True))
    _post(fake, cid, _pod("train-1", "gpu-1", ns="ml"))  # another node: untouched
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_name="dev", hostname="gpu-2", drain=True,
                        rancher_cleanup=True))
    delete_node(ctx, backend)
    out = output(ctx)
    assert "Drained gpu-2: evicted 2 pod(s), 2 eviction(s) refused by disruption budgets and retried" in out
    assert "kept 1 DaemonSet/mirror pod(s)" in out
    assert _pods_on(fake, cid, "gpu-2") == ["plugin-x"] and _pods_on(fake, cid, "gpu-1") == ["train-1"]
    assert "node_baremetal_dev_gpu-2" not in backend.state("mgr").nodes("cluster_baremetal_dev")


def test_drain_timeout_destroys_nothing(env):  # noqa: F811 - fixture
    fake, agent, backend, base = env
    cid = _cluster(fake, agent, backend, base)
    _post(fake, cid, _pod("pinned", "gpu-1", ns="ml", refusals="always"))
    ctx = make_ctx(dict(base, cluster_manager="mgr", cluster_name="dev", hostname="gpu-1", drain=True,
                        drain_timeout="0.3"))
    with pytest.raises(TKError, match=r"drain of gpu-1 timed out after 0.3s; pods still on the node: ml/pinned"):
        delete_node(ctx, backend)
    # nothing destroyed; the node stays cordoned
    assert "gpu-1" in backend.state("mgr").nodes("cluster_baremetal_dev")
    node = next(n for n in fake.k8s_nodes(cid) if n["metadata"]["name"] == "gpu-1")
    assert node["spec"].get("unschedulable") is True
    assert "unschedulable" not in next(n for n in fake.k8s_nodes(cid) if n["metadata"]["name"] == "gpu-2")["spec"]


def test_client_drain_primitives(env):  # noqa: F811 - fixture
    fake, agent, backend, base = env
    cid = _cluster(fake, agent, backend, base)
    from triton_kubernetes_amd.executor.base import outputs_from_tfstate
    from triton_kubernetes_amd.state import MANAGER_KEY

    mgr = outputs_from_tfstate(backend.read_tfstate("mgr"), MANAGER_KEY)
    client = RancherClient(mgr["rancher_url"], mgr["rancher_access_key"], mgr["rancher_secret_key"])
    _post(fake, cid, _pod("a", "gpu-1"))
    assert [p["metadata"]["name"] for p in client.node_pods(cid, "gpu-1")] == ["a"]
    assert client.node_pods(cid, "gpu-2") == []
    assert client.evict_pod(cid, "default", "a") == 201 and client.evict_pod(cid, "default", "a") == 404
    client.cordon(cid, "gpu-1")
    client.cordon(cid, "gpu-1", False)
    assert "unschedulable" not in next(n for n in client.k8s_nodes(cid) if n["metadata"]["name"] == "gpu-1")["spec"]


def test_drain_cordon_uncordon_commands(env):  # noqa: F811 - fixture
    from triton_kubernetes_amd.cli.main import dispatch

    fake, agent, backend, base = env
    cid = _cluster(fake, agent, backend, base)
    _post(fake, cid, _pod("train-0", "gpu-1", ns="ml"))
    sel = dict(base, cluster_manager="mgr", cluster_name="dev", hostname="gpu-1")

    def unschedulable():
        return next(n for n in fake.k8s_nodes(cid) if n["metadata"]["name"] == "gpu-1")["spec"].get("unschedulable")

    ctx = make_ctx(sel)
    assert dispatch(ctx, backend, "drain", "node") == 0
    assert "Drained gpu-1: evicted 1 pod(s)" in output(ctx) and _pods_on(fake, cid, "gpu-1") == []
    assert unschedulable() is True
    assert "gpu-1" in backend.state("mgr").nodes("cluster_baremetal_dev")  # still in the cluster
    ctx = make_ctx(sel)
    assert dispatch(ctx, backend, "uncordon", "node") == 0 and "gpu-1 uncordoned" in output(ctx)
    assert unschedulable() is None
    assert dispatch(make_ctx(sel), backend, "cordon", "node") == 0 and unschedulable() is True


def test_unmanaged_pods_need_force(env):  # noqa: F811 - fixture
    from triton_kubernetes_amd.cli.main import dispatch

    fake, agent, backend, base = env
    cid = _cluster(fake, agent, backend, base)
    _post(fake, cid, _pod("scratch", "gpu-1", owner=None))  # a bare pod: gone for good once evicted
    _post(fake, cid, _pod("train-0", "gpu-1", ns="ml"))
    sel = dict(base, cluster_manager="mgr", cluster_name="dev", hostname="gpu-1")
    with pytest.raises(TKError, match=r"runs pods no controller manages .*default/scratch; set drain_force"):
        dispatch(make_ctx(sel), backend, "drain", "node")
    assert _pods_on(fake, cid, "gpu-1") == ["scratch", "train-0"]  # nothing evicted
    ctx = make_ctx(dict(sel, drain_force=True))
    assert dispatch(ctx, backend, "drain", "node") == 0 and _pods_on(fake, cid, "gpu-1") == []
