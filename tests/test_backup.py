"""backup cluster / restore cluster (reference README.md:16, never implemented there)."""

import json

import pytest

from triton_kubernetes_amd.backend import LocalBackend
from triton_kubernetes_amd.cloud.aws import S3Client
from triton_kubernetes_amd.cloud.fake_s3 import FakeS3
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.rancher.client import RancherClient
from triton_kubernetes_amd.rancher.fake import FakeRancher
from triton_kubernetes_amd.workflows import new_cluster, new_manager
from triton_kubernetes_amd.workflows.backup import backup_cluster, restore_cluster, sanitize

from helpers import make_ctx, output


@pytest.fixture
def cluster(tmp_path):
    fake = FakeRancher.for_manager("mgr", "tk-admin-pw-0123").start()
    backend = LocalBackend(str(tmp_path / "state"))
    base = {"executor": "direct"}
    new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr", rancher_admin_password="tk-admin-pw-0123",
                              rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="u", bastion_host="", key_path="k")), backend)
    new_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="prod",
                              k8s_version="v1.28.10-rancher1-1", k8s_network_provider="calico")), backend)
    tf = json.loads(backend.read_tfstate("mgr"))
    mgr = tf["module_outputs"]["cluster-manager"]
    cid = tf["module_outputs"]["cluster_baremetal_prod"]["rancher_cluster_id"]
    client = RancherClient(mgr["rancher_url"], mgr["rancher_access_key"], mgr["rancher_secret_key"])
    for ns in ("ml", "web", "kube-system"):
        client.k8s(cid, "POST", "/api/v1/namespaces", {"apiVersion": "v1", "kind": "Namespace",
                                                        "metadata": {"name": ns}})
    objs = [
        ("/apis/apps/v1/namespaces/ml/deployments",
         {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "trainer", "namespace": "ml",
                                                                     "annotations": {"a": "b"}},
          "spec": {"replicas": 2, "selector": {"matchLabels": {"app": "trainer"}},
                   "template": {"metadata": {"labels": {"app": "trainer"}},
                                "spec": {"containers": [{"name": "t", "image": "rocm/pytorch:latest"}]}}}}),
        ("/api/v1/namespaces/ml/configmaps",
         {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cfg", "namespace": "ml"}, "data": {"k": "v"}}),
        ("/api/v1/namespaces/ml/configmaps",
         {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "kube-root-ca.crt", "namespace": "ml"}}),
        ("/api/v1/namespaces/ml/secrets",
         {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "sa-tok", "namespace": "ml", "annotations": {
             "kubernetes.io/service-account.name": "default"}}, "type": "kubernetes.io/service-account-token"}),
        ("/api/v1/namespaces/ml/services",
         {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "svc", "namespace": "ml"},
          "spec": {"clusterIP": "10.43.0.7", "ports": [{"port": 80}]}}),
        ("/apis/batch/v1/namespaces/web/jobs",
         {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "owned", "namespace": "web",
                                                               "ownerReferences": [{"kind": "CronJob"}]},
          "spec": {"template": {"spec": {"restartPolicy": "Never",
                                         "containers": [{"name": "j", "image": "busybox:1.36"}]}}}}),
        ("/api/v1/namespaces/web/configmaps",
         {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "site", "namespace": "web"}}),
    ]
    for path, obj in objs:
        client.k8s(cid, "POST", path, obj)
    yield fake, backend, client, cid
    fake.stop()


def _ctx(**kw):
    return make_ctx(dict({"cluster_manager": "mgr", "cluster_name": "prod"}, **kw))


def test_sanitize_rules():
    assert sanitize({"kind": "Pod", "metadata": {"ownerReferences": [{}]}}) is None
    svc = sanitize({"kind": "Service", "metadata": {"name": "s", "uid": "u", "resourceVersion": "3"},
                    "spec": {"clusterIP": "1.2.3.4", "clusterIPs": ["1.2.3.4"], "ports": []}, "status": {}})
    assert svc == {"kind": "Service", "metadata": {"name": "s"}, "spec": {"ports": []}}
    # a headless service stays headless
    headless = sanitize({"kind": "Service", "metadata": {"name": "h"}, "spec": {"clusterIP": "None",
                                                                                "clusterIPs": ["None"]}})
    assert headless["spec"] == {"clusterIP": "None", "clusterIPs": ["None"]}
    # a Job loses the selector and controller-uid labels the API server generated ...
    gen = {"batch.kubernetes.io/controller-uid": "u1", "controller-uid": "u1", "job-name": "j",
           "batch.kubernetes.io/job-name": "j", "app": "train"}
    job = sanitize({"kind": "Job", "metadata": {"name": "j"},
                    "spec": {"selector": {"matchLabels": {"batch.kubernetes.io/controller-uid": "u1"}},
                             "template": {"metadata": {"labels": dict(gen)}, "spec": {}}}})
    assert "selector" not in job["spec"] and job["spec"]["template"]["metadata"]["labels"] == {"app": "train"}
    # ... unless it chose them itself
    manual = sanitize({"kind": "Job", "metadata": {"name": "m"},
                       "spec": {"manualSelector": True, "selector": {"matchLabels": {"app": "x"}},
                                "template": {"metadata": {"labels": {"app": "x"}}}}})
    assert manual["spec"]["selector"] == {"matchLabels": {"app": "x"}}


def test_backup_to_state_backend_and_restore(cluster):
    fake, backend, client, cid = cluster
    ctx = _ctx()
    name = backup_cluster(ctx, backend)
    assert "Backed up 6 objects from 2 namespaces of cluster 'prod'" in output(ctx)
    archive = json.loads(backend.read_blob("mgr", name))
    assert archive["namespaces"] == ["ml", "web"] and archive["cluster_id"] == cid
    kinds = sorted((o["object"]["kind"], o["object"]["metadata"]["name"]) for o in archive["objects"])
    assert kinds == [("ConfigMap", "cfg"), ("ConfigMap", "site"), ("Deployment", "trainer"),
                     ("Namespace", "ml"), ("Namespace", "web"), ("Service", "svc")]
    for o in archive["objects"]:
        assert "uid" not in o["object"]["metadata"] and "status" not in o["object"]
    svc = next(o["object"] for o in archive["objects"] if o["object"]["kind"] == "Service")
    assert "clusterIP" not in svc["spec"]
    # lose the ml namespace's objects, then restore
    for path in ("/apis/apps/v1/namespaces/ml/deployments/trainer", "/api/v1/namespaces/ml/configmaps/cfg"):
        client.k8s(cid, "DELETE", path)
    ctx = _ctx(backup_namespaces=["ml"])
    assert restore_cluster(ctx, backend) == 4  # ns, cm, svc, deployment (PUT over the existing ones)
    assert client.k8s(cid, "GET", "/apis/apps/v1/namespaces/ml/deployments/trainer")["spec"]["replicas"] == 2


def test_backup_selected_namespaces_and_errors(cluster):
    fake, backend, client, cid = cluster
    ctx = _ctx(backup_namespaces="web")
    backup_cluster(ctx, backend)
    assert "Backed up 2 objects from 1 namespaces" in output(ctx)
    with pytest.raises(TKError, match="Namespace 'nope' does not exist in cluster 'prod'."):
        backup_cluster(_ctx(backup_namespaces=["nope"]), backend)
    with pytest.raises(TKError, match="Unsupported backup_target 'tape'"):
        backup_cluster(_ctx(backup_target="tape"), backend)
    with pytest.raises(TKError, match="Backup 'missing.json' does not exist."):
        restore_cluster(_ctx(backup_name="missing.json"), backend)


def test_backup_to_s3_with_signatures(cluster):
    fake, backend, client, cid = cluster
    s3 = FakeS3(page_size=1).start()
    try:
        ctx = _ctx(backup_target="s3", s3_bucket="bk", aws_access_key=s3.access_key, aws_secret_key=s3.secret_key,
                   aws_region=s3.region, s3_endpoint=s3.url)
        first = backup_cluster(ctx, backend)
        import time

        time.sleep(1.1)  # next second: a distinct archive name
        second = backup_cluster(ctx, backend)
        assert first != second and ("bk", f"triton-kubernetes/mgr/{second}") in s3.objects
        assert s3.rejected == 0
        # archives hold Secrets: stored with server-side encryption (a signed header)
        assert s3.encryption[("bk", f"triton-kubernetes/mgr/{second}")] == "AES256"
        keys = S3Client(s3.access_key, s3.secret_key, s3.region, s3.url).list_keys("bk", "triton-kubernetes/")
        assert len(keys) == 2  # paginated 1 per page
        ctx = _ctx(backup_target="s3", s3_bucket="bk", aws_access_key=s3.access_key, aws_secret_key=s3.secret_key,
                   aws_region=s3.region, s3_endpoint=s3.url)
        assert restore_cluster(ctx, backend) == 6
        assert second in output(ctx)  # newest archive restored
        bad = S3Client(s3.access_key, "wrong", s3.region, s3.url)
        with pytest.raises(TKError):
            bad.put_object("bk", "x", b"1")
        assert s3.rejected == 1
    finally:
        s3.stop()


def test_cli_backup_command(cluster, tk_home, monkeypatch):
    fake, backend, client, cid = cluster
    import io

    from triton_kubernetes_amd.cli.main import run

    monkeypatch.setenv("TRITON_KUBERNETES_HOME", backend.root)
    out = io.StringIO()
    cfg = tk_home / "b.yaml"
    cfg.write_text("backend_provider: local\ncluster_manager: mgr\ncluster_name: prod\n")
    assert run(["--non-interactive", "--config", str(cfg), "backup", "cluster"], out=out) == 0
    assert "Backed up" in out.getvalue()
    out = io.StringIO()
    assert run(["backup", "node"], out=out) == 255
    assert out.getvalue() == 'invalid argument "node" for "triton-kubernetes backup"\n'
