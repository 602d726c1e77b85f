"""Rancher v3 client (S3/S4 semantics) against the fake server; k8s add-on manifests; waiter timeouts."""

import hashlib
import json
import subprocess
import time

import pytest

from triton_kubernetes_amd import versions
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.k8s.manifests import addon_manifests, apply_manifests, gpu_job_manifest
from triton_kubernetes_amd.rancher.client import RancherClient, ca_checksum, wait_until
from triton_kubernetes_amd.rancher.fake import FAKE_CACERTS, FakeRancher, tunnel_params
from triton_kubernetes_amd.readiness.waiter import ReadinessSpec, wait_ready


@pytest.fixture
def rancher():
    fake = FakeRancher(bootstrap_password="b00tstrap-only").start()
    client = RancherClient(fake.url)
    outs = client.bootstrap("n3w-passw0rd-123", fake.url, "b00tstrap-only", timeout=10)
    yield fake, RancherClient(fake.url, outs["rancher_access_key"], outs["rancher_secret_key"]), outs
    fake.stop()


def test_ca_checksum_matches_reference_shasum():
    # rancher_cluster.sh: echo "$cacerts" | shasum -a 256  -> trailing newline included
    assert ca_checksum("abc") == hashlib.sha256(b"abc\n").hexdigest()
    # Rancher's CAChecksum: one trailing newline, never two; no CA -> no checksum
    assert ca_checksum("abc\n") == ca_checksum("abc")
    assert ca_checksum("") == ""


def test_served_cacerts_hash_to_the_cluster_checksum():
    """What a node downloads from /cacerts hashes to the checksum the cluster reports,
    whether or not the stored bundle ends with a newline."""
    import urllib.request

    for pem in (FAKE_CACERTS, FAKE_CACERTS.rstrip("\n") + "\n"):
        fake = FakeRancher().start()
        try:
            fake.state.settings["cacerts"] = pem
            body = urllib.request.urlopen(fake.url + "/cacerts", timeout=10).read()
            assert hashlib.sha256(body).hexdigest() == ca_checksum(pem)
        finally:
            fake.stop()


def test_bootstrap_s3(rancher):
    fake, client, outs = rancher
    assert fake.state.admin_password == "n3w-passw0rd-123"
    assert fake.state.settings["server-url"] == fake.url
    assert outs["rancher_url"] == fake.url and outs["rancher_access_key"] and outs["rancher_secret_key"]
    assert client.ping()
    # neither admin/admin (Rancher >= 2.6 has none) nor the bootstrap password works now
    for pw in ("admin", "b00tstrap-only"):
        with pytest.raises(TKError):
            RancherClient(fake.url).login("admin", pw)


def test_ensure_cluster_is_idempotent_s4(rancher):
    """RKE1 (the reference's v3 cluster): found by name, token reused."""
    fake, client, _ = rancher
    a = client.ensure_cluster("dev", "v1.28.15-rancher1-1", "calico")
    b = client.ensure_cluster("dev", distribution="rke1")
    assert a.cluster_id == b.cluster_id and not a.existed and b.existed
    assert a.registration_token == b.registration_token  # reused, not re-created
    assert a.ca_checksum == ca_checksum(FAKE_CACERTS)
    rke = fake.state.clusters[a.cluster_id]["rancherKubernetesEngineConfig"]
    assert rke["kubernetesVersion"] == "v1.28.15-rancher1-1" and rke["network"]["plugin"] == "calico"
    assert client.ensure_cluster("other", distribution="rke1").cluster_id != a.cluster_id


def test_ensure_rke2_cluster_is_idempotent(rancher):
    """RKE2 (default): a provisioning.cattle.io/v1 Cluster in fleet-default; its management
    cluster (c-m-...) holds the registration token."""
    fake, client, _ = rancher
    a = client.ensure_cluster("dev2", "v1.30.10+rke2r1", "cilium")
    b = client.ensure_cluster("dev2")
    assert a.cluster_id.startswith("c-m-") and a.cluster_id == b.cluster_id and not a.existed and b.existed
    assert a.registration_token == b.registration_token
    obj = fake.state.v2_clusters["fleet-default/dev2"]
    assert obj["spec"]["kubernetesVersion"] == "v1.30.10+rke2r1"
    assert obj["spec"]["rkeConfig"]["machineGlobalConfig"]["cni"] == "cilium"
    assert obj["status"]["clusterName"] == a.cluster_id
    # a name taken by the other distribution is refused both ways (nodes could not join it)
    with pytest.raises(TKError, match="already exists as an RKE2 cluster"):
        client.ensure_cluster("dev2", distribution="rke1")
    client.ensure_cluster("dev1", distribution="rke1")
    with pytest.raises(TKError, match="already exists as an RKE1 cluster"):
        client.ensure_cluster("dev1", distribution="rke2")
    # KDM: a release the server does not offer is replaced by its release of that minor,
    # a minor it does not offer is refused before anything is created
    c = client.ensure_cluster("dev3", "v1.31.2+rke2r1")
    assert fake.state.v2_clusters["fleet-default/dev3"]["spec"]["kubernetesVersion"] == "v1.31.6+rke2r1"
    assert "not offered" in client.last_version_note
    with pytest.raises(TKError, match="not offered"):
        client.ensure_cluster("old", "v1.27.16+rke2r2")
    assert "fleet-default/old" not in fake.state.v2_clusters and c.cluster_id
    client.delete_cluster(a.cluster_id)
    assert "fleet-default/dev2" not in fake.state.v2_clusters and a.cluster_id not in fake.state.clusters


def test_registration_token_filled_in_after_create(rancher):
    """The token value appears only after the create returns (the server's controller
    fills it in): the client polls the token object, and the S4 script does the same."""
    import os

    from triton_kubernetes_amd.terraform.catalog import MODULES_DIR

    fake, client, outs = rancher
    info = client.ensure_cluster("async")
    assert info.registration_token and info.registration_token in fake.state.reg_tokens
    script = os.path.join(MODULES_DIR, "bare-metal-rancher-k8s", "files", "ensure_cluster.sh")
    for dist, version in (("rke1", "v1.28"), ("rke2", "v1.30")):
        query = {"name": f"scripted-{dist}", "version": version, "network": "flannel", "distribution": dist,
                 "api_url": fake.url, "access_key": outs["rancher_access_key"], "secret_key": outs["rancher_secret_key"]}
        first = json.loads(subprocess.run(["bash", script], input=json.dumps(query), capture_output=True, text=True,
                                          check=True, timeout=60).stdout)
        assert first["registration_token"] in fake.state.reg_tokens
        assert first["ca_checksum"] == ca_checksum(FAKE_CACERTS)
        # the minor was resolved against the server's KDM list
        if dist == "rke1":
            rke = fake.state.clusters[first["cluster_id"]]["rancherKubernetesEngineConfig"]
            assert rke["kubernetesVersion"].startswith("v1.28.")
        else:
            obj = fake.state.v2_clusters["fleet-default/scripted-rke2"]
            assert obj["spec"]["kubernetesVersion"] == "v1.30.10+rke2r1"
            assert first["cluster_id"] == obj["status"]["clusterName"]
        again = json.loads(subprocess.run(["bash", script], input=json.dumps(query), capture_output=True, text=True,
                                          check=True, timeout=60).stdout)
        assert again == first  # found by name, token reused


def test_registry_passed_to_rke(rancher):
    fake, client, _ = rancher
    info = client.ensure_cluster("reg", k8s_registry="r.example", k8s_registry_username="u",
                                 k8s_registry_password="p", distribution="rke1")
    rke = fake.state.clusters[info.cluster_id]["rancherKubernetesEngineConfig"]
    assert rke["privateRegistries"] == [{"url": "r.example", "user": "u", "password": "p"}]
    # RKE2: a docker.io mirror + credentials in the cluster's rkeConfig (nodes run no docker login)
    client.ensure_cluster("reg2", k8s_registry="r.example", k8s_registry_username="u", k8s_registry_password="p")
    regs = fake.state.v2_clusters["fleet-default/reg2"]["spec"]["rkeConfig"]["registries"]
    assert regs["mirrors"]["docker.io"]["endpoint"] == ["https://r.example"]
    # credentials live in a basic-auth Secret of fleet-default the config names
    assert fake.registry_auth(regs["configs"]["r.example"]["authConfigSecretName"]) == {"username": "u",
                                                                                         "password": "p"}


def _register(fake, token, host, roles, labels=None, capacity=None, kind="system-agent"):
    from triton_kubernetes_amd.cloud.http import HTTPClient

    hdrs = {"X-API-Tunnel-Token": token,
            "X-API-Tunnel-Params": tunnel_params(host, roles, labels or {}, capacity or {}),
            "X-Cattle-Agent-Kind": kind}
    return HTTPClient(base_url=fake.url).request("POST", "/v3/connect/register", headers=hdrs, data=b"{}").json()


def test_agent_kind_must_match_the_distribution(rancher):
    """An RKE2 cluster takes rancher-system-agent nodes only, an RKE1 cluster rancher-agent ones."""
    from triton_kubernetes_amd.cloud.http import HTTPError

    fake, client, _ = rancher
    rke2 = client.ensure_cluster("k2")
    rke1 = client.ensure_cluster("k1", distribution="rke1")
    with pytest.raises(HTTPError) as exc:
        _register(fake, rke2.registration_token, "a", {"worker": True}, kind="rancher-agent")
    assert exc.value.status == 400 and b"rancher-system-agent" in exc.value.body
    with pytest.raises(HTTPError):
        _register(fake, rke1.registration_token, "b", {"worker": True})
    _register(fake, rke2.registration_token, "a", {"worker": True})
    _register(fake, rke1.registration_token, "b", {"worker": True}, kind="rancher-agent")


def test_cluster_lifecycle_and_gpu_allocatable(rancher):
    fake, client, _ = rancher
    info = client.ensure_cluster("gpu")
    assert client.cluster_state(info.cluster_id) != "active"
    _register(fake, info.registration_token, "cp", {"etcd": True, "controlplane": True, "worker": False})
    _register(fake, info.registration_token, "g1", {"etcd": False, "controlplane": False, "worker": True},
              {"amd.com/gpu.present": "true"}, {"amd.com/gpu": 8})
    wait_until(lambda: client.cluster_state(info.cluster_id) == "active", 5, "active")
    nodes = {n["metadata"]["name"]: n for n in client.k8s_nodes(info.cluster_id)}
    assert nodes["g1"]["metadata"]["labels"]["amd.com/gpu.present"] == "true"
    assert "amd.com/gpu" not in nodes["g1"]["status"].get("allocatable", {})  # no device plugin yet
    base = {"node_labeller_image": "", "rccl_env_injector": "false", "rccl_gate": "false"}
    applied = apply_manifests(client, info.cluster_id, addon_manifests(base))
    assert applied == ["DaemonSet/amdgpu-device-plugin", "ConfigMap/rccl-env"]
    nodes = {n["metadata"]["name"]: n for n in client.k8s_nodes(info.cluster_id)}
    assert str(nodes["g1"]["status"]["allocatable"]["amd.com/gpu"]) == "8"
    # re-apply: 409 -> PUT
    assert apply_manifests(client, info.cluster_id, addon_manifests(base)) == applied
    client.delete_cluster(info.cluster_id)
    client.delete_cluster(info.cluster_id)  # 404 tolerated
    assert client.find_cluster("gpu") is None


def test_device_plugin_model_gates_gpu_allocatable(rancher):
    """amd.com/gpu is advertised only where a real device-plugin pod would run and register:
    the right image, the kubelet socket and /sys mounted, a node the pod schedules on
    (Ready, GPU label, taints tolerated), after the plugin's start-up time."""
    import copy

    from triton_kubernetes_amd.k8s.manifests import device_plugin_daemonset

    fake, client, _ = rancher
    fake.state.device_plugin_seconds = 0.3
    info = client.ensure_cluster("dp")
    gpu = {"amd.com/gpu.present": "true"}
    _register(fake, info.registration_token, "cp", {"etcd": True, "controlplane": True})
    _register(fake, info.registration_token, "g1", {"worker": True}, gpu, {"amd.com/gpu": 8})
    _register(fake, info.registration_token, "g2", {"worker": True}, {}, {"amd.com/gpu": 8})  # not labelled
    from triton_kubernetes_amd.cloud.http import HTTPClient

    tainted = {"X-API-Tunnel-Token": info.registration_token, "X-Cattle-Agent-Kind": "system-agent",
               "X-API-Tunnel-Params": tunnel_params("g3", {"worker": True}, gpu, {"amd.com/gpu": 8},
                                                    [{"key": "dedicated", "value": "x", "effect": "NoSchedule"}])}
    HTTPClient(base_url=fake.url).request("POST", "/v3/connect/register", headers=tainted, data=b"{}")
    wait_until(lambda: client.cluster_state(info.cluster_id) == "active", 5, "active")
    path = "/apis/apps/v1/namespaces/kube-system/daemonsets"

    def gpus():
        return {n["metadata"]["name"]: n["status"]["allocatable"].get("amd.com/gpu")
                for n in client.k8s_nodes(info.cluster_id)}

    good = device_plugin_daemonset(versions.DEVICE_PLUGIN_IMAGE)
    for bad in (device_plugin_daemonset(versions.NODE_LABELLER_IMAGE),  # the labeller tag is no plugin
                device_plugin_daemonset("busybox:1.36")):
        bad["metadata"]["name"] = "not-a-plugin"
        client.k8s(info.cluster_id, "POST", path, bad)
        no_socket = copy.deepcopy(good)
        no_socket["metadata"]["name"] = "no-socket"
        no_socket["spec"]["template"]["spec"]["containers"][0]["volumeMounts"] = [{"name": "sys", "mountPath": "/sys"}]
        client.k8s(info.cluster_id, "POST", path, no_socket)
        time.sleep(0.35)
        assert set(gpus().values()) == {None}
        client.k8s(info.cluster_id, "DELETE", f"{path}/not-a-plugin")
        client.k8s(info.cluster_id, "DELETE", f"{path}/no-socket")
    client.k8s(info.cluster_id, "POST", path, good)
    ds = client.k8s(info.cluster_id, "GET", f"{path}/{good['metadata']['name']}")
    assert ds["status"]["desiredNumberScheduled"] == 1 and ds["status"]["numberReady"] == 0
    assert gpus()["g1"] is None  # the plugin pod is still starting
    wait_until(lambda: gpus()["g1"] == "8", 5, "plugin registered")
    # only g1: g2 lacks the GPU label (nodeSelector), g3's taint is not tolerated, cp has no GPUs
    assert gpus() == {"cp": None, "g1": "8", "g2": None, "g3": None}
    ds = client.k8s(info.cluster_id, "GET", f"{path}/{good['metadata']['name']}")
    assert ds["status"]["numberReady"] == 1
    # the plugin going away takes the resource with it
    client.k8s(info.cluster_id, "DELETE", f"{path}/{good['metadata']['name']}")
    assert gpus()["g1"] is None


def test_bad_registration_token_rejected(rancher):
    fake, _, _ = rancher
    with pytest.raises(TKError):
        _register(fake, "nope", "x", {"worker": True})


def test_wait_until_adaptive_and_timeout():
    calls = []

    def fn():
        calls.append(time.monotonic())
        return "done" if len(calls) >= 4 else None

    assert wait_until(fn, 5, "x", first=0.02) == "done"
    gaps = [b - a for a, b in zip(calls, calls[1:])]
    # doubling: 20, 40, 80 ms.  A sleep never ends early, so lower bounds hold on a loaded CPU
    assert gaps[1] >= 0.038 and gaps[2] >= 0.078, gaps
    with pytest.raises(TKError, match="timed out after 0s waiting for never"):
        wait_until(lambda: None, 0.05, "never", first=0.01)


def test_waiter_times_out_on_missing_node(rancher):
    fake, client, _ = rancher
    info = client.ensure_cluster("partial")
    for h, roles in (("a", {"etcd": True}), ("b", {"controlplane": True}), ("c", {"worker": True})):
        _register(fake, info.registration_token, h, roles)
    spec = ReadinessSpec(info.cluster_id, ["a", "b", "c", "d"], timeout=0.3)
    with pytest.raises(TKError, match="4 nodes Ready"):
        wait_ready(client, spec)
    rep = wait_ready(client, ReadinessSpec(info.cluster_id, ["a", "b", "c"], timeout=5))
    assert set(rep.phases) == {"cluster_active", "nodes_ready"} and rep.ready_seconds >= 0


def test_gpu_job_manifest_affinity(tmp_path):
    job = gpu_job_manifest("train", "img", ["run"], gpus_per_pod=8, pods=4)
    pod = job["spec"]["template"]["spec"]
    exprs = pod["affinity"]["nodeAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"][
        "nodeSelectorTerms"][0]["matchExpressions"]
    keys = {e["key"]: e["values"] for e in exprs}
    assert keys == {"amd.com/gpu.present": ["true"], "amd.com/gpu.count": ["8"],
                    "amd.com/xgmi.fully-connected": ["true"]}
    term = pod["affinity"]["podAffinity"]["preferredDuringSchedulingIgnoredDuringExecution"][0]["podAffinityTerm"]
    assert term["topologyKey"] == "amd.com/xgmi.hive-id"
    assert pod["containers"][0]["resources"]["limits"]["amd.com/gpu"] == "8"
    assert pod["containers"][0]["envFrom"] == [{"configMapRef": {"name": "rccl-env"}}]
    # the node's own RCCL file (discovered RDMA ports) is sourced over the ConfigMap
    cmd = pod["containers"][0]["command"]
    assert cmd[:2] == ["/bin/sh", "-c"] and cmd[3:] == ["run"] and ". /etc/rccl/rccl.env" in cmd[2]
    assert pod["volumes"][0]["hostPath"]["path"] == "/etc/rccl"
    env_file = tmp_path / "rccl.env"
    env_file.write_text('NCCL_IB_HCA="=mlx5_0:1"\n')
    out = subprocess.run(["/bin/sh", "-c", cmd[2].replace("/etc/rccl/rccl.env", str(env_file)), "sh", "-c",
                          'echo "$NCCL_IB_HCA $NCCL_DEBUG"'], capture_output=True, text=True,
                         env={"NCCL_DEBUG": "WARN", "PATH": "/usr/bin:/bin"}, check=True).stdout
    assert out.strip() == "=mlx5_0:1 WARN"
    single = gpu_job_manifest("one", "img", ["x"], gpus_per_pod=1)["spec"]["template"]["spec"]["affinity"]
    assert "podAffinity" not in single
    assert len(single["nodeAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"]["nodeSelectorTerms"][0][
        "matchExpressions"]) == 2


def test_addon_manifest_options():
    names = [f'{o["kind"]}/{o["metadata"]["name"]}' for _, o in addon_manifests(
        {"node_labeller_image": "rocm/k8s-device-plugin:labeller", "rccl_gate": "true",
         "rccl_probe_image": "tk/rccl:1", "rccl_env_injector": "false"})]
    assert names == ["DaemonSet/amdgpu-device-plugin", "ConfigMap/rccl-env",
                     "ServiceAccount/amdgpu-node-labeller", "ClusterRole/amdgpu-node-labeller",
                     "ClusterRoleBinding/amdgpu-node-labeller", "DaemonSet/amdgpu-node-labeller", "Job/rccl-ready"]
    cm = addon_manifests({})[1][1]
    assert cm["data"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


@pytest.mark.parametrize("dist,version", [("rke1", "v1.28.15-rancher1-1"), ("rke2", "v1.29.14+rke2r1")])
def test_terraform_cluster_script_against_fake(rancher, tmp_path, dist, version):
    """The cluster modules' data "external" program (S4) speaks to Rancher like RancherClient does."""
    import subprocess

    from triton_kubernetes_amd.terraform import scripts

    fake, client, outs = rancher
    script = tmp_path / "ensure_cluster.sh"
    script.write_text(scripts.RANCHER_CLUSTER)
    query = {"name": "tf", "version": version, "network": "calico", "api_url": fake.url, "distribution": dist,
             "access_key": outs["rancher_access_key"], "secret_key": outs["rancher_secret_key"],
             "registry": "r.example", "registry_username": "u", "registry_password": "p"}

    def run():
        proc = subprocess.run(["bash", str(script)], input=json.dumps(query), capture_output=True, text=True,
                              timeout=60)
        assert proc.returncode == 0, proc.stderr
        return json.loads(proc.stdout)

    first, second = run(), run()
    assert first == second  # found by name, registration token reused
    info = client.ensure_cluster("tf", distribution=dist)
    assert first == {"cluster_id": info.cluster_id, "registration_token": info.registration_token,
                     "ca_checksum": ca_checksum(FAKE_CACERTS)}
    if dist == "rke1":
        rke = fake.state.clusters[info.cluster_id]["rancherKubernetesEngineConfig"]
        assert rke["network"]["plugin"] == "calico"
        assert rke["privateRegistries"] == [{"url": "r.example", "user": "u", "password": "p"}]
    else:
        rke = fake.state.v2_clusters["fleet-default/tf"]["spec"]["rkeConfig"]
        assert rke["machineGlobalConfig"]["cni"] == "calico"
        secret = rke["registries"]["configs"]["r.example"]["authConfigSecretName"]
        assert fake.registry_auth(secret) == {"username": "u", "password": "p"}
