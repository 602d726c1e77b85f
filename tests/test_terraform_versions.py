"""The Terraform path on the Terraform versions the packaged modules require.

Three rules a real Terraform enforces and the fake now enforces too
(``tests/fixtures/fake_terraform.py``):

* >= 0.15: a root output over a ``sensitive`` module output must be ``sensitive``;
* >= 1.3: the ``manta`` backend no longer exists (``init`` fails), so the executor runs a
  local backend in its work dir and carries ``terraform.tfstate`` to and from Manta
  under the Manta lock (reference ``backend/manta/backend.go:196-205``,
  ``shell/run_terraform.go:11-80``);
* the modules' ``required_version`` (``>= 1.4``: they use ``terraform_data``).
"""

import json
import os
import subprocess
import sys

import pytest

from triton_kubernetes_amd import workflows as wf
from triton_kubernetes_amd.backend import LocalBackend
from triton_kubernetes_amd.backend.manta import MantaBackend
from triton_kubernetes_amd.cloud.fake_manta import FakeManta
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.executor.terraform import render
from triton_kubernetes_amd.state import State
from triton_kubernetes_amd.terraform import catalog, constraints, hcl
from triton_kubernetes_amd.terraform.generate import REQUIRED_VERSION, modules
from triton_kubernetes_amd.terraform.plan import plan_root
from triton_kubernetes_amd.utils.sshkeys import load_private_key

from helpers import FAKE_TF, install_fake_terraform, make_ctx, make_ssh_key, output, tf_calls

PW = "tk-admin-pw-0123"
MGR = {"manager_cloud_provider": "baremetal", "name": "mgr", "rancher_admin_password": PW, "host": "10.0.0.10",
       "ssh_user": "ubuntu", "bastion_host": "", "key_path": "~/.ssh/id_rsa", "executor": "terraform"}
CLUSTER = {"cluster_manager": "mgr", "cluster_cloud_provider": "baremetal", "name": "dev",
           "k8s_version": "v1.28.10-rancher1-1", "k8s_network_provider": "flannel", "executor": "terraform",
           "nodes": [{"rancher_host_label": "worker", "node_count": 2, "hostname": "dev-w", "ssh_user": "u",
                      "key_path": "k", "bastion_host": "", "hosts": ["10.0.0.13", "10.0.0.14"]}]}


@pytest.fixture
def manta(tmp_path):
    key_path = make_ssh_key(tmp_path / "id_rsa")
    key = load_private_key(key_path)
    fake = FakeManta("acct").start()
    fake.add_key(key)
    be = MantaBackend("acct", key_path, key.fingerprint_md5(), "https://triton", fake.url)
    yield fake, be
    fake.stop()


def _fake_tf(tmp_path, doc, *argv, version="1.5.7"):
    d = tmp_path / "wd"
    d.mkdir(exist_ok=True)
    (d / "main.tf.json").write_text(json.dumps(doc))
    env = dict(os.environ, FAKE_TF_VERSION=version)
    env.pop("FAKE_TF_LOG", None)
    return subprocess.run([sys.executable, FAKE_TF, *argv], cwd=d, env=env, capture_output=True, text=True)


def _manager_state(backend_block=None):
    st = State("mgr")
    src = catalog.module_source(catalog.PACKAGE_ROOT, "terraform/modules/bare-metal-rancher", "x")
    st.set_manager({"source": src, "name": "mgr", "host": "h", "rancher_admin_password": PW})
    if backend_block:
        st.set_terraform_backend_config(*backend_block)
    return st


# --- the rules themselves ---------------------------------------------------------------------
def test_catalog_sensitivity_matches_module_files():
    """The executor's sensitivity source (the generator) agrees with every outputs.tf."""
    for mod in modules():
        body = hcl.check_module(os.path.join(catalog.MODULES_DIR, mod.name)).files["outputs.tf"]
        declared = {b.labels[0]: b.body.attr("sensitive") is not None for b in body.blocks if b.type == "output"}
        assert set(declared) == set(catalog.CATALOG[mod.name].outputs), mod.name
        assert {n for n, s in declared.items() if s} == set(catalog.sensitive_outputs(mod.name)), mod.name
    assert "rancher_secret_key" in catalog.sensitive_outputs("bare-metal-rancher")
    assert "rancher_cluster_registration_token" in catalog.sensitive_outputs("triton-rancher-k8s")


def test_rendered_root_outputs_are_marked_sensitive():
    doc = json.loads(render(_manager_state(), (1, 5, 7)).body)
    assert doc["output"]["cluster-manager__rancher_secret_key"]["sensitive"] is True
    assert "sensitive" not in doc["output"]["cluster-manager__rancher_url"]
    assert plan_root(doc, (1, 5, 7)) == []


def test_fake_terraform_rejects_unmarked_sensitive_root_output(tmp_path):
    doc = json.loads(render(_manager_state(), (1, 5, 7)).body)
    doc["output"]["cluster-manager__rancher_secret_key"].pop("sensitive")
    res = _fake_tf(tmp_path, doc, "apply", "-auto-approve")
    assert res.returncode == 1 and "Output refers to sensitive values" in res.stderr
    assert any("sensitive" in e for e in plan_root(doc, (1, 5, 7)))
    # 0.14 did not have the rule
    assert _fake_tf(tmp_path, doc, "apply", version="0.14.11").returncode == 0
    assert plan_root(doc, (0, 14, 11)) == [] or all("required_version" in e for e in plan_root(doc, (0, 14, 11)))


def test_fake_terraform_and_plan_reject_manta_backend_from_1_3(tmp_path):
    doc = {"terraform": {"backend": {"manta": {"account": "a", "key_material": "k", "key_id": "i",
                                               "path": "/triton-kubernetes/mgr"}}}}
    res = _fake_tf(tmp_path, doc, "init", "-force-copy")
    assert res.returncode == 1 and 'There is no backend type named "manta"' in res.stderr
    assert _fake_tf(tmp_path, doc, "init", version="1.2.9").returncode == 0
    assert any("manta" in e for e in plan_root(doc, (1, 3, 0)))
    assert plan_root(doc, (1, 2, 9)) == []


def test_required_version_is_1_4_everywhere():
    assert REQUIRED_VERSION == ">= 1.4"
    for name in catalog.CATALOG:
        reqs = constraints.required_versions(os.path.join(catalog.MODULES_DIR, name))
        assert reqs == [">= 1.4"], name
        uses_tfdata = "terraform_data" in open(os.path.join(catalog.MODULES_DIR, name, "main.tf")).read()
        if uses_tfdata:
            assert not constraints.satisfies((1, 3, 9), reqs[0])


def test_constraint_grammar():
    s = constraints.satisfies
    assert s((1, 4, 0), ">= 1.4") and not s((1, 3, 9), ">= 1.4")
    assert s((1, 5, 7), "~> 1.4") and not s((2, 0, 0), "~> 1.4")
    assert s((1, 4, 9), "~> 1.4.2") and not s((1, 5, 0), "~> 1.4.2") and not s((1, 4, 1), "~> 1.4.2")
    assert s((1, 6, 0), ">= 1.4, < 2.0") and not s((2, 1, 0), ">= 1.4, < 2.0")
    assert s((0, 11, 2), "0.11.2") and not s((0, 11, 3), "= 0.11.2") and s((1, 0, 0), "!= 0.11.2")


def test_too_old_terraform_fails_before_init(tmp_path, monkeypatch):
    log = install_fake_terraform(tmp_path, monkeypatch, version="1.3.9")
    with pytest.raises(TKError, match=r"requires Terraform >= 1.4; found v1.3.9"):
        wf.new_manager(make_ctx(MGR), LocalBackend(str(tmp_path / "s")))
    assert [c["argv"][0] for c in tf_calls(log)] == ["version"]


# --- Manta-backed runs through the executor ---------------------------------------------------------
def test_manta_create_get_destroy_with_terraform_1_5(tmp_path, monkeypatch, manta):
    fake, be = manta
    log = install_fake_terraform(tmp_path, monkeypatch, version="1.5.7")
    tfstate = "/acct/stor/triton-kubernetes/mgr/terraform.tfstate"

    wf.new_manager(make_ctx(dict(MGR, backend_provider="manta")), be)
    calls = tf_calls(log)
    init = next(c for c in calls if c["argv"][0] == "init")
    assert init["doc"]["terraform"]["backend"] == {"local": {"path": "terraform.tfstate"}}
    persisted = json.loads(be.state("mgr").bytes())
    assert "manta" in persisted["terraform"]["backend"]  # the stored document keeps the reference layout
    st1 = json.loads(fake.objects[tfstate][0])
    assert st1["serial"] == 1 and [r["module"] for r in st1["resources"]] == ["module.cluster-manager"]

    open(log, "w").close()
    wf.new_cluster(make_ctx(dict(CLUSTER, backend_provider="manta")), be)
    apply = next(c for c in tf_calls(log) if c["argv"][0] == "apply")
    # the apply started from the state the manager's apply left in Manta
    assert apply["prior"]["serial"] == 1 and apply["prior"]["lineage"] == st1["lineage"]
    assert apply["prior"]["modules"] == ["cluster-manager"]
    st2 = json.loads(be.read_tfstate("mgr"))
    assert st2["serial"] == 2 and st2["lineage"] == st1["lineage"] and len(st2["resources"]) == 4

    ctx = make_ctx({"cluster_manager": "mgr", "executor": "terraform"})
    wf.get_manager(ctx, be)
    assert "rancher_secret_key = fake-cluster-manager__rancher_secret_key" in output(ctx)
    assert json.loads(be.read_tfstate("mgr"))["serial"] == 2  # get does not write state back

    wf.delete_node(make_ctx({"cluster_manager": "mgr", "cluster_name": "dev", "hostname": "dev-w-2",
                             "executor": "terraform"}), be)
    st3 = json.loads(be.read_tfstate("mgr"))
    assert st3["serial"] == 3 and "module.node_baremetal_dev_dev-w-2" not in [r["module"] for r in st3["resources"]]

    wf.delete_manager(make_ctx({"cluster_manager": "mgr", "executor": "terraform"}), be)
    assert be.states() == [] and not any("/triton-kubernetes/mgr" in p for p in fake.objects)
    assert fake.rejected == 0
    assert "/acct/stor/triton-kubernetes/mgr/.lock" not in fake.objects


def test_manta_failed_apply_still_uploads_partial_state(tmp_path, monkeypatch, manta):
    fake, be = manta
    install_fake_terraform(tmp_path, monkeypatch, version="1.5.7")
    wf.new_manager(make_ctx(dict(MGR, backend_provider="manta")), be)
    install_fake_terraform(tmp_path, monkeypatch, version="1.5.7", fail="apply")
    with pytest.raises(TKError):
        wf.new_cluster(make_ctx(dict(CLUSTER, backend_provider="manta")), be)
    st = json.loads(be.read_tfstate("mgr"))
    # the fake creates half of the 3 new modules before failing; Manta has them recorded
    assert st["serial"] == 2 and len(st["resources"]) == 2
    assert "/acct/stor/triton-kubernetes/mgr/.lock" not in fake.objects


def test_manta_with_terraform_1_2_keeps_native_backend(tmp_path, monkeypatch, manta):
    """Before 1.3 Terraform still has the manta backend: the block goes through as is
    (reference-era modules, which 1.2 can run; the packaged ones need 1.4)."""
    fake, be = manta
    log = install_fake_terraform(tmp_path, monkeypatch, version="1.2.9")
    wf.new_manager(make_ctx(dict(MGR, backend_provider="manta", source_url="github.com/joyent/triton-kubernetes",
                                 source_ref="master")), be)
    init = next(c for c in tf_calls(log) if c["argv"][0] == "init")
    assert "manta" in init["doc"]["terraform"]["backend"]
    assert be.read_tfstate("mgr") is None  # Terraform itself talks to Manta (the fake keeps it aside)


def test_manta_lock_is_reentrant_and_renewed(manta, monkeypatch):
    import threading
    import time

    fake, be = manta
    path = "/acct/stor/triton-kubernetes/mgr/.lock"
    # TTL and waits sized for a loaded CPU (every Manta request is signed): the heartbeat
    # renews well inside the TTL, and the other writer's wait spans more than one TTL
    with be.lock("mgr", ttl=1.5):
        first = fake.objects[path]
        with be.lock("mgr"):  # same thread: no deadlock
            pass
        assert path in fake.objects
        time.sleep(2.0)  # past the TTL: the heartbeat has re-PUT it
        assert fake.objects[path] != first
        got = []

        def other():
            try:
                with be.lock("mgr", timeout=1.8, poll=0.05):
                    got.append(True)
            except TKError:
                got.append(False)

        t = threading.Thread(target=other)
        t.start()
        t.join()
        assert got == [False]  # still held: never looked expired
    assert path not in fake.objects


def test_manta_lock_lost_to_a_takeover_refuses_writes(manta):
    """a holder whose lock expired and was taken over (a suspended laptop) must
    not go on writing the tfstate / document over the new holder's."""
    import time

    from triton_kubernetes_amd.errors import BackendError

    fake, be = manta
    path = "/acct/stor/triton-kubernetes/mgr/.lock"
    st = State("mgr")
    with be.lock("mgr", ttl=0.3):
        be.persist_state(st)  # held: fine
        # another CLI found the lock expired and replaced it (If-Match on the old etag)
        fake.objects[path] = (json.dumps({"token": "other", "expires": time.time() + 900}).encode(),
                              "application/json", "etag-of-the-other-writer")
        # the heartbeat's If-Match fails: the lock is lost (waited for, not slept on: the
        # heartbeat may run late on a loaded CPU)
        lost = be._held.lost["mgr"]
        assert lost.wait(10)
        with pytest.raises(BackendError, match="taken over by another writer"):
            be.write_tfstate("mgr", b"{}")
        with pytest.raises(BackendError, match="taken over"):
            be.persist_state(st)
    assert json.loads(fake.objects[path][0])["token"] == "other"  # the new holder's lock is left alone
    del fake.objects[path]
    with be.lock("mgr"):
        be.persist_state(st)  # a fresh lock writes again
