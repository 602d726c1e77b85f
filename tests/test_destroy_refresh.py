"""A destroy never runs the create-side data sources.

The modules read two things through ``data "external"`` (reference
``terraform/modules/triton-rancher/main.tf:128-144``, ``rancher_cluster.sh:17-42``):

* the manager's API key, over SSH to the manager host (``read_api_key.sh``);
* the Rancher cluster, found *or created* by name (``ensure_cluster.sh``).

Terraform reads data sources while refreshing, and ``terraform destroy`` refreshes first
unless told not to.  So, before this change, ``destroy manager`` could never succeed once
the manager host was gone, and ``destroy node`` re-created a Rancher cluster that had
been removed out of band.  The executor now destroys with ``-refresh=false`` (the state is
authoritative) and sets the modules' ``tk_operation`` to ``destroy``, which makes both
programs find-only and tolerant of a host that is gone.

The fake Terraform runs the modules' real programs during refresh here
(``FAKE_TF_EXTERNAL=1``), against a fake ``ssh`` (``fixtures/fake_ssh.py``) and the
in-process Rancher fake; each test also runs the destroy the way the old code did, to
show the hazard is real in the fake.
"""

import json
import os
import shutil
import subprocess
import sys

import pytest

from triton_kubernetes_amd import workflows as wf
from triton_kubernetes_amd.backend import LocalBackend
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.executor.terraform import TerraformExecutor, render
from triton_kubernetes_amd.models import baremetal
from triton_kubernetes_amd.rancher.client import RancherClient
from triton_kubernetes_amd.rancher.fake import FakeRancher
from triton_kubernetes_amd.terraform import catalog

from helpers import FAKE_TF, HERE, install_fake_terraform, make_ctx, tf_calls

PW = "tk-admin-pw-0123"
MGR = {"manager_cloud_provider": "baremetal", "name": "mgr", "rancher_admin_password": PW, "host": "10.0.0.10",
       "ssh_user": "ubuntu", "bastion_host": "", "key_path": "~/.ssh/id_rsa", "executor": "terraform"}
API_KEY = {"name": "token-tk", "token": "token-tk:s3cret"}


@pytest.fixture
def env(tmp_path, monkeypatch):
    log = install_fake_terraform(tmp_path, monkeypatch)
    monkeypatch.setenv("FAKE_TF_EXTERNAL", "1")
    ssh = tmp_path / "bin" / "ssh"
    ssh.write_text(f"#!/bin/sh\nexec {sys.executable} {os.path.join(HERE, 'fixtures', 'fake_ssh.py')} \"$@\"\n")
    ssh.chmod(0o755)
    hosts = tmp_path / "hosts"
    hosts.mkdir()
    monkeypatch.setenv("FAKE_SSH_HOSTS", str(hosts))
    (hosts / "10.0.0.10").mkdir()
    (hosts / "10.0.0.10" / "rancher_api_key").write_text(json.dumps(API_KEY))
    return log, hosts, LocalBackend(str(tmp_path / "state"))


def _run_fake(tmp_path, state, *argv):
    """The fake Terraform on the rendered document, as an old executor would have run it."""
    d = tmp_path / f"wd-{len(os.listdir(tmp_path))}"
    d.mkdir()
    (d / "main.tf.json").write_bytes(render(state, (1, 5, 7)).body)
    return subprocess.run([sys.executable, FAKE_TF, *argv], cwd=d, capture_output=True, text=True,
                          env=dict(os.environ, FAKE_TF_LOG=""))


def test_destroy_manager_after_its_host_is_gone(tmp_path, env):
    log, hosts, be = env
    wf.new_manager(make_ctx(MGR), be)
    ctx = make_ctx({"cluster_manager": "mgr", "executor": "terraform"})
    wf.get_manager(ctx, be)
    assert "rancher_access_key = token-tk" in ctx.out.getvalue()  # read over (fake) SSH at apply

    shutil.rmtree(hosts / "10.0.0.10")  # the manager machine is gone
    st = be.state("mgr")
    # the hazard: a destroy that refreshes runs read_api_key.sh against the missing host
    old = _run_fake(tmp_path, st, "destroy", "-auto-approve")
    assert old.returncode == 1 and "External Program Execution Failed" in old.stderr
    assert "No route to host" in old.stderr
    # an apply still needs the host, and says so
    with pytest.raises(TKError):  # (Terraform's own error went to the inherited stderr)
        TerraformExecutor().apply(st, be)
    # should Terraform refresh anyway, the script knows it is a destroy
    assert _run_fake(tmp_path, st, "destroy", "-auto-approve", "-var=tk_operation=destroy").returncode == 0

    open(log, "w").close()
    wf.delete_manager(make_ctx({"cluster_manager": "mgr", "executor": "terraform"}), be)
    destroy = [c for c in tf_calls(log) if c["argv"][0] == "destroy"][0]
    assert "-refresh=false" in destroy["argv"]
    assert be.states() == []


@pytest.fixture
def rancher():
    fake = FakeRancher(bootstrap_password="b00tstrap-only").start()
    outs = RancherClient(fake.url).bootstrap("n3w-passw0rd-123", fake.url, "b00tstrap-only", timeout=10)
    yield fake, RancherClient(fake.url, outs["rancher_access_key"], outs["rancher_secret_key"]), outs
    fake.stop()


def _cluster_names(fake):
    return sorted(c.get("name") for c in fake.state.clusters.values())


def test_destroy_node_does_not_recreate_a_cluster_removed_out_of_band(tmp_path, env, rancher):
    log, hosts, be = env
    fake, client, outs = rancher
    st = be.state("mgr")
    baremetal.new_manager(make_ctx(MGR), st, "mgr")
    name = baremetal.new_cluster(make_ctx({"name": "dev", "k8s_version": "v1.28.10-rancher1-1",
                                           "k8s_network_provider": "flannel"}), None, st)
    key = st.clusters()[name]
    cluster = st.module(key)
    # the cluster talks to the in-process Rancher (the manager module's own URL is https://<host>)
    cluster.update(rancher_api_url=fake.url, rancher_access_key=outs["rancher_access_key"],
                   rancher_secret_key=outs["rancher_secret_key"])
    st.set_module(key, cluster)
    baremetal.new_node(make_ctx({"rancher_host_label": "worker", "node_count": 2, "hostname": "dev-w",
                                 "ssh_user": "u", "bastion_host": "", "key_path": "k",
                                 "hosts": ["10.0.0.13", "10.0.0.14"]}), "mgr", key, None, st)
    st.set_terraform_backend_config(*be.state_terraform_config("mgr"))
    TerraformExecutor().apply(st, be)  # ensure_cluster.sh creates "dev"
    be.persist_state(st)
    assert _cluster_names(fake) == ["dev"]
    cid = client.find_cluster("dev")["id"]
    # the data source's result became the module's output
    assert json.loads(be.read_tfstate("mgr"))["outputs"][f"{key}__rancher_cluster_id"]["value"] == cid

    client.delete_cluster(cid)  # removed out of band (Rancher UI, another tool)
    assert _cluster_names(fake) == []

    # with tk_operation=destroy a refreshing destroy only looks: nothing re-created
    res = _run_fake(tmp_path, be.state("mgr"), "destroy", "-auto-approve", "-var=tk_operation=destroy",
                    "-target=module.node_baremetal_dev_dev-w-2")
    assert res.returncode == 0, res.stderr
    assert _cluster_names(fake) == []

    open(log, "w").close()
    wf.delete_node(make_ctx({"cluster_manager": "mgr", "cluster_name": "dev", "hostname": "dev-w-1",
                             "executor": "terraform"}), be)
    destroy = [c for c in tf_calls(log) if c["argv"][0] == "destroy"][0]
    assert destroy["argv"][:4] == ["destroy", "-auto-approve", "-refresh=false", "-var=tk_operation=destroy"]
    assert _cluster_names(fake) == []  # still gone
    assert "dev-w-1" not in be.state("mgr").nodes(key)

    # the hazard, for the record: the old destroy (refresh, operation apply) re-creates it
    old = _run_fake(tmp_path, be.state("mgr"), "destroy", "-auto-approve", "-target=module.node_baremetal_dev_dev-w-2")
    assert old.returncode == 0, old.stderr
    assert _cluster_names(fake) == ["dev"]


def test_find_only_scripts_outside_apply(tmp_path, env, rancher):
    """The programs themselves: find-only and tolerant of a missing host / Rancher."""
    _, hosts, _ = env
    fake, client, outs = rancher
    mod = os.path.join(catalog.MODULES_DIR, "bare-metal-rancher-k8s", "files", "ensure_cluster.sh")
    q = {"name": "ghost", "version": "v1.28.10-rancher1-1", "network": "flannel", "distribution": "rke1",
         "api_url": fake.url, "access_key": outs["rancher_access_key"], "secret_key": outs["rancher_secret_key"]}
    for op in ("destroy", "read"):
        res = subprocess.run(["bash", mod], input=json.dumps(dict(q, operation=op)), capture_output=True, text=True,
                             timeout=60)
        assert res.returncode == 0 and json.loads(res.stdout) == {"cluster_id": "", "registration_token": "",
                                                                 "ca_checksum": ""}
    assert "ghost" not in _cluster_names(fake)
    created = json.loads(subprocess.run(["bash", mod], input=json.dumps(dict(q, operation="apply")),
                                        capture_output=True, text=True, timeout=60, check=True).stdout)
    found = json.loads(subprocess.run(["bash", mod], input=json.dumps(dict(q, operation="destroy")),
                                      capture_output=True, text=True, timeout=60, check=True).stdout)
    assert found == created  # an existing cluster is reported as is
    gone = subprocess.run(["bash", mod], input=json.dumps(dict(q, api_url="http://127.0.0.1:9", operation="destroy")),
                          capture_output=True, text=True, timeout=60)
    assert gone.returncode == 0 and json.loads(gone.stdout)["cluster_id"] == ""

    read_key = os.path.join(catalog.MODULES_DIR, "bare-metal-rancher", "files", "read_api_key.sh")
    labels = os.path.join(catalog.MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host", "files", "read_gpu_labels.sh")
    down = {"host": "10.9.9.9", "ssh_user": "u", "key_path": "k", "bastion_host": ""}
    for script, empty in ((read_key, {"access_key": "", "secret_key": "", "known_hosts": "", "ca_certs": ""}),
                          (labels, {"labels": "{}", "known_hosts": ""})):
        res = subprocess.run(["bash", script], input=json.dumps(dict(down, operation="destroy")), capture_output=True,
                             text=True, timeout=60)
        assert res.returncode == 0 and json.loads(res.stdout) == empty, res.stderr
        res = subprocess.run(["bash", script], input=json.dumps(dict(down, operation="apply")), capture_output=True,
                             text=True, timeout=60)
        assert res.returncode != 0 and "10.9.9.9" in res.stderr
    res = subprocess.run(["bash", read_key], input=json.dumps({"host": "10.0.0.10", "ssh_user": "u", "key_path": "k",
                                                               "bastion_host": "", "operation": "apply"}),
                         capture_output=True, text=True, timeout=60, check=True)
    got = json.loads(res.stdout)
    assert (got["access_key"], got["secret_key"]) == ("token-tk", "s3cret")
    assert got["known_hosts"].startswith("10.0.0.10 ssh-ed25519 ")  # first contact: pinned and reported


def test_fake_terraform_refuses_undeclared_var(tmp_path):
    d = tmp_path / "wd"
    d.mkdir()
    (d / "main.tf.json").write_text("{}")
    res = subprocess.run([sys.executable, FAKE_TF, "destroy", "-auto-approve", "-var=tk_operation=destroy"], cwd=d,
                         capture_output=True, text=True)
    assert res.returncode == 1 and "Value for undeclared variable" in res.stderr
