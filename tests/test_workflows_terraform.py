"""create / destroy / get through the TerraformExecutor against a fake ``terraform``.

Covers the reference flows of SURVEY.md §3.1-3.5 end to end: temp dir +
``main.tf.json``, ``init -force-copy``, ``apply -auto-approve``, version-aware
destroy flags and outputs, persist-after-apply, failure semantics.
"""

import json
import os

import pytest

from triton_kubernetes_amd.backend import LocalBackend
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.executor.terraform import TerraformExecutor, parse_version, render_document
from triton_kubernetes_amd.state import State
from triton_kubernetes_amd.workflows import (delete_cluster, delete_manager, delete_node, get_cluster, get_manager,
                                              new_cluster, new_manager, new_node)
from triton_kubernetes_amd.workflows.create import read_status

from helpers import install_fake_terraform, make_ctx, output, tf_calls

MGR = {"manager_cloud_provider": "baremetal", "name": "mgr", "rancher_admin_password": "tk-admin-pw-0123", "host": "10.0.0.10",
       "ssh_user": "ubuntu", "bastion_host": "", "key_path": "~/.ssh/id_rsa", "executor": "terraform"}
CLUSTER = {"cluster_manager": "mgr", "cluster_cloud_provider": "baremetal", "name": "dev",
           "k8s_version": "v1.28.10-rancher1-1", "k8s_network_provider": "flannel", "executor": "terraform",
           "nodes": [
               {"rancher_host_label": "etcd", "node_count": 1, "hostname": "dev-etcd", "ssh_user": "ubuntu",
                "key_path": "~/.ssh/id_rsa", "bastion_host": "", "hosts": ["10.0.0.11"]},
               {"rancher_host_label": "control", "node_count": 1, "hostname": "dev-control", "ssh_user": "ubuntu",
                "key_path": "~/.ssh/id_rsa", "bastion_host": "", "hosts": ["10.0.0.12"]},
               {"rancher_host_label": "worker", "node_count": 2, "hostname": "dev-worker", "ssh_user": "ubuntu",
                "key_path": "~/.ssh/id_rsa", "bastion_host": "", "hosts": ["10.0.0.13", "10.0.0.14"]},
           ]}


@pytest.fixture
def backend(tmp_path):
    return LocalBackend(str(tmp_path / "state"))


def test_create_manager_cluster_node_and_destroy(tmp_path, monkeypatch, backend):
    log = install_fake_terraform(tmp_path, monkeypatch, version="1.5.7")
    new_manager(make_ctx(MGR), backend)
    calls = tf_calls(log)
    # the apply, then the read-back of the SSH host keys its key read pinned (parallel/hostkeys.py)
    assert [c["argv"][0] for c in calls] == ["version", "init", "apply", "output"]
    assert calls[1]["argv"] == ["init", "-force-copy", "-input=false"]
    assert calls[2]["argv"] == ["apply", "-auto-approve", "-input=false"]
    assert os.path.basename(calls[2]["cwd"]).startswith("triton-kubernetes-")
    assert not os.path.exists(calls[2]["cwd"])  # temp dir removed
    doc = calls[2]["doc"]
    assert doc["terraform"]["backend"]["local"]["path"] == os.path.join(backend.root, "mgr", "terraform.tfstate")
    assert doc["output"]["cluster-manager__rancher_url"] == {"value": "${module.cluster-manager.rancher_url}"}
    persisted = json.loads(open(os.path.join(backend.root, "mgr", "main.tf.json")).read())
    assert "output" not in persisted  # rendered only for Terraform >= 0.12
    assert backend.states() == ["mgr"]

    ctx = make_ctx(CLUSTER)
    new_cluster(ctx, backend)
    assert "2 nodes added: dev-worker-1, dev-worker-2" in output(ctx)
    st = backend.state("mgr")
    assert sorted(st.nodes("cluster_baremetal_dev")) == ["dev-control-1", "dev-etcd-1", "dev-worker-1",
                                                          "dev-worker-2"]

    # get manager / cluster read the root outputs
    ctx = make_ctx({"cluster_manager": "mgr", "executor": "terraform"})
    get_manager(ctx, backend)
    assert "rancher_url = fake-cluster-manager__rancher_url" in output(ctx)
    ctx = make_ctx({"cluster_manager": "mgr", "cluster_name": "dev", "executor": "terraform"})
    get_cluster(ctx, backend)
    assert "rancher_cluster_id = fake-cluster_baremetal_dev__rancher_cluster_id" in output(ctx)

    # add one more worker
    new_node(make_ctx({"cluster_manager": "mgr", "cluster_name": "dev", "rancher_host_label": "worker",
                       "node_count": 1, "hostname": "dev-worker", "ssh_user": "u", "bastion_host": "",
                       "key_path": "k", "hosts": ["10.0.0.15"], "executor": "terraform"}), backend)
    assert "dev-worker-3" in backend.state("mgr").nodes("cluster_baremetal_dev")

    # destroy one node: -target=module.<node>, and the >=0.15 flag
    open(log, "w").close()
    delete_node(make_ctx({"cluster_manager": "mgr", "cluster_name": "dev", "hostname": "dev-worker-3",
                          "executor": "terraform"}), backend)
    destroy = [c for c in tf_calls(log) if c["argv"][0] == "destroy"][0]
    # the state is authoritative for a destroy: no refresh (which would re-run the create-side
    # data sources), and the modules' data sources told it is a destroy should one run
    assert destroy["argv"] == ["destroy", "-auto-approve", "-refresh=false", "-var=tk_operation=destroy",
                               "-target=module.node_baremetal_dev_dev-worker-3"]
    assert destroy["doc"]["variable"]["tk_operation"] == {"type": "string", "default": "apply"}
    assert destroy["doc"]["module"]["cluster_baremetal_dev"]["tk_operation"] == "${var.tk_operation}"
    assert "dev-worker-3" not in backend.state("mgr").nodes("cluster_baremetal_dev")

    # destroy the cluster: cluster + every node targeted, modules removed
    open(log, "w").close()
    delete_cluster(make_ctx({"cluster_manager": "mgr", "cluster_name": "dev", "executor": "terraform"}), backend)
    destroy = [c for c in tf_calls(log) if c["argv"][0] == "destroy"][0]
    assert destroy["argv"][:5] == ["destroy", "-auto-approve", "-refresh=false", "-var=tk_operation=destroy",
                                    "-target=module.cluster_baremetal_dev"]
    assert len(destroy["argv"]) == 5 + 4
    assert backend.state("mgr").clusters() == {}

    delete_manager(make_ctx({"cluster_manager": "mgr", "executor": "terraform"}), backend)
    assert backend.states() == []


def test_terraform_011_flags_and_module_outputs(tmp_path, monkeypatch, backend):
    """0.11 runs the reference's own (0.11-syntax) modules; the packaged ones need >= 1.4."""
    log = install_fake_terraform(tmp_path, monkeypatch, version="0.11.2")
    new_manager(make_ctx(dict(MGR, source_url="github.com/joyent/triton-kubernetes", source_ref="master")), backend)
    apply = [c for c in tf_calls(log) if c["argv"][0] == "apply"][0]
    assert "output" not in apply["doc"]  # 0.11: no rendered root outputs
    open(log, "w").close()
    delete_manager(make_ctx({"cluster_manager": "mgr", "executor": "terraform"}), backend)
    destroy = [c for c in tf_calls(log) if c["argv"][0] == "destroy"][0]
    assert destroy["argv"] == ["destroy", "-force", "-refresh=false"]  # reference modules: no tk_operation


def test_duplicate_manager_name_and_failed_apply_resume(tmp_path, monkeypatch, backend):
    install_fake_terraform(tmp_path, monkeypatch)
    new_manager(make_ctx(MGR), backend)
    with pytest.raises(TKError) as exc:
        new_manager(make_ctx(MGR), backend)
    assert str(exc.value) == "A Cluster Manager with the name 'mgr' already exists."

    install_fake_terraform(tmp_path, monkeypatch, fail="apply")
    with pytest.raises(TKError) as exc:
        new_manager(make_ctx(dict(MGR, name="broken")), backend)
    assert "exit status 1" in str(exc.value)
    assert "broken" in backend.states()  # desired state persisted for cleanup / resume
    assert read_status(backend, "broken")["phase"] == "apply_failed"
    install_fake_terraform(tmp_path, monkeypatch)
    ctx = make_ctx(dict(MGR, name="broken"))
    new_manager(ctx, backend)  # resumes instead of "already exists"
    assert "Resuming creation of 'broken'" in output(ctx)
    assert read_status(backend, "broken")["phase"] == "applied"


def test_unsupported_providers(backend, tmp_path, monkeypatch):
    install_fake_terraform(tmp_path, monkeypatch)
    with pytest.raises(TKError) as exc:
        new_manager(make_ctx(dict(MGR, manager_cloud_provider="vsphere")), backend)
    assert str(exc.value) == "Unsupported cloud provider 'vsphere', cannot create manager"
    new_manager(make_ctx(MGR), backend)
    with pytest.raises(TKError) as exc:
        new_cluster(make_ctx(dict(CLUSTER, cluster_cloud_provider="ibm")), backend)
    assert str(exc.value) == "Unsupported cloud provider 'ibm', cannot create cluster"
    with pytest.raises(TKError) as exc:
        new_cluster(make_ctx({}), LocalBackend(str(tmp_path / "empty")))
    assert str(exc.value) == \
        "No cluster managers, please create a cluster manager before creating a kubernetes cluster."


def test_interactive_cancel_does_not_apply(tmp_path, monkeypatch, backend):
    log = install_fake_terraform(tmp_path, monkeypatch)
    vals = dict(MGR)
    vals.pop("name")
    ctx = make_ctx(vals, answers=["mgr2", "", "", "", "No"], non_interactive=False)
    new_manager(ctx, backend)
    assert "Manager creation canceled." in output(ctx)
    assert not [c for c in tf_calls(log) if c["argv"][0] == "apply"]
    assert backend.states() == []


def test_version_parsing_and_render():
    assert parse_version("Terraform v0.11.2\n") == (0, 11, 2)
    assert parse_version('{"terraform_version": "1.6.0"}') == (1, 6, 0)
    st = State("x")
    st.add_cluster("aws", "c", {"source": "x//terraform/modules/aws-rancher-k8s?ref=m", "name": "c"})
    doc = json.loads(render_document(st, (1, 0, 0)))
    assert "cluster_aws_c__aws_subnet_id" in doc["output"]
    assert TerraformExecutor(version=(0, 14, 0)).destroy_flags() == ["-force"]
    assert TerraformExecutor(version=(1, 0, 0)).destroy_flags() == ["-auto-approve"]


def test_missing_terraform_binary(tmp_path, monkeypatch, backend):
    monkeypatch.setenv("PATH", str(tmp_path))
    with pytest.raises(TKError) as exc:
        new_manager(make_ctx(MGR), backend)
    assert str(exc.value).startswith('exec: "terraform": executable file not found in $PATH')
