"""The reference's own silent-install examples (``/root/reference/examples/silent-install``),
unmodified, through this CLI: what a user switching over meets, one refusal at a time, each
cleared by one change to the file.

``create-manager.yaml``:
1. it lacks ``manager_cloud_provider``, which the reference CLI refuses in
   non-interactive mode (``/root/reference/create/manager.go:33-36``) with
   ``manager_cloud_provider must be specified``; so does this one;
2. ``rancher_admin_password: admin``: Rancher v2.10 takes 12 characters or more;
3. ``master_triton_machine_package: k4-highcpu-kvm-1.75G``: too small for the Rancher
   v2.10 server.

``cluster-triton-ha.yaml``:
1. Kubernetes ``v1.8.10-rancher1-1``, which the reference's Rancher offered
   (``/root/reference/create/cluster.go:349-356``) and Rancher v2.10 does not;
2. ``triton_machine_package: k4-highcpu-kvm-1.75G`` on every node group: too small for a
   Kubernetes node.
After that it creates the same 3 etcd / 3 control / 4 worker layout under the same
hostnames.

Skipped where the reference tree is not present."""

import json
import os

import pytest
import yaml

from triton_kubernetes_amd import versions
from triton_kubernetes_amd.cli.main import run

from helpers import install_fake_terraform, make_ssh_key

EX = "/root/reference/examples/silent-install"
pytestmark = pytest.mark.skipif(not os.path.isdir(EX), reason="reference tree not present")

# (what the previous refusal asked to change, the refusal that follows it; None: it runs)
MANAGER_STEPS = [
    ({}, "manager_cloud_provider must be specified"),
    ({"manager_cloud_provider": "triton"}, "UI Admin password must be at least 12 characters"),
    ({"rancher_admin_password": "a-longer-admin-pw"}, "has 1.75 GiB of memory"),
    ({"master_triton_machine_package": "k4-highcpu-kvm-7.75G"}, None),
]
CLUSTER_STEPS = [
    ({}, "Kubernetes version 'v1.8.10-rancher1-1' is not an RKE1 release offered by Rancher"),
    ({"k8s_version": versions.DEFAULT_K8S_VERSION}, "has 1.75 GiB of memory"),
    ({"nodes": lambda nodes: [dict(n, triton_machine_package="k4-highcpu-kvm-7.75G") for n in nodes]}, None),
]


def _cli(*argv):
    import io

    out = io.StringIO()
    return run(list(argv), out=out), out.getvalue()


def _walk(tmp_path, name, cmd, steps, **base):
    """Apply the steps' changes one after the other; each run must end with the refusal the
    step names (and change nothing), the last one must pass."""
    doc = yaml.safe_load(open(os.path.join(EX, name)))
    for change, refusal in [(base, "")] + list(steps):
        if refusal == "":  # the test's own settings (key, offline, executor), not a step
            refusal = None
        for k, v in change.items():
            if v is None:
                doc.pop(k, None)
            elif callable(v):  # a change to every entry of a list (the node groups)
                doc[k] = v(doc[k])
            else:
                doc[k] = v
        if change is base:
            continue
        path = tmp_path / name
        path.write_text(yaml.safe_dump(doc))
        code, out = _cli("--non-interactive", "--config", str(path), "create", cmd)
        if refusal is None:
            assert code == 0, out
        else:
            assert code != 0 and refusal in out.strip().splitlines()[-1], (change, out)
    return out


def test_reference_manager_example_is_refused_as_the_reference_refuses_it(tk_home):
    code, out = _cli("--non-interactive", "--config", os.path.join(EX, "create-manager.yaml"), "create", "manager")
    assert code != 0
    assert out.strip().splitlines()[-1] == "manager_cloud_provider must be specified"
    assert not (tk_home / ".triton-kubernetes" / "test-manager").exists()


def test_reference_examples_create_after_the_listed_changes(tk_home, tmp_path, monkeypatch):
    install_fake_terraform(tmp_path, monkeypatch)
    key = make_ssh_key(tmp_path / "id_rsa")
    base = dict(triton_key_path=key, cloud_validation=False, executor="terraform")
    _walk(tmp_path, "create-manager.yaml", "manager", MANAGER_STEPS, **base)
    state_path = tk_home / ".triton-kubernetes" / "test-manager" / "main.tf.json"
    # the example's fixed key id is of its author's key, not of the one given here
    _walk(tmp_path, "cluster-triton-ha.yaml", "cluster", CLUSTER_STEPS, triton_key_id=None, **base)
    mods = json.load(open(state_path))["module"]
    nodes = sorted(k for k in mods if k.startswith("node_triton_triton-ha_"))
    roles = sorted(next(iter(mods[k]["rancher_host_labels"])) for k in nodes)
    assert roles == ["control"] * 3 + ["etcd"] * 3 + ["worker"] * 4
    assert {mods[k]["hostname"].rstrip("0123456789-") for k in nodes} == {"triton-ha-e", "triton-ha-c", "triton-ha-w"}
