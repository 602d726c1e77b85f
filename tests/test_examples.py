"""The shipped silent-install examples drive the CLI end to end (fake terraform on PATH)."""

import json
import os


from triton_kubernetes_amd.cli.main import run

from helpers import install_fake_terraform, make_ssh_key, tf_calls

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples", "silent-install")


def _cli(*argv):
    import io

    out = io.StringIO()
    return run(list(argv), out=out), out.getvalue()


def _with_overrides(tmp_path, name, **extra):
    import yaml

    doc = yaml.safe_load(open(os.path.join(EX, name)))
    doc.update(extra)
    path = tmp_path / name
    path.write_text(yaml.safe_dump(doc))
    return str(path)


def test_examples_parse():
    import yaml

    names = sorted(os.listdir(EX))
    assert "cluster-baremetal-mi355x.yaml" in names and "cluster-triton-ha.yaml" in names
    for n in names:
        assert isinstance(yaml.safe_load(open(os.path.join(EX, n))), dict), n


def test_baremetal_mi355x_examples_via_cli(tk_home, tmp_path, monkeypatch):
    log = install_fake_terraform(tmp_path, monkeypatch)
    key = make_ssh_key(tmp_path / "id_rsa")
    mgr = _with_overrides(tmp_path, "baremetal-manager.yaml", key_path=key, executor="terraform")
    code, out = _cli("--non-interactive", "--config", mgr, "create", "manager")
    assert code == 0, out
    cl = _with_overrides(tmp_path, "cluster-baremetal-mi355x.yaml", executor="terraform", wait=False)
    code, out = _cli("--non-interactive", "--config", cl, "create", "cluster")
    assert code == 0, out
    assert "4 nodes added: mi355x-gpu-1, mi355x-gpu-2, mi355x-gpu-3, mi355x-gpu-4" in out
    doc = tf_calls(log)[-1]["doc"]
    mods = doc["module"]
    assert "addons_baremetal_mi355x" in mods
    gpu = mods["node_baremetal_mi355x_mi355x-gpu-1"]
    assert gpu["source"].endswith("terraform/modules/bare-metal-mi355x-rancher-k8s-host")
    assert gpu["rccl_env"]["NCCL_SOCKET_IFNAME"] == "ens50f0" and gpu["gpu_count"] == "8"
    assert sum(1 for k in mods if k.startswith("node_")) == 8
    state = json.load(open(tk_home / ".triton-kubernetes" / "mi355x-manager" / "main.tf.json"))
    assert sorted(state["module"]) == sorted(mods)


def test_triton_examples_offline(tk_home, tmp_path, monkeypatch):
    install_fake_terraform(tmp_path, monkeypatch)
    key = make_ssh_key(tmp_path / "id_rsa")
    mgr = _with_overrides(tmp_path, "create-manager.yaml", triton_key_path=key, cloud_validation=False,
                          executor="terraform")
    code, out = _cli("--non-interactive", "--config", mgr, "create", "manager")
    assert code == 0, out
    cl = _with_overrides(tmp_path, "cluster-triton-ha.yaml", triton_key_path=key, cloud_validation=False,
                         executor="terraform")
    code, out = _cli("--non-interactive", "--config", cl, "create", "cluster")
    assert code == 0, out
    state = json.load(open(tk_home / ".triton-kubernetes" / "test-manager" / "main.tf.json"))
    nodes = [k for k in state["module"] if k.startswith("node_triton_triton-ha_")]
    assert len(nodes) == 10
    roles = [next(iter(state["module"][k]["rancher_host_labels"])) for k in nodes]
    assert sorted(roles) == ["control"] * 3 + ["etcd"] * 3 + ["worker"] * 4


def test_adopt_manager_example_via_cli(tk_home, tmp_path):
    """The adopted-server example against the fake Rancher: the given bootstrap password is
    used (and kept in the state backend, not in main.tf.json); nothing derived from the
    admin password reaches the server."""
    import yaml

    from triton_kubernetes_amd import versions
    from triton_kubernetes_amd.rancher.fake import FakeRancher

    doc = yaml.safe_load(open(os.path.join(EX, "adopt-manager.yaml")))
    with FakeRancher(bootstrap_password=doc["rancher_bootstrap_password"]) as fake:
        path = _with_overrides(tmp_path, "adopt-manager.yaml", host="rancher+" + fake.url)
        code, out = _cli("--non-interactive", "--config", path, "create", "manager")
        assert code == 0, out
        assert fake.state.admin_password == doc["rancher_admin_password"]
        derived = versions.bootstrap_password(doc["name"], doc["rancher_admin_password"]).encode()
        assert not any(derived in b for b in fake.request_bodies)
    state_dir = tk_home / ".triton-kubernetes" / doc["name"]
    assert doc["rancher_bootstrap_password"] not in (state_dir / "main.tf.json").read_text()
