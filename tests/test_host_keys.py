"""Pinned SSH host keys (``parallel/hostkeys.py``): trust on first use, refuse a change.

The reference connects everywhere with host-key checking off.  Here the first contact
pins a host's key in the cluster manager's state backend (blob ``known_hosts``) and every
later SSH connection -- the DirectExecutor's plans and cleanup scripts, the bastion hop,
the Terraform modules' key and label reads -- is checked against it.  The fake ``ssh``
(``fixtures/fake_ssh.py``) checks keys the way OpenSSH does and runs the remote command
locally.
"""

import json
import os
import stat
import sys

import pytest

from triton_kubernetes_amd.backend import LocalBackend
from triton_kubernetes_amd.cli.main import dispatch
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.parallel import hostkeys
from triton_kubernetes_amd.rancher.fake import FakeRancher
from triton_kubernetes_amd.workflows import delete_node, new_cluster, new_manager

from helpers import HERE, make_ctx

PW = "tk-admin-pw-0123"


def _exe(path, body):
    path.write_text(body)
    path.chmod(path.stat().st_mode | stat.S_IEXEC)


@pytest.fixture
def hosts(tmp_path, monkeypatch):
    bindir = tmp_path / "bin"
    bindir.mkdir()
    _exe(bindir / "ssh", f"#!/bin/sh\nexec {sys.executable} {os.path.join(HERE, 'fixtures', 'fake_ssh.py')} \"$@\"\n")
    _exe(bindir / "scp", "#!/bin/sh\nexit 0\n")
    _exe(bindir / "sudo", "#!/bin/bash\ncase \"$1\" in tee) cat >/dev/null;; esac; exit 0\n")
    _exe(bindir / "docker", "#!/bin/sh\nexit 0\n")
    monkeypatch.setenv("PATH", f"{bindir}:{os.environ['PATH']}")
    d = tmp_path / "hosts"
    d.mkdir()
    for h in ("10.1.0.1", "10.1.0.2", "10.1.0.3", "jump.example"):
        (d / h).mkdir()
    monkeypatch.setenv("FAKE_SSH_HOSTS", str(d))
    monkeypatch.setenv("FAKE_SSH_EXEC", "1")
    monkeypatch.setenv("FAKE_SSH_LOG", str(tmp_path / "ssh.jsonl"))
    return d


def _pinned(backend):
    return (backend.read_blob("mgr", hostkeys.BLOB) or b"").decode()


def _cluster(tmp_path, fake):
    backend = LocalBackend(str(tmp_path / "state"))
    base = {"executor": "direct"}
    new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr", rancher_admin_password=PW,
                              rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="ubuntu", bastion_host="", key_path="k")), backend)
    nodes = [{"rancher_host_label": "etcd", "node_count": 1, "hostname": "e", "ssh_user": "core",
              "bastion_host": "", "key_path": "k", "hosts": ["10.1.0.1"]},
             {"rancher_host_label": "worker", "node_count": 1, "hostname": "w", "ssh_user": "core",
              "bastion_host": "jump.example", "key_path": "k", "hosts": ["10.1.0.2"]}]
    new_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="dev",
                              k8s_version="v1.28.10-rancher1-1", k8s_network_provider="flannel", nodes=nodes)),
                backend)
    return backend


def test_first_contact_pins_every_host_and_the_bastion(tmp_path, hosts):
    with FakeRancher.for_manager("mgr", PW) as fake:
        backend = _cluster(tmp_path, fake)
    pinned = _pinned(backend)
    for h in ("10.1.0.1", "10.1.0.2", "jump.example"):
        assert hostkeys.keys_for(pinned, h), (h, pinned)
    calls = [json.loads(ln) for ln in open(tmp_path / "ssh.jsonl")]
    assert calls and all(c["opts"].get("stricthostkeychecking") == "accept-new" for c in calls)
    assert not any(c["opts"].get("userknownhostsfile") == "/dev/null" for c in calls)


def test_changed_host_key_is_refused_with_a_clear_error(tmp_path, hosts):
    with FakeRancher.for_manager("mgr", PW) as fake:
        backend = _cluster(tmp_path, fake)
        before = _pinned(backend)
        # 10.1.0.1 now answers with another key (reinstalled -- or an impostor)
        (hosts / "10.1.0.1" / "host_key").write_text("ssh-ed25519 AAAAC3NzaC1lZDI1NTE5AAAAIMPOSTORKEYxxxxxxxxxxxxxxxxxxxxxxxxxxx")
        ctx = make_ctx({"executor": "direct", "cluster_manager": "mgr", "cluster_name": "dev", "hostname": "e-1",
                        "node_cleanup": True})
        with pytest.raises(TKError) as exc:
            delete_node(ctx, backend)
        msg = str(exc.value)
        assert "the SSH host key of 10.1.0.1 does not match the key pinned for cluster manager \"mgr\"" in msg
        assert "forget host-key" in msg
        assert _pinned(backend) == before  # nothing re-pinned
        assert "e-1" in backend.state("mgr").nodes("cluster_baremetal_dev")  # and nothing destroyed

        # the operator checked the new key out of band: forget the old one, and it is pinned anew
        out = make_ctx({"cluster_manager": "mgr", "host": "10.1.0.1"})
        dispatch(out, backend, "forget", "host-key")
        assert "Forgot 1 pinned SSH host key(s) of 10.1.0.1" in out.out.getvalue()
        delete_node(make_ctx({"executor": "direct", "cluster_manager": "mgr", "cluster_name": "dev",
                              "hostname": "e-1", "node_cleanup": True}), backend)
        assert hostkeys.keys_for(_pinned(backend), "10.1.0.1") == [
            "ssh-ed25519 AAAAC3NzaC1lZDI1NTE5AAAAIMPOSTORKEYxxxxxxxxxxxxxxxxxxxxxxxxxxx"]


def test_changed_bastion_key_is_refused(tmp_path, hosts):
    with FakeRancher.for_manager("mgr", PW) as fake:
        backend = _cluster(tmp_path, fake)
        (hosts / "jump.example" / "host_key").write_text("ssh-ed25519 AAAAC3NzaC1lZDI1NTE5AAAAIBASTIONxxxxxxxxxxxxxxxxxxxxxxxxxxxx")
        ctx = make_ctx({"executor": "direct", "cluster_manager": "mgr", "cluster_name": "dev", "hostname": "w-1",
                        "node_cleanup": True})
        with pytest.raises(TKError, match=r"10\.1\.0\.2 \(or its bastion jump\.example\) does not match"):
            delete_node(ctx, backend)


def test_store_merge_and_forget(tmp_path):
    from triton_kubernetes_amd.backend import MemoryBackend

    be = MemoryBackend()
    a = hostkeys.HostKeys(be, "m")
    b = hostkeys.HostKeys(be, "m")  # a second CLI on the same manager
    with open(a.path, "a") as fh:
        fh.write("h1 ssh-ed25519 AAAA1\n")
    with open(b.path, "a") as fh:
        fh.write("h2 ssh-ed25519 AAAA2\n")
    assert a.save() and b.save() and not b.save()
    text = be.read_blob("m", hostkeys.BLOB).decode()
    assert hostkeys.keys_for(text, "h1") == ["ssh-ed25519 AAAA1"] and hostkeys.keys_for(text, "h2")
    assert a.forget("h1") == 1 and hostkeys.keys_for(be.read_blob("m", hostkeys.BLOB).decode(), "h1") == []
    # OpenSSH writes "[host]:port" when an ssh_config Port is not 22: found and forgotten too
    with open(a.path, "a") as fh:
        fh.write("[h3]:2222 ssh-ed25519 AAAA3\n")
    assert a.save() and a.keys_for("h3") == ["ssh-ed25519 AAAA3"]
    assert a.forget("h3") == 1 and a.keys_for("h3") == []
    a.close()
    b.close()
    assert not os.path.exists(a.path)


def test_terraform_path_pins_the_manager_and_refuses_a_changed_key(tmp_path, hosts, monkeypatch):
    """The Terraform modules' SSH read (read_api_key.sh) connects with the manager's pinned
    keys, pins the manager on first contact and reports it (tk_ssh_known_hosts), which the
    executor merges into the store; a changed key then fails the next apply, and pinned
    hosts get host_key in their provisioner connections."""
    from helpers import install_fake_terraform, tf_calls

    log = install_fake_terraform(tmp_path, monkeypatch)
    monkeypatch.setenv("FAKE_TF_EXTERNAL", "1")
    monkeypatch.delenv("FAKE_SSH_EXEC")
    (hosts / "10.1.0.1" / "rancher_api_key").write_text(json.dumps({"name": "token-a", "token": "token-a:s"}))
    backend = LocalBackend(str(tmp_path / "state"))
    mgr = {"manager_cloud_provider": "baremetal", "name": "mgr", "rancher_admin_password": PW, "host": "10.1.0.1",
           "ssh_user": "ubuntu", "bastion_host": "", "key_path": "~/.ssh/id_rsa", "executor": "terraform"}
    new_manager(make_ctx(mgr), backend)
    apply = [c for c in tf_calls(log) if c["argv"][0] == "apply"][0]
    assert apply["doc"]["variable"]["tk_known_hosts"] == {"type": "string", "default": ""}  # nothing pinned yet
    pinned = _pinned(backend)
    assert hostkeys.keys_for(pinned, "10.1.0.1"), pinned

    # the next run renders the pinned key into the modules
    ctx = make_ctx({"cluster_manager": "mgr", "executor": "terraform"})
    open(log, "w").close()
    from triton_kubernetes_amd.workflows import get_manager

    get_manager(ctx, backend)
    assert "rancher_access_key = token-a" in ctx.out.getvalue() and "tk_ssh_known_hosts" not in ctx.out.getvalue()
    doc = [c for c in tf_calls(log) if c["argv"][0] == "init"][0]["doc"]
    assert doc["module"]["cluster-manager"]["host_key"] == hostkeys.keys_for(pinned, "10.1.0.1")[0]
    assert "10.1.0.1 ssh-ed25519" in doc["variable"]["tk_known_hosts"]["default"]

    # the manager now answers with another key: the key read refuses, the apply fails
    (hosts / "10.1.0.1" / "host_key").write_text("ssh-ed25519 AAAAC3NzaC1lZDI1NTE5AAAAIOTHERKEYxxxxxxxxxxxxxxxxxxxxxxxxxxxxx")
    cluster = {"cluster_manager": "mgr", "cluster_cloud_provider": "baremetal", "name": "dev",
               "k8s_version": "v1.28.10-rancher1-1", "k8s_network_provider": "flannel", "executor": "terraform"}
    with pytest.raises(TKError):
        new_cluster(make_ctx(cluster), backend)
    assert _pinned(backend) == pinned


def test_host_with_several_key_types_pins_the_one_terraform_negotiates(tmp_path, hosts):
    """a host with ed25519, ecdsa and rsa keys.  Go's x/crypto/ssh (Terraform's
    provisioner client) prefers ECDSA, then RSA, then Ed25519; OpenSSH by default presents
    Ed25519.  Every ssh of this framework offers Go's order, so the first contact pins the
    ECDSA key, UpdateHostKeys pins the other two, and the Terraform render shows each
    module the ECDSA key -- the one its connection will be presented."""
    from triton_kubernetes_amd.executor.terraform import render

    keys = {"ssh-ed25519": "AAAAC3NzaC1lZDI1NTE5AAAAIEDxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxx",
            "ecdsa-sha2-nistp256": "AAAAE2VjZHNhLXNoYTItbmlzdHAyNTYAAAAIbmlzdHAyNTYAAABBBECDSAxxxxxxxxx",
            "ssh-rsa": "AAAAB3NzaC1yc2EAAAADAQABAAABAQDRSAxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxx"}
    for h in ("10.1.0.1", "10.1.0.2", "jump.example"):
        (hosts / h / "host_keys").write_text("".join(f"{t} {b}\n" for t, b in keys.items()))
    with FakeRancher.for_manager("mgr", PW) as fake:
        backend = _cluster(tmp_path, fake)
    pinned = _pinned(backend)
    first = [ln.split()[1] for ln in pinned.splitlines() if ln.startswith("10.1.0.1 ")]
    assert first[0] == "ecdsa-sha2-nistp256" and sorted(first) == sorted(keys)  # negotiated first, then the rest
    calls = [json.loads(ln) for ln in open(tmp_path / "ssh.jsonl")]
    assert all(c["opts"]["hostkeyalgorithms"].split(",")[0] == "ecdsa-sha2-nistp256" and
               c["opts"]["hostkeyalgorithms"].split(",")[-1] == "ssh-ed25519" for c in calls)
    st = backend.state("mgr")
    doc = json.loads(render(st, (1, 5, 7), known_hosts=pinned).body)
    node = doc["module"]["node_baremetal_dev_e-1"]
    assert node["host_key"] == f"ecdsa-sha2-nistp256 {keys['ecdsa-sha2-nistp256']}"
    assert hostkeys.preferred_key([f"ssh-ed25519 x", "ssh-rsa y"]) == "ssh-rsa y"
    assert hostkeys.preferred_key(["ssh-ed25519 x"]) == "ssh-ed25519 x"
