"""SSH delivery path with a fake ``ssh``/``scp`` on PATH (fake SSH runner).

The fake records its argv per call and runs the remote command locally under
stub ``sudo``/``docker``, so the rendered bootstrap script really executes.
"""

import json
import os
import stat

import pytest

from triton_kubernetes_amd.backend import LocalBackend
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.parallel.transport import HostRef, SSHTransport
from triton_kubernetes_amd.rancher.fake import FakeRancher
from triton_kubernetes_amd.workflows import new_cluster, new_manager

from helpers import make_ctx


def _exe(path, body):
    path.write_text("#!/bin/bash\n" + body + "\n")
    path.chmod(path.stat().st_mode | stat.S_IEXEC)


@pytest.fixture
def fake_ssh(tmp_path, monkeypatch):
    bindir = tmp_path / "bin"
    bindir.mkdir()
    log = tmp_path / "ssh.jsonl"
    sudo_log = tmp_path / "sudo.log"
    # argv logged as JSON; hosts named fail-* exit 255 like an unreachable host
    _exe(bindir / "ssh", f'''
python3 - "$@" <<'PY' >> {log}
import json, sys
print(json.dumps(sys.argv[1:]))
PY
target="${{@: -2:1}}"
case "$target" in *@fail-*) echo "ssh: connect to host: Connection refused" >&2; exit 255;; esac
remote="${{@: -1}}"
exec bash -c "$remote"''')
    _exe(bindir / "scp", f'echo "scp $*" >> {log}')
    _exe(bindir / "sudo", f'echo "$*" >> {sudo_log}; case "$1" in tee) cat >/dev/null;; esac; exit 0')
    _exe(bindir / "docker", "exit 0")
    monkeypatch.setenv("PATH", f"{bindir}:{os.environ['PATH']}")
    return log, sudo_log


def _calls(log):
    return [json.loads(ln) for ln in open(log) if ln.startswith("[")]


def test_ssh_argv_options(tmp_path):
    t = SSHTransport(control_dir=str(tmp_path))
    argv = t.ssh_argv(HostRef("10.0.0.5", "core", "~/.ssh/k", "bastion.example", "jump"), "bash -s")
    assert argv[0] == "ssh" and argv[-2:] == ["core@10.0.0.5", "bash -s"]
    joined = " ".join(argv)
    assert "BatchMode=yes" in joined and "ControlMaster=auto" in joined and f"ControlPath={tmp_path}/%C" in joined
    assert os.path.expanduser("~/.ssh/k") in argv
    # the bastion hop is a ProxyCommand with the same host-key options (-J would drop them)
    proxy = next(a for a in argv if a.startswith("ProxyCommand="))
    assert "-W %h:%p jump@bastion.example" in proxy and "StrictHostKeyChecking=accept-new" in proxy
    # never the reference's StrictHostKeyChecking=no: trust on first use, a changed key refused
    assert "StrictHostKeyChecking=no" not in joined and "UserKnownHostsFile=/dev/null" not in joined
    assert "StrictHostKeyChecking=accept-new" in joined and f"UserKnownHostsFile={tmp_path}/known_hosts" in joined
    strict = SSHTransport(strict_host_keys=True, control_dir=str(tmp_path)).ssh_argv(HostRef("h"), "x")
    assert "StrictHostKeyChecking=yes" in " ".join(strict)


def test_cluster_over_ssh_runs_rendered_plans(tmp_path, fake_ssh):
    log, sudo_log = fake_ssh
    fake = FakeRancher.for_manager("mgr", "tk-admin-pw-0123").start()
    try:
        backend = LocalBackend(str(tmp_path / "state"))
        base = {"executor": "direct"}
        new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr", rancher_admin_password="tk-admin-pw-0123",
                                  rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="ubuntu", bastion_host="", key_path="k")),
                    backend)
        nodes = [{"rancher_host_label": "etcd", "node_count": 1, "hostname": "e", "ssh_user": "core",
                  "bastion_host": "", "key_path": "~/.ssh/id", "hosts": ["10.1.0.1"]},
                 {"rancher_host_label": "worker", "node_count": 2, "hostname": "w", "ssh_user": "core",
                  "bastion_host": "jump.example", "key_path": "~/.ssh/id", "hosts": ["10.1.0.2", "10.1.0.3"]}]
        new_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="ssh",
                                  k8s_version="v1.28.10-rancher1-1", k8s_network_provider="flannel", nodes=nodes)),
                    backend)
        calls = _calls(log)
        targets = sorted(c[-2] for c in calls)
        assert targets == ["core@10.1.0.1", "core@10.1.0.2", "core@10.1.0.3"]
        jumped = [c for c in calls if any(a.startswith("ProxyCommand=") for a in c)]
        assert sorted(c[-2] for c in jumped) == ["core@10.1.0.2", "core@10.1.0.3"]
        assert all(any(a.startswith("ProxyCommand=") and a.endswith("core@jump.example") for a in c) for c in jumped)
        sudo = open(sudo_log).read()
        assert "hostnamectl set-hostname e-1" in sudo and "hostnamectl set-hostname w-2" in sudo
        runs = [ln for ln in sudo.splitlines() if ln.startswith("docker run")]
        assert len(runs) == 3
        assert sum("--etcd" in r for r in runs) == 1 and sum("--worker" in r for r in runs) == 2
        assert all(f"--server {fake.url}" in r for r in runs)
        # tfstate checkpoint carries each host's step timings
        tf = json.loads(backend.read_tfstate("mgr"))
        assert all(tf["module_state"][k]["status"] == "ok" for k in tf["module_state"])
    finally:
        fake.stop()


def test_unreachable_host_fails_only_its_module(tmp_path, fake_ssh):
    fake = FakeRancher.for_manager("mgr", "tk-admin-pw-0123").start()
    try:
        backend = LocalBackend(str(tmp_path / "state"))
        base = {"executor": "direct"}
        new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr", rancher_admin_password="tk-admin-pw-0123",
                                  rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="ubuntu", bastion_host="", key_path="k")),
                    backend)
        nodes = [{"rancher_host_label": "worker", "node_count": 2, "hostname": "w", "ssh_user": "core",
                  "bastion_host": "", "key_path": "k", "hosts": ["10.2.0.1", "fail-10.2.0.2"]}]
        with pytest.raises(TKError) as exc:
            new_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name="x",
                                      k8s_version="v1.28.10-rancher1-1", k8s_network_provider="flannel",
                                      nodes=nodes)), backend)
        assert "w-2" in str(exc.value) and "re-run to resume" in str(exc.value)
        tf = json.loads(backend.read_tfstate("mgr"))
        st = {k: v["status"] for k, v in tf["module_state"].items()}
        assert st["node_baremetal_x_w-1"] == "ok" and st["node_baremetal_x_w-2"] == "failed"
    finally:
        fake.stop()
