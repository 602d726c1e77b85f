"""Destroy, then re-create on the same bare-metal host (VERDICT r4 "Next round" #1).

Bare-metal MI355X hosts are never re-imaged, so ``create cluster A`` -> ``destroy cluster
A`` -> ``create cluster B`` on the same hosts is the normal path.  The reference never
uninstalled anything (Q7); round 4 cleaned only RKE1 containers, over SSH only, opt-in.

The fakes model what a real host does (``rancher/fake/hostsim.py``): a join leaves
rancher-system-agent and RKE2 behind, and a second cluster's join on a host that still
holds them is refused (the real join fails later: a node that never turns Ready).  Every
delivery path is run end to end against that model:

* DirectExecutor, node-agent hosts (sim agents: the host is the agent's root);
* DirectExecutor, SSH hosts (``fixtures/fake_ssh.py`` runs the scripts against
  ``<host>/root`` with a ``sudo`` that acts only inside it);
* TerraformExecutor (``fixtures/fake_terraform.py`` runs the modules' destroy-time
  provisioner against the same host roots).

Each path also runs with ``node_cleanup: false`` -- round 4's behaviour for agent hosts,
RKE2 and Terraform -- and that second create fails, with the join record's reason.
"""

import json
import os
import stat
import subprocess
import sys
import tempfile

import pytest

from triton_kubernetes_amd import versions
from triton_kubernetes_amd import workflows as wf
from triton_kubernetes_amd.backend import LocalBackend
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.node import cleanup
from triton_kubernetes_amd.node.agent import NodeAgent
from triton_kubernetes_amd.node.labels import synthetic_topology
from triton_kubernetes_amd.rancher.fake import FakeRancher, hostsim
from triton_kubernetes_amd.rancher.fake.provisioning import SYSTEM_AGENT_INSTALL_SCRIPT

from helpers import HERE, install_fake_terraform, make_ctx, output

PW = "tk-admin-pw-0123"
TOKEN = "teardown-token-0123456"


def _exe(path, body):
    path.write_text(body)
    path.chmod(path.stat().st_mode | stat.S_IEXEC)


def _stub_bin(tmp_path):
    """``sudo`` that runs what touches the host root (and the installer, and docker) and
    only records the rest -- nothing here may change the machine the tests run on; a
    ``docker`` with Docker's filter semantics over the host root's container table
    (``fixtures/fake_docker.py``)."""
    bindir = tmp_path / "bin"
    bindir.mkdir(exist_ok=True)
    log = tmp_path / "sudo.log"
    _exe(bindir / "sudo", f'''#!/bin/bash
echo "$*" >> {log}
[ -n "${{TK_HOST_ROOT:-}}" ] || {{ case "$1" in tee) cat >/dev/null;; esac; exit 0; }}
case "$1" in sh|docker) exec "$@";; esac
for a in "$@"; do case "$a" in "$TK_HOST_ROOT"/*) exec "$@";; esac; done
case "$1" in tee) cat >/dev/null;; esac
exit 0
''')
    _exe(bindir / "docker", f"#!/bin/sh\nexec {sys.executable} {os.path.join(HERE, 'fixtures', 'fake_docker.py')} \"$@\"\n")
    _exe(bindir / "hostnamectl", "#!/bin/sh\nexit 0\n")
    return bindir, log


# --- the pieces ---------------------------------------------------------------------------------


def test_cleanup_script_uninstalls_rke2_and_the_agent(tmp_path, monkeypatch):
    bindir, _ = _stub_bin(tmp_path)
    root = tmp_path / "host"
    hostsim.install(str(root), "https://r.example", "tok-a")
    cleanup.write_join_record(lambda p: str(root) + p, cleanup.join_record("https://r.example", "tok-a", "rke2", "n"))
    (root / "opt/triton-kubernetes/bin").mkdir(parents=True)
    (root / "opt/triton-kubernetes/bin/gpu-burnin").write_text("tool")
    env = dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}", TK_HOST_ROOT=str(root))
    proc = subprocess.run(["bash", "-s"], input=cleanup.cleanup_script(), env=env, capture_output=True, text=True)
    assert proc.returncode == 0, proc.stderr
    rep = cleanup.parse_cleanup_markers(proc.stdout)
    assert rep["ok"] and rep["complete"]
    ran = [a["what"] for a in rep["actions"] if a["status"] == "ok"]
    assert ran == ["/usr/local/bin/rancher-system-agent-uninstall.sh", "/usr/local/bin/rke2-killall.sh",
                   "/usr/local/bin/rke2-uninstall.sh"]
    for gone in ("var/lib/rancher", "etc/rancher", "usr/local/bin/rke2", cleanup.JOIN_RECORD.lstrip("/")):
        assert not (root / gone).exists(), gone
    assert (root / "opt/triton-kubernetes/bin/gpu-burnin").exists()  # the node tools stay
    assert hostsim.conflict(str(root), "https://other.example", "tok-b") is None


def test_cleanup_script_reports_a_failing_uninstaller(tmp_path):
    bindir, _ = _stub_bin(tmp_path)
    root = tmp_path / "host"
    hostsim.install(str(root), "https://r.example", "tok-a")
    _exe(root / "usr/local/bin/rke2-uninstall.sh", "#!/bin/sh\necho boom >&2; exit 3\n")
    env = dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}", TK_HOST_ROOT=str(root))
    proc = subprocess.run(["bash", "-s"], input=cleanup.cleanup_script(), env=env, capture_output=True, text=True)
    assert proc.returncode == 1
    rep = cleanup.parse_cleanup_markers(proc.stdout)
    assert not rep["ok"] and {"what": "/usr/local/bin/rke2-uninstall.sh", "status": "failed"} in rep["actions"]


def test_join_guard_refuses_another_cluster_only(tmp_path):
    root = tmp_path / "host"
    cleanup.write_join_record(lambda p: str(root) + p, cleanup.join_record("https://r", "tok-a", "rke2", "gpu-1"))

    def run(token):
        script = "set -e\n" + cleanup.join_guard_shell("https://r", token) + "echo joined\n"
        return subprocess.run(["bash", "-c", script], env=dict(os.environ, TK_HOST_ROOT=str(root)),
                              capture_output=True, text=True)

    same, other = run("tok-a"), run("tok-b")
    assert same.returncode == 0 and "joined" in same.stdout
    assert other.returncode == 1 and "still a node of another cluster" in other.stderr and "gpu-1" in other.stderr
    assert cleanup.refusal(cleanup.read_join_record(lambda p: str(root) + p), "https://r", "tok-b")
    assert cleanup.refusal(None, "https://r", "tok-b") is None  # no record: never refused


FAKE_DOCKER = os.path.join(HERE, "fixtures", "fake_docker.py")
AGENT_TAGGED = f"rancher/rancher-agent:{versions.RANCHER_VERSION}"
AGENT_REGISTRY = f"registry.example:5000/rancher/rancher-agent:{versions.RANCHER_VERSION}"


def _docker(root, *argv, check=True):
    proc = subprocess.run([sys.executable, FAKE_DOCKER, *argv], env=dict(os.environ, TK_HOST_ROOT=str(root)),
                          capture_output=True, text=True)
    if check:
        assert proc.returncode == 0, proc.stderr
    return proc


def _names(root):
    return sorted(ln.split()[-1] for ln in _docker(root, "ps", "-a", "--format", "{{.ID}} {{.Names}}")
                  .stdout.splitlines())


def _rke1_host(root, agent_image=AGENT_TAGGED, server="https://r", token="tok-a"):
    """An RKE1 node as Docker shows it after a join: the agent (a tagged image), RKE's
    kubelet / kube-proxy, the kubelet's pod containers and sandboxes -- plus a container
    of the machine's owner that no teardown may touch, and an RKE helper without a label."""
    _docker(root, "run", "-d", "--privileged", "--restart=unless-stopped", "--net=host", "-v",
            "/etc/kubernetes:/etc/kubernetes", agent_image, "--server", server, "--token", token, "--worker")
    _docker(root, "run", "-d", "--name", "rke-etcd-port-listener", "rancher/rke-tools:v0.1.96")
    _docker(root, "run", "-d", "--name", "owners-nginx", "nginx:1.25")
    hostsim.install(str(root), server, token, distribution="rke1")


def test_fake_docker_has_dockers_filter_semantics(tmp_path):
    """Contract: the double answers as Docker does.  An untagged ``ancestor=`` means
    ``:latest`` -- so round 5's ``ancestor=rancher/rancher-agent`` matched no agent running
    a tagged image, which is why the agent survived the teardown."""
    root = tmp_path / "host"
    _rke1_host(root)
    ids = lambda *f: _docker(root, "ps", "-aq", *[x for flt in f for x in ("--filter", flt)]).stdout.split()  # noqa
    assert ids("ancestor=rancher/rancher-agent") == []  # the round-5 filter: nothing
    # the agent and the cattle-node-agent pod (the same image); docker.io/ is implied
    assert len(ids(f"ancestor={AGENT_TAGGED}")) == len(ids(f"ancestor=docker.io/{AGENT_TAGGED}")) == 2
    assert len(ids("label=io.rancher.rke.container.name")) == 2  # kubelet, kube-proxy
    assert len(ids("label=io.kubernetes.pod.namespace")) == 4  # 2 pods x (container + sandbox)
    assert len(ids("label=io.kubernetes.pod.namespace=kube-system", "name=flannel")) == 2  # AND of kinds
    assert len(ids("name=kube-proxy", "name=kubelet")) == 2  # OR within a kind
    # RKE's fixed container names: a second join while the first cluster's containers remain
    again = _docker(root, "run", "-d", AGENT_TAGGED, "--server", "https://r", "--token", "tok-a", check=False)
    assert again.returncode == 125 and "Conflict" in again.stderr
    other = _docker(root, "run", "-d", AGENT_TAGGED, "--server", "https://r2", "--token", "tok-b", check=False)
    assert other.returncode == 1 and "still running" in other.stderr
    assert _docker(root, "rm", "-f", "nope", check=False).returncode == 1


@pytest.mark.parametrize("agent_image", [AGENT_TAGGED, AGENT_REGISTRY, "docker.io/" + AGENT_TAGGED,
                                         f"rancher/rancher-agent@sha256:{'a' * 64}"])
def test_cleanup_script_removes_the_rke1_agent_and_every_pod_container(tmp_path, agent_image):
    """the agent (any registry, tag or digest), RKE's containers, its
    unlabelled helpers and every kubelet-launched ``k8s_*`` container go; the owner's stays."""
    bindir, _ = _stub_bin(tmp_path)
    root = tmp_path / "host"
    _rke1_host(root, agent_image)
    assert len(_names(root)) == 9
    env = dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}", TK_HOST_ROOT=str(root))
    proc = subprocess.run(["bash", "-s"], input=cleanup.cleanup_script(), env=env, capture_output=True, text=True)
    assert proc.returncode == 0, proc.stderr
    rep = cleanup.parse_cleanup_markers(proc.stdout)
    assert rep["ok"] and {"what": "rke1-containers", "status": "ok"} in rep["actions"]
    assert _names(root) == ["owners-nginx"]
    assert not (root / "etc/kubernetes").exists() and not (root / "var/lib/etcd").exists()


def test_cleanup_script_removes_a_custom_agent_image_named_by_the_join_record(tmp_path):
    """An agent image of another repository altogether (``rancher_agent_image``): the join
    record (SSH, agents) or Terraform's ``TK_AGENT_IMAGE`` names it."""
    bindir, _ = _stub_bin(tmp_path)
    for how in ("record", "env"):
        root = tmp_path / how
        _docker(root, "run", "-d", "mirror.example/acme/agent:v9", "--server", "https://r", "--token", "t")
        _docker(root, "run", "-d", "--name", "owners-nginx", "nginx:1.25")
        env = dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}", TK_HOST_ROOT=str(root))
        if how == "record":
            cleanup.write_join_record(lambda p, r=root: str(r) + p, cleanup.join_record(
                "https://r", "t", "rke1", "n", agent_image="mirror.example/acme/agent:v9"))
        else:
            env["TK_AGENT_IMAGE"] = "mirror.example/acme/agent:v9"
        proc = subprocess.run(["bash", "-s"], input=cleanup.cleanup_script(), env=env, capture_output=True,
                              text=True)
        assert proc.returncode == 0, proc.stderr
        assert _names(root) == ["owners-nginx"], how


def test_cleanup_script_skips_everything_when_terraform_says_node_cleanup_false(tmp_path):
    bindir, _ = _stub_bin(tmp_path)
    root = tmp_path / "host"
    _rke1_host(root)
    hostsim.install(str(root), "https://r", "tok-a")
    env = dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}", TK_HOST_ROOT=str(root), TK_NODE_CLEANUP="false")
    proc = subprocess.run(["bash", "-s"], input=cleanup.cleanup_script(), env=env, capture_output=True, text=True)
    assert proc.returncode == 0 and "::tk-cleanup node_cleanup skipped" in proc.stdout
    assert len(_names(root)) == 9 and (root / "usr/local/bin/rke2-uninstall.sh").exists()


def test_agent_exec_cleanup_runs_fixed_argv(tmp_path):
    """Exec mode: the uninstallers found at their fixed paths, the RKE1 containers from
    ``docker ps`` as Docker answers it, the directories -- no shell text involved."""
    root = tmp_path / "host"
    hostsim.install(str(root), "https://r", "tok")
    _rke1_host(root, AGENT_REGISTRY)
    calls = []

    def run_argv(argv, stdin=None, timeout=0):
        calls.append(argv)
        env = dict(os.environ, TK_HOST_ROOT=str(root))
        if argv[0].endswith(".sh"):
            subprocess.run(argv, env=env, check=True)
            return ""
        assert argv[0] == "/usr/bin/docker"
        proc = subprocess.run([sys.executable, FAKE_DOCKER, *argv[1:]], env=env, capture_output=True, text=True)
        if proc.returncode:
            raise RuntimeError(proc.stderr)
        return proc.stdout

    rep = cleanup.cleanup_host(lambda p: str(root) + p, run_argv, docker="/usr/bin/docker")
    assert rep["ok"], rep
    assert [c[0] for c in calls[:3]] == [str(root) + "/usr/local/bin/rancher-system-agent-uninstall.sh",
                                         str(root) + "/usr/local/bin/rke2-killall.sh",
                                         str(root) + "/usr/local/bin/rke2-uninstall.sh"]
    assert {"what": "rke1-containers", "status": "ok", "count": "8"} in rep["actions"]
    assert _names(root) == ["owners-nginx"]
    assert not (root / "var/lib/rancher").exists()


def test_sim_agent_with_root_slash_models_no_host():
    a = NodeAgent(name="x", mode="sim", token="t" * 20)
    assert a.root == "/" and not a._host_is_sandbox()
    assert a.cleanup() == {"ok": True, "simulated": True, "actions": [], "ms": 0.0}


# --- the fake refuses what the real host fails on (contract) -------------------------------------


def test_fake_installer_refuses_a_host_of_another_cluster(tmp_path):
    root = tmp_path / "host"
    script = tmp_path / "install.sh"
    script.write_text(SYSTEM_AGENT_INSTALL_SCRIPT)
    with FakeRancher.for_manager("mgr", PW) as fake:
        _, tok_a, _ = fake.registration("a", "rke2")
        _, tok_b, _ = fake.registration("b", "rke2")
        env = dict(os.environ, TK_HOST_ROOT=str(root))
        first = subprocess.run(["sh", str(script), "--server", fake.url, "--token", tok_a, "--node-name", "n1",
                                "--worker"], env=env, capture_output=True, text=True)
        assert first.returncode == 0, first.stderr
        assert (root / "usr/local/bin/rke2-uninstall.sh").exists()
        again = subprocess.run(["sh", str(script), "--server", fake.url, "--token", tok_a, "--node-name", "n1",
                                "--worker"], env=env, capture_output=True, text=True)
        assert again.returncode == 0, again.stderr  # re-registration with the same cluster
        second = subprocess.run(["sh", str(script), "--server", fake.url, "--token", tok_b, "--node-name", "n1",
                                 "--worker"], env=env, capture_output=True, text=True)
        assert second.returncode == 1 and "already installed" in second.stderr
        # agent uninstalled but RKE2 left: still refused
        subprocess.run([str(root / "usr/local/bin/rancher-system-agent-uninstall.sh")], env=env, check=True)
        third = subprocess.run(["sh", str(script), "--server", fake.url, "--token", tok_b, "--node-name", "n1",
                                "--worker"], env=env, capture_output=True, text=True)
        assert third.returncode == 1 and "rke2-uninstall.sh" in third.stderr
        subprocess.run([str(root / "usr/local/bin/rke2-uninstall.sh")], env=env, check=True)
        fourth = subprocess.run(["sh", str(script), "--server", fake.url, "--token", tok_b, "--node-name", "n1",
                                 "--worker"], env=env, capture_output=True, text=True)
        assert fourth.returncode == 0, fourth.stderr


# --- A -> destroy -> B, every delivery path ---------------------------------------------------------


def _mgr(fake, backend, base):
    wf.new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr", rancher_admin_password=PW,
                                 rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="ubuntu", bastion_host="", key_path="k")),
                   backend)


def _cluster_cfg(base, name, cp, workers, gpu=True):
    return dict(base, cluster_manager="mgr", cluster_cloud_provider="baremetal", name=name,
                k8s_version=versions.DEFAULT_K8S_VERSION, k8s_network_provider="canal", nodes=[
                    {"rancher_host_label": "control", "node_count": 1, "hostname": f"{name}-cp", "ssh_user": "u",
                     "bastion_host": "", "key_path": "k", "hosts": [cp]},
                    {"rancher_host_label": "worker", "node_count": len(workers), "hostname": f"{name}-gpu",
                     "ssh_user": "u", "bastion_host": "", "key_path": "k", "hosts": workers,
                     **({"gpu": "mi355x", "gpu_count": 8, "gpu_burnin": "quick"} if gpu else {})}])


@pytest.fixture
def agents(tmp_path):
    fake = FakeRancher.for_manager("mgr", PW).start()
    made = []

    def agent(name, gpus=0):
        a = NodeAgent(name=name, mode="sim", devices=list(range(gpus)), token=TOKEN, root=tempfile.mkdtemp(),
                      topology_override=synthetic_topology(gpus) if gpus else None,
                      burnin_override=lambda d, l: {"ok": True})
        made.append(a)
        return "agent+" + a.serve(), a

    yield fake, agent, LocalBackend(str(tmp_path / "state"))
    for a in made:
        a.stop()
    fake.stop()


@pytest.mark.parametrize("node_cleanup", [True, False])
def test_agent_hosts_destroy_then_recreate(agents, node_cleanup):
    fake, agent, backend = agents
    base = {"executor": "direct", "agent_token": TOKEN}
    _mgr(fake, backend, base)
    (cp, cp_agent), (gpu, gpu_agent) = agent("cp"), agent("g", gpus=8)
    wf.new_cluster(make_ctx(_cluster_cfg(base, "a", cp, [gpu])), backend)
    assert os.path.exists(gpu_agent.path(hostsim.CONNECTION_INFO))
    assert os.path.exists(gpu_agent.path(cleanup.JOIN_RECORD))
    d = make_ctx(dict(base, cluster_manager="mgr", cluster_name="a", node_cleanup=node_cleanup))
    wf.delete_cluster(d, backend)
    ctx_b = make_ctx(_cluster_cfg(base, "b", cp, [gpu]))
    if node_cleanup:
        assert "Cleaned up host a-gpu-1 (rancher-system-agent-uninstall.sh, rke2-killall.sh, rke2-uninstall.sh)" \
            in output(d)
        assert not os.path.exists(gpu_agent.path(hostsim.CONNECTION_INFO))
        wf.new_cluster(ctx_b, backend)  # the same two hosts join cluster B
        cid_b = next(c["id"] for c in fake.state.clusters.values() if c["name"] == "b")
        assert {n["hostname"] for n in fake.state.cluster_nodes[cid_b].values()} == {"b-cp-1", "b-gpu-1"}
    else:
        assert "Cleaned up" not in output(d)
        with pytest.raises(TKError, match="still a node of another cluster"):
            wf.new_cluster(ctx_b, backend)


def test_agent_cleanup_failure_is_reported_not_fatal(agents):
    fake, agent, backend = agents
    base = {"executor": "direct", "agent_token": TOKEN}
    _mgr(fake, backend, base)
    (cp, _), (gpu, gpu_agent) = agent("cp"), agent("g", gpus=8)
    wf.new_cluster(make_ctx(_cluster_cfg(base, "a", cp, [gpu])), backend)
    gpu_agent.stop()  # the host died
    d = make_ctx(dict(base, cluster_manager="mgr", cluster_name="a"))
    wf.delete_cluster(d, backend)
    assert "WARNING: cleanup of host a-gpu-1 failed" in output(d) and "Cleaned up host a-cp-1" in output(d)
    assert backend.state("mgr").clusters() == {}  # the destroy went through


@pytest.fixture
def ssh_hosts(tmp_path, monkeypatch):
    bindir, sudo_log = _stub_bin(tmp_path)
    _exe(bindir / "ssh", f"#!/bin/sh\nexec {sys.executable} {os.path.join(HERE, 'fixtures', 'fake_ssh.py')} \"$@\"\n")
    _exe(bindir / "scp", "#!/bin/sh\nexit 0\n")
    monkeypatch.setenv("PATH", f"{bindir}:{os.environ['PATH']}")
    hosts = tmp_path / "hosts"
    for h in ("10.2.0.1", "10.2.0.2"):
        (hosts / h).mkdir(parents=True)
    monkeypatch.setenv("FAKE_SSH_HOSTS", str(hosts))
    monkeypatch.setenv("FAKE_SSH_EXEC", "1")
    monkeypatch.setenv("FAKE_SSH_HOST_ROOT", "1")
    return hosts, sudo_log


@pytest.mark.parametrize("node_cleanup", [True, False])
def test_ssh_hosts_destroy_then_recreate(tmp_path, ssh_hosts, node_cleanup):
    """RKE2 over SSH: the rendered plan really runs (the fake's installer models the host),
    the cleanup script really runs against the host's root."""
    hosts, _ = ssh_hosts
    with FakeRancher.for_manager("mgr", PW) as fake:
        backend = LocalBackend(str(tmp_path / "state"))
        base = {"executor": "direct"}
        _mgr(fake, backend, base)
        wf.new_cluster(make_ctx(_cluster_cfg(base, "a", "10.2.0.1", ["10.2.0.2"], gpu=False)), backend)
        root = hosts / "10.2.0.2" / "root"
        assert (root / hostsim.CONNECTION_INFO.lstrip("/")).exists()
        assert json.loads((root / cleanup.JOIN_RECORD.lstrip("/")).read_text())["hostname"] == "a-gpu-1"
        d = make_ctx(dict(base, cluster_manager="mgr", cluster_name="a", node_cleanup=node_cleanup))
        wf.delete_cluster(d, backend)
        ctx_b = make_ctx(_cluster_cfg(base, "b", "10.2.0.1", ["10.2.0.2"], gpu=False))
        if node_cleanup:
            assert "Cleaned up host a-gpu-1" in output(d)
            assert not (root / "var/lib/rancher").exists() and not (root / "usr/local/bin/rke2-uninstall.sh").exists()
            wf.new_cluster(ctx_b, backend)
            assert json.loads((root / cleanup.JOIN_RECORD.lstrip("/")).read_text())["hostname"] == "b-gpu-1"
        else:
            with pytest.raises(TKError, match="still a node of another cluster"):
                wf.new_cluster(ctx_b, backend)


@pytest.mark.parametrize("teardown", ["current", "round5"])
def test_ssh_rke1_hosts_destroy_then_recreate(tmp_path, ssh_hosts, monkeypatch, teardown):
    """RKE1 over SSH, A -> destroy -> B: the node's Docker is the fake with
    Docker's semantics (``fixtures/fake_docker.py``): the join runs the tagged agent, which
    brings up RKE's containers and the kubelet's pods.  The teardown must leave none of
    them, or B's agent finds A's still running.  ``round5``: the old selection (an untagged
    ``ancestor=`` filter and RKE's label only) -- A's agent and pods survive, and B fails."""
    hosts, _ = ssh_hosts
    if teardown == "round5":
        monkeypatch.setattr(cleanup, "RKE1_LABELS", ("io.rancher.rke.container.name",))
        monkeypatch.setattr(cleanup, "RKE1_REPOS", ())
        join_record = cleanup.join_record  # ... and no agent image in the join record
        monkeypatch.setattr(cleanup, "join_record", lambda *a, **k: dict(join_record(*a[:4])))
    with FakeRancher.for_manager("mgr", PW) as fake:
        backend = LocalBackend(str(tmp_path / "state"))
        base = {"executor": "direct", "k8s_distribution": "rke1"}
        _mgr(fake, backend, {"executor": "direct"})
        rke1 = lambda name: dict(_cluster_cfg(base, name, "10.2.0.1", ["10.2.0.2"], gpu=False),  # noqa: E731
                                 k8s_version=versions.DEFAULT_RKE1_VERSION)
        wf.new_cluster(make_ctx(rke1("a")), backend)
        root = hosts / "10.2.0.2" / "root"
        rec = json.loads((root / cleanup.JOIN_RECORD.lstrip("/")).read_text())
        assert rec["distribution"] == "rke1"
        assert rec.get("agent_image") == (versions.AGENT_IMAGE if teardown == "current" else None)
        table = json.loads((root / "var/lib/docker/fake-containers.json").read_text())
        assert any(c["image"] == versions.AGENT_IMAGE and c["name"].startswith("agent_") for c in table)
        assert sum(c["name"].startswith("k8s_") for c in table) == 4
        d = make_ctx(dict(base, cluster_manager="mgr", cluster_name="a"))
        wf.delete_cluster(d, backend)
        ctx_b = make_ctx(rke1("b"))
        if teardown == "current":
            assert "Cleaned up host a-gpu-1" in output(d)
            assert _names(root) == []
            wf.new_cluster(ctx_b, backend)
            assert json.loads((root / cleanup.JOIN_RECORD.lstrip("/")).read_text())["hostname"] == "b-gpu-1"
        else:
            left = _names(root)
            assert any(n.startswith("agent_") for n in left) and any(n.startswith("k8s_") for n in left)
            with pytest.raises(TKError, match="another rancher-agent"):
                wf.new_cluster(ctx_b, backend)


@pytest.mark.parametrize("node_cleanup", [True, False])
def test_terraform_destroy_then_recreate(tmp_path, monkeypatch, capfd, node_cleanup):
    """TerraformExecutor: the host modules' destroy-time provisioner (``when = destroy``)
    runs the same cleanup script; ``node_cleanup = false`` in the module drops it."""
    install_fake_terraform(tmp_path, monkeypatch)
    bindir, _ = _stub_bin(tmp_path)
    monkeypatch.setenv("PATH", f"{bindir}:{os.environ['PATH']}")
    hosts = tmp_path / "hosts"
    hosts.mkdir()
    monkeypatch.setenv("FAKE_TF_HOSTS", str(hosts))
    backend = LocalBackend(str(tmp_path / "state"))
    base = {"executor": "terraform"}
    wf.new_manager(make_ctx(dict(base, manager_cloud_provider="baremetal", name="mgr", rancher_admin_password=PW,
                                 host="10.0.0.10", ssh_user="ubuntu", bastion_host="", key_path="~/.ssh/id_rsa")),
                   backend)
    cfg_a = _cluster_cfg(base, "a", "10.3.0.1", ["10.3.0.2"])
    for n in cfg_a["nodes"]:
        n["node_cleanup"] = node_cleanup
    wf.new_cluster(make_ctx(cfg_a), backend)
    rec = hosts / "10.3.0.2" / "root" / "var/lib/rancher/agent/rancher2_connection_info.json"
    assert rec.exists()
    assert backend.state("mgr").module("node_baremetal_a_a-gpu-1")["node_cleanup"] is node_cleanup
    wf.delete_cluster(make_ctx(dict(base, cluster_manager="mgr", cluster_name="a")), backend)
    ctx_b = make_ctx(_cluster_cfg(base, "b", "10.3.0.1", ["10.3.0.2"]))
    if node_cleanup:
        assert not rec.exists()
        wf.new_cluster(ctx_b, backend)
        assert "cluster_baremetal_b" in json.loads(rec.read_text())["cluster"]
    else:
        assert rec.exists()
        capfd.readouterr()
        with pytest.raises(TKError):
            wf.new_cluster(ctx_b, backend)
        assert "already installed on this host" in capfd.readouterr().err  # terraform's own output


def test_modules_destroy_provisioner_references_only_self():
    """Terraform refuses a destroy-time provisioner that references var./local./other
    resources; the planner does too, and the shipped host modules pass."""
    from triton_kubernetes_amd.terraform import catalog
    from triton_kubernetes_amd.terraform.plan import plan_module

    for name in ("bare-metal-rancher-k8s-host", "bare-metal-mi355x-rancher-k8s-host"):
        text = open(os.path.join(catalog.CATALOG[name].local_dir, "main.tf")).read()
        assert "when       = destroy" in text and "on_failure = continue" in text
        assert os.path.exists(os.path.join(catalog.CATALOG[name].local_dir, "files", "cleanup_host.sh"))
    src = catalog.CATALOG["bare-metal-rancher-k8s-host"].local_dir
    with tempfile.TemporaryDirectory() as d:
        import shutil

        dst = os.path.join(d, "m")
        shutil.copytree(src, dst)
        main = os.path.join(dst, "main.tf")
        text = open(main).read()
        open(main, "w").write(text.replace("host             = self.input.host", "host             = var.host"))
        inputs = {"hostname": "h", "rancher_api_url": "https://r", "rancher_cluster_registration_token": "t",
                  "rancher_cluster_ca_checksum": "c", "rancher_host_labels": {"worker": "true"}, "host": "10.0.0.1"}
        rep = plan_module(dst, inputs, check_files=False)
        assert any("invalid reference from destroy provisioner: var" in e for e in rep.errors), rep.errors
        open(main, "w").write(text.replace("when       = destroy", "when       = sometimes"))
        rep = plan_module(dst, inputs, check_files=False)
        assert any("when: must be one of create, destroy" in e for e in rep.errors), rep.errors


def _host_module_copy(tmp_path, count_form: bool):
    """The shipped bare-metal host module -- or, ``count_form``, the round-5 shape of its
    cleanup resource (``count = var.node_cleanup ? 1 : 0``, no flag in ``input``)."""
    import shutil

    from triton_kubernetes_amd.terraform import catalog

    dst = tmp_path / ("mod-count" if count_form else "mod")
    shutil.copytree(catalog.CATALOG["bare-metal-rancher-k8s-host"].local_dir, dst, symlinks=False)
    if count_form:
        main = dst / "main.tf"
        text = main.read_text()
        text = text.replace('resource "terraform_data" "node_cleanup" {\n',
                            'resource "terraform_data" "node_cleanup" {\n  count            = var.node_cleanup ? 1 : 0\n')
        text = text.replace("    node_cleanup     = var.node_cleanup\n", "")
        main.write_text(text)
    return str(dst)


def _apply_host(tmp_path, mod, node_cleanup, cmd="apply"):
    doc = {"terraform": {"backend": {"local": {"path": str(tmp_path / "tf.tfstate")}}},
           "module": {"node_h": {"source": mod, "hostname": "h", "host": "10.9.0.1", "ssh_user": "u",
                                 "key_path": "k", "rancher_api_url": "https://r",
                                 "rancher_cluster_registration_token": "tok-a", "rancher_cluster_ca_checksum": "c",
                                 "rancher_host_labels": {"worker": "true"}, "node_cleanup": node_cleanup}}}
    work = tmp_path / "work"
    work.mkdir(exist_ok=True)
    (work / "main.tf.json").write_text(json.dumps(doc))
    return subprocess.run(["terraform", cmd, "-auto-approve"], cwd=work, capture_output=True, text=True)


@pytest.mark.parametrize("count_form", [False, True])
def test_turning_node_cleanup_off_on_a_host_in_service_tears_nothing_down(tmp_path, monkeypatch, count_form):
    """with ``count = var.node_cleanup ? 1 : 0`` turning the flag off on an
    applied host destroyed instance [0] -- running its destroy-time teardown on a live node.
    The resource now always exists and carries the flag in ``input``: the re-apply updates
    it in place, and the later destroy skips the teardown.  ``count_form`` pins the fake's
    Terraform semantics on the round-5 shape (that re-apply does tear the host down)."""
    install_fake_terraform(tmp_path, monkeypatch)
    bindir, _ = _stub_bin(tmp_path)
    monkeypatch.setenv("PATH", f"{bindir}:{os.environ['PATH']}")
    hosts = tmp_path / "hosts"
    hosts.mkdir()
    monkeypatch.setenv("FAKE_TF_HOSTS", str(hosts))
    mod = _host_module_copy(tmp_path, count_form)
    root = hosts / "10.9.0.1" / "root"
    first = _apply_host(tmp_path, mod, True)
    assert first.returncode == 0, first.stderr
    conn = root / "var/lib/rancher/agent/rancher2_connection_info.json"
    hostsim.install(str(root), "https://r", "tok-a")  # what the join left (RKE2, the agent)
    assert conn.exists()
    flip = _apply_host(tmp_path, mod, False)
    assert flip.returncode == 0, flip.stderr
    if count_form:
        assert "Destroying... (remote-exec)" in flip.stdout and not conn.exists()  # the live node torn down
        return
    assert "Destroying" not in flip.stdout and conn.exists()
    assert (root / "usr/local/bin/rke2-uninstall.sh").exists()
    gone = _apply_host(tmp_path, mod, False, cmd="destroy")
    assert gone.returncode == 0, gone.stderr
    assert "::tk-cleanup node_cleanup skipped" in gone.stdout and conn.exists()


def test_destroy_uses_the_flag_as_last_applied(tmp_path, monkeypatch):
    """``self.input`` is the resource as last applied: a destroy tears down when the applied
    flag is on, whatever the configuration now says."""
    install_fake_terraform(tmp_path, monkeypatch)
    bindir, _ = _stub_bin(tmp_path)
    monkeypatch.setenv("PATH", f"{bindir}:{os.environ['PATH']}")
    hosts = tmp_path / "hosts"
    hosts.mkdir()
    monkeypatch.setenv("FAKE_TF_HOSTS", str(hosts))
    mod = _host_module_copy(tmp_path, False)
    root = hosts / "10.9.0.1" / "root"
    assert _apply_host(tmp_path, mod, True).returncode == 0
    hostsim.install(str(root), "https://r", "tok-a")
    gone = _apply_host(tmp_path, mod, False, cmd="destroy")  # not applied: self.input still says true
    assert gone.returncode == 0, gone.stderr
    assert "rke2-uninstall.sh ok" in gone.stdout and not (root / "usr/local/bin/rke2-uninstall.sh").exists()
