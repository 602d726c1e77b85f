"""Pinned versions are coherent across every delivery path, and the fake Rancher enforces
what a real Rancher v2.10.3 enforces (bootstrap password, KDM Kubernetes lists of RKE1 and RKE2,
password length).

Reference: ``/root/reference/create/cluster.go:349-356`` (k8s choices of its pinned
server) and ``/root/reference/terraform/modules/triton-rancher/variables.tf:14-22``.
"""

import os
import re

import pytest

from triton_kubernetes_amd import versions
from triton_kubernetes_amd.errors import ConfigError, TKError
from triton_kubernetes_amd.models import baremetal
from triton_kubernetes_amd.node import manager as node_manager
from triton_kubernetes_amd.node import plan as node_plan
from triton_kubernetes_amd.rancher.client import RancherClient
from triton_kubernetes_amd.rancher.fake import FakeRancher
from triton_kubernetes_amd.state import State
from triton_kubernetes_amd.terraform import generate
from triton_kubernetes_amd.terraform.catalog import MODULES_DIR

from helpers import make_ctx

OLD = "v1.9.5-rancher1-1"  # the reference's default: no RKE1 release of Rancher 2.10


def _var_default(module: str, var: str) -> str:
    text = open(os.path.join(MODULES_DIR, module, "variables.tf"), encoding="utf-8").read()
    m = re.search(r'variable "%s" \{.*?default\s+=\s+"([^"]*)"' % var, text, re.S)
    assert m, (module, var)
    return m.group(1)


def test_defaults_agree_everywhere():
    assert versions.DEFAULT_DISTRIBUTION == "rke2"
    assert versions.DEFAULT_K8S_VERSION in [v for _, v in versions.RKE2_VERSIONS]
    assert versions.DEFAULT_RKE1_VERSION in [v for _, v in versions.K8S_VERSIONS]
    for mod in ("bare-metal-rancher-k8s", "triton-rancher-k8s", "aws-rancher-k8s", "gcp-rancher-k8s",
                "azure-rancher-k8s", "vsphere-rancher-k8s"):
        assert _var_default(mod, "k8s_version") == versions.DEFAULT_K8S_VERSION
        assert _var_default(mod, "k8s_distribution") == versions.DEFAULT_DISTRIBUTION
        assert _var_default(mod, "k8s_network_provider") in versions.RKE2_CNIS
    for mod in ("bare-metal-rancher-k8s-host", "bare-metal-mi355x-rancher-k8s-host", "triton-rancher-k8s-host"):
        assert _var_default(mod, "k8s_distribution") == versions.DEFAULT_DISTRIBUTION
    for mod in ("bare-metal-rancher", "triton-rancher", "aws-rancher", "gcp-rancher", "azure-rancher"):
        assert _var_default(mod, "rancher_server_image") == versions.SERVER_IMAGE
        assert _var_default(mod, "docker_engine_install_url") == versions.DOCKER_INSTALL_URL
    for mod in ("bare-metal-rancher-k8s-host", "bare-metal-mi355x-rancher-k8s-host", "aws-rancher-k8s-host"):
        assert _var_default(mod, "rancher_agent_image") == versions.AGENT_IMAGE
        assert _var_default(mod, "docker_engine_install_url") == versions.DOCKER_INSTALL_URL
    assert node_manager.DEFAULT_SERVER_IMAGE == versions.SERVER_IMAGE
    assert node_manager.DEFAULT_DOCKER_INSTALL_URL == node_plan.DEFAULT_DOCKER_INSTALL_URL == versions.DOCKER_INSTALL_URL
    assert node_plan.DEFAULT_AGENT_IMAGE == versions.AGENT_IMAGE
    assert versions.SERVER_IMAGE.endswith(versions.RANCHER_VERSION) and versions.AGENT_IMAGE.endswith(
        versions.RANCHER_VERSION)
    for img in (versions.DEVICE_PLUGIN_IMAGE, versions.NODE_LABELLER_IMAGE, versions.RCCL_PROBE_IMAGE):
        assert ":" in img and not img.endswith(":latest") and "latest" not in img.split(":")[1]
    assert _var_default("rancher-k8s-mi355x-addons", "device_plugin_image") == versions.DEVICE_PLUGIN_IMAGE


def test_cli_rejects_kubernetes_releases_outside_the_pinned_rancher():
    st = State("mgr")
    st.set_manager({"source": "x", "name": "mgr"})
    ctx = make_ctx({"name": "dev", "k8s_version": OLD, "k8s_network_provider": "flannel"})
    with pytest.raises(ConfigError, match="not an RKE1 release offered by Rancher v2.10.3"):
        baremetal.new_cluster(ctx, None, st)
    # the display name maps to the pinned release of the distribution (RKE2 unless the
    # release string or k8s_distribution says RKE1); a patch release of a pinned minor passes
    for extra, given, want, dist in (({}, "v1.29", "v1.29.14+rke2r1", "rke2"),
                                     ({"k8s_distribution": "rke1"}, "v1.28", "v1.28.15-rancher1-1", "rke1"),
                                     ({}, "v1.28.12-rancher1-1", "v1.28.12-rancher1-1", "rke1"),
                                     ({}, "v1.30.4+rke2r1", "v1.30.4+rke2r1", "rke2")):
        st = State("mgr")
        st.set_manager({"source": "x", "name": "mgr"})
        baremetal.new_cluster(make_ctx(dict(extra, name="dev", k8s_version=given, k8s_network_provider="flannel")),
                              None, st)
        assert st.get("module.cluster_baremetal_dev.k8s_version") == want
        assert st.get("module.cluster_baremetal_dev.k8s_distribution") == dist
    # an RKE1-only minor is not an RKE2 release; a release of the other distribution is refused
    for bad, match in (({"k8s_version": "v1.28"}, "not an RKE2 release"),
                       ({"k8s_version": "v1.29.14+rke2r1", "k8s_distribution": "rke1"}, "is an RKE2 release"),
                       ({"k8s_version": "v1.29", "k8s_network_provider": "weave"}, "not a RKE2 network provider")):
        st = State("mgr")
        st.set_manager({"source": "x", "name": "mgr"})
        with pytest.raises(ConfigError, match=match):
            baremetal.new_cluster(make_ctx(dict({"name": "dev", "k8s_network_provider": "flannel"}, **bad)), None, st)


def test_short_admin_password_rejected():
    st = State("mgr")
    ctx = make_ctx({"name": "mgr", "rancher_admin_password": "admin", "host": "10.0.0.1", "ssh_user": "u",
                    "bastion_host": "", "key_path": "k"})
    with pytest.raises(ConfigError, match="at least 12 characters"):
        baremetal.new_manager(ctx, st, "mgr")


def test_fake_rancher_has_no_admin_admin_and_enforces_kdm():
    with FakeRancher() as fake:  # started without CATTLE_BOOTSTRAP_PASSWORD: random first password
        with pytest.raises(TKError):
            RancherClient(fake.url).login("admin", "admin")
    with FakeRancher(bootstrap_password="b00t-b00t-b00t") as fake:
        with pytest.raises(TKError):
            RancherClient(fake.url).bootstrap("long-enough-pw", fake.url, "admin", timeout=5)
        with pytest.raises(TKError, match="at least 12"):  # password-min-length
            RancherClient(fake.url).bootstrap("short", fake.url, "b00t-b00t-b00t", timeout=5)
        outs = RancherClient(fake.url).bootstrap("long-enough-pw", fake.url, "b00t-b00t-b00t", timeout=5)
        client = RancherClient(fake.url, outs["rancher_access_key"], outs["rancher_secret_key"])
        assert client.k8s_versions() == [v for _, v in versions.K8S_VERSIONS]
        with pytest.raises(TKError, match="not offered"):  # client-side check against the server list
            client.ensure_cluster("old", OLD)
        with pytest.raises(TKError, match="HTTP 422"):  # and the server itself refuses it
            client.create_cluster("old", OLD, "flannel")
        assert client.ensure_cluster("new").cluster_id
        # re-running the bootstrap after the password change (resume) logs in with the admin password
        again = RancherClient(fake.url).bootstrap("long-enough-pw", fake.url, "b00t-b00t-b00t", timeout=5)
        assert again["rancher_access_key"] and fake.state.admin_password == "long-enough-pw"


def test_same_minor_release_substituted_from_the_server_list():
    with FakeRancher(bootstrap_password="b00t-b00t-b00t", k8s_versions=["v1.28.15-rancher1-1", "v1.27.16-rancher1-1"]) \
            as fake:
        outs = RancherClient(fake.url).bootstrap("long-enough-pw", fake.url, "b00t-b00t-b00t", timeout=5)
        client = RancherClient(fake.url, outs["rancher_access_key"], outs["rancher_secret_key"])
        info = client.ensure_cluster("dev", "v1.28.10-rancher1-1")
        rke = fake.state.clusters[info.cluster_id]["rancherKubernetesEngineConfig"]
        assert rke["kubernetesVersion"] == "v1.28.15-rancher1-1"
        assert "using v1.28.15-rancher1-1" in client.last_version_note
        with pytest.raises(TKError):
            client.ensure_cluster("gone", "v1.26.15-rancher1-1")
    with FakeRancher(bootstrap_password="b00t-b00t-b00t", rke2_versions=["v1.30.12+rke2r1"]) as fake:
        outs = RancherClient(fake.url).bootstrap("long-enough-pw", fake.url, "b00t-b00t-b00t", timeout=5)
        client = RancherClient(fake.url, outs["rancher_access_key"], outs["rancher_secret_key"])
        client.ensure_cluster("dev", "v1.30.10+rke2r1")
        assert fake.state.v2_clusters["fleet-default/dev"]["spec"]["kubernetesVersion"] == "v1.30.12+rke2r1"
        with pytest.raises(TKError, match="not offered"):
            client.ensure_cluster("gone", versions.DEFAULT_K8S_VERSION)  # v1.31: not in this server's KDM
        with pytest.raises(TKError, match="HTTP 422"):  # and the server itself refuses it
            client.create_v2_cluster("gone", versions.DEFAULT_K8S_VERSION, "canal")


def test_bootstrap_password_is_random_and_never_on_a_command_line(tmp_path):
    """the first-login password is random, kept in the state backend (0600),
    handed to the server in a 0600 env file removed after start, and no function of the
    admin password appears in any host command line, container env or rendered script."""
    import stat

    from triton_kubernetes_amd.backend import LocalBackend
    from triton_kubernetes_amd.rancher import bootstrap_secret

    be = LocalBackend(str(tmp_path / "state"))
    pw = bootstrap_secret.ensure(be, "mgr")
    assert len(pw) >= 32 and bootstrap_secret.ensure(be, "mgr") == pw  # kept, not regenerated
    blob = tmp_path / "state" / "mgr" / bootstrap_secret.BLOB
    assert stat.S_IMODE(os.stat(blob).st_mode) == 0o600
    assert pw != versions.bootstrap_password("mgr", "tk-admin-pw-0123")
    admin = "tk-admin-pw-0123"
    derived = versions.bootstrap_password("mgr", admin)
    script = node_manager.manager_install_script({"rancher_admin_password": admin}, pw)
    assert "--env-file" in script and "-e CATTLE_BOOTSTRAP_PASSWORD" not in script
    assert admin not in script and derived not in script
    run = next(ln for ln in script.splitlines() if "docker run" in ln)
    assert pw not in run  # the command line names the file, not the value
    assert "| sudo sh" not in script  # downloaded, then run
    for mod in ("bare-metal-rancher", "triton-rancher", "aws-rancher", "gcp-rancher", "azure-rancher"):
        main = open(os.path.join(MODULES_DIR, mod, "main.tf"), encoding="utf-8").read()
        assert "sha256(" not in main and "bootstrap_password = var.rancher_bootstrap_password" in main
        server = open(os.path.join(MODULES_DIR, mod, "files", "install_rancher_server.sh.tftpl")).read()
        assert "--env-file" in server and "-e CATTLE_BOOTSTRAP_PASSWORD" not in server
        setup = open(os.path.join(MODULES_DIR, mod, "files", "setup_rancher.sh.tftpl")).read()
        assert "rancher_admin_password" not in setup  # set over SSH stdin by read_api_key.sh
        assert '"password":"admin"' not in setup and "--data-binary @-" in setup


def test_docker_install_checksum_is_enforced_when_given():
    lines = node_manager.docker_install_lines("https://x/24.0.sh", "ab" * 32)
    assert "sha256sum -c" in lines and "curl -fsSL -o /tmp/tk-install-docker.sh" in lines
    assert "sha256sum" not in node_manager.docker_install_lines("https://x/24.0.sh")
    tpl = generate.scripts.DOCKER_INSTALL
    assert '%{ if docker_install_sha256 != "" ~}' in tpl and "| sudo sh" not in tpl
