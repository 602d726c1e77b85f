"""Machine- and version-independent module sources in the persisted ``main.tf.json``.

The reference persists ``github.com/joyent/triton-kubernetes//terraform/modules/<m>?ref=``
(``/root/reference/create/manager.go:160-171``, ``create/cluster.go:20-21``), so any
operator on any machine can apply a shared (Manta) document.  This CLI's modules ship in
its package, so the document names them ``tk::terraform/modules/<m>?ref=v<version>`` and
only the document an executor runs sees this install's directory
(``terraform/catalog.py:resolve_source``).  Covered here:

* the persisted document holds no filesystem path of the install;
* a manager created from install root A gets a node and is destroyed from install root B
  (A deleted in between), through the CLI as separate processes;
* a Manta document written by operator A (own key path, own install) applies from
  operator B;
* a document pinned to another version of the modules is refused by both executors until
  ``migrate manager`` re-pins it; documents of earlier versions (absolute paths) get a
  clear error and are rewritten by ``migrate manager``;
* the fake Terraform refuses an unresolved ``tk::`` source, so a rendering bug cannot pass.
"""

import json
import os
import shutil
import subprocess
import sys

import pytest
import yaml

from triton_kubernetes_amd import __version__
from triton_kubernetes_amd import workflows as wf
from triton_kubernetes_amd.backend import LocalBackend, MemoryBackend
from triton_kubernetes_amd.backend.manta import MantaBackend
from triton_kubernetes_amd.cloud.fake_manta import FakeManta
from triton_kubernetes_amd.errors import ExecutorError, TKError
from triton_kubernetes_amd.executor.direct import DirectExecutor
from triton_kubernetes_amd.executor.terraform import render
from triton_kubernetes_amd.state import State
from triton_kubernetes_amd.terraform import catalog
from triton_kubernetes_amd.utils.sshkeys import load_private_key
from triton_kubernetes_amd.workflows.migrate import migrate_manager, plan_migration

from helpers import FAKE_TF, install_fake_terraform, make_ctx, make_ssh_key, tf_calls

PKG = os.path.dirname(os.path.abspath(catalog.__file__ + "/.."))
PW = "tk-admin-pw-0123"
MGR = {"manager_cloud_provider": "baremetal", "name": "mgr", "rancher_admin_password": PW, "host": "10.0.0.10",
       "ssh_user": "ubuntu", "bastion_host": "", "key_path": "~/.ssh/id_rsa", "executor": "terraform"}
CLUSTER = {"cluster_manager": "mgr", "cluster_cloud_provider": "baremetal", "name": "dev",
           "k8s_version": "v1.28.10-rancher1-1", "k8s_network_provider": "flannel", "executor": "terraform",
           "nodes": [{"rancher_host_label": "worker", "node_count": 1, "hostname": "dev-w", "ssh_user": "u",
                      "key_path": "~/.ssh/id_rsa", "bastion_host": "", "hosts": ["10.0.0.13"]}]}
NODE = {"cluster_manager": "mgr", "cluster_name": "dev", "rancher_host_label": "worker", "node_count": 1,
        "hostname": "dev-w", "ssh_user": "u", "key_path": "~/.ssh/id_rsa", "bastion_host": "",
        "hosts": ["10.0.0.14"], "executor": "terraform"}


def _strings(v):
    if isinstance(v, str):
        yield v
    elif isinstance(v, dict):
        for x in v.values():
            yield from _strings(x)
    elif isinstance(v, list):
        for x in v:
            yield from _strings(x)


def _install(root) -> str:
    """A copy of the package under ``root`` (another venv / machine / version directory)."""
    shutil.copytree(PKG, os.path.join(root, "triton_kubernetes_amd"),
                    ignore=shutil.ignore_patterns("__pycache__", "*.so", "lib", "csrc"))
    return str(root)


def _cli(install: str, cfg: dict, *argv: str, cwd, env_extra=None) -> subprocess.CompletedProcess:
    path = os.path.join(str(cwd), f"cfg-{len(os.listdir(str(cwd)))}.yaml")
    with open(path, "w") as fh:
        yaml.safe_dump(cfg, fh)
    env = dict(os.environ, PYTHONPATH=install, **(env_extra or {}))
    proc = subprocess.run([sys.executable, "-m", "triton_kubernetes_amd", "--config", path, "--non-interactive",
                           *argv], cwd=str(cwd), env=env, capture_output=True, text=True, timeout=120)
    assert proc.returncode == 0, (argv, proc.stdout, proc.stderr)
    return proc


def _module_dirs(call) -> set:
    return {m["source"] for m in call["doc"].get("module", {}).values()}


# --- the persisted form ---------------------------------------------------------------------
def test_persisted_document_names_no_install_path(tmp_path, monkeypatch):
    log = install_fake_terraform(tmp_path, monkeypatch)
    be = LocalBackend(str(tmp_path / "state"))
    wf.new_manager(make_ctx(MGR), be)
    wf.new_cluster(make_ctx(CLUSTER), be)
    wf.new_node(make_ctx(NODE), be)
    text = open(os.path.join(be.root, "mgr", "main.tf.json")).read()
    doc = json.loads(text)
    assert catalog.PACKAGE_ROOT not in text and catalog.MODULES_DIR not in text
    for key, block in doc["module"].items():
        assert block["source"] == f"tk::{catalog.module_from_source(block['source']).path}?ref=v{__version__}", key
        # no value of any module block is a filesystem path of the operator's machine
        assert not [s for s in _strings(block) if s.startswith("/")], key
    # ... while Terraform was given this install's directories, which exist
    apply = [c for c in tf_calls(log) if c["argv"][0] == "apply"][-1]
    for src in _module_dirs(apply):
        assert src.startswith(catalog.MODULES_DIR + os.sep) and os.path.isdir(src)


def test_source_url_still_persists_the_reference_form():
    st = State("mgr")
    from triton_kubernetes_amd.models import baremetal

    baremetal.new_manager(make_ctx(dict(MGR, source_url="github.com/me/fork", source_ref="v1")), st, "mgr")
    assert st.manager()["source"] == "github.com/me/fork//terraform/modules/bare-metal-rancher?ref=v1"
    assert catalog.resolve_source(st.manager()["source"]) == st.manager()["source"]  # untouched by render


def test_fake_terraform_refuses_an_unresolved_tk_source(tmp_path):
    d = tmp_path / "wd"
    d.mkdir()
    (d / "main.tf.json").write_text(json.dumps(
        {"module": {"cluster-manager": {"source": "tk::terraform/modules/bare-metal-rancher?ref=v0.8.2"}}}))
    res = subprocess.run([sys.executable, FAKE_TF, "init"], cwd=d, capture_output=True, text=True)
    assert res.returncode == 1 and "download not supported for scheme 'tk'" in res.stderr


# --- two installs, one document ----------------------------------------------------------------
@pytest.mark.slow
def test_manager_created_from_root_a_is_extended_and_destroyed_from_root_b(tmp_path, monkeypatch):
    """An upgrade into a new venv (or a second checkout) on the same machine: the local
    backend is shared, the package directory is not."""
    log = install_fake_terraform(tmp_path, monkeypatch)
    home = tmp_path / "home"
    home.mkdir()
    env = {"HOME": str(home), "BACKEND_PROVIDER": "local"}
    a = _install(tmp_path / "root-a")
    b = _install(tmp_path / "root-b")
    work = tmp_path / "work"
    work.mkdir()

    _cli(a, MGR, "create", "manager", cwd=work, env_extra=env)
    _cli(a, CLUSTER, "create", "cluster", cwd=work, env_extra=env)
    a_calls = [c for c in tf_calls(log) if c["argv"][0] == "apply"]
    assert a_calls and all(s.startswith(a + os.sep) for c in a_calls for s in _module_dirs(c))
    shutil.rmtree(a)  # install A is gone: nothing may still point into it

    open(log, "w").close()
    _cli(b, NODE, "create", "node", cwd=work, env_extra=env)
    apply = [c for c in tf_calls(log) if c["argv"][0] == "apply"][-1]
    assert all(s.startswith(b + os.sep) for s in _module_dirs(apply))
    assert "node_baremetal_dev_dev-w-2" in apply["doc"]["module"]
    # B's apply started from A's state: nothing re-created, the new node added
    assert apply["prior"]["modules"] == ["cluster-manager", "cluster_baremetal_dev", "node_baremetal_dev_dev-w-1"]

    _cli(b, {"cluster_manager": "mgr", "executor": "terraform"}, "destroy", "manager", cwd=work, env_extra=env)
    assert not os.path.exists(home / ".triton-kubernetes" / "mgr")


@pytest.mark.slow
def test_manta_document_from_operator_a_applies_from_operator_b(tmp_path, monkeypatch):
    """Two operators share a Manta-backed manager: each has its own install directory and
    its own path to the account key."""
    log = install_fake_terraform(tmp_path, monkeypatch)
    key_a = make_ssh_key(tmp_path / "a-id_rsa")
    key = load_private_key(key_a)
    (tmp_path / "b-keys").mkdir()
    key_b = str(tmp_path / "b-keys" / "triton.pem")
    shutil.copy(key_a, key_b)
    fake = FakeManta("acct").start()
    try:
        fake.add_key(key)
        manta = {"backend_provider": "manta", "triton_account": "acct", "triton_key_id": key.fingerprint_md5(),
                 "triton_url": "https://triton", "manta_url": fake.url}
        a = _install(tmp_path / "operator-a")
        b = _install(tmp_path / "operator-b")
        work = tmp_path / "work"
        work.mkdir()
        _cli(a, dict(MGR, triton_key_path=key_a, **manta), "create", "manager", cwd=work)
        _cli(a, dict(CLUSTER, triton_key_path=key_a, **manta), "create", "cluster", cwd=work)
        stored = json.loads(fake.objects["/acct/stor/triton-kubernetes/mgr/main.tf.json"][0])
        assert not [s for blk in stored["module"].values() for s in _strings(blk) if s.startswith("/")]
        shutil.rmtree(a)

        open(log, "w").close()
        _cli(b, dict(NODE, triton_key_path=key_b, **manta), "create", "node", cwd=work)
        apply = [c for c in tf_calls(log) if c["argv"][0] == "apply"][-1]
        assert all(s.startswith(b + os.sep) for s in _module_dirs(apply))
        assert apply["prior"]["modules"] == ["cluster-manager", "cluster_baremetal_dev", "node_baremetal_dev_dev-w-1"]
        be = MantaBackend("acct", key_b, key.fingerprint_md5(), "https://triton", fake.url)
        assert "dev-w-2" in be.state("mgr").nodes("cluster_baremetal_dev")
        _cli(b, dict({"cluster_manager": "mgr", "executor": "terraform", "triton_key_path": key_b}, **manta),
             "destroy", "manager", cwd=work)
        assert be.states() == []
    finally:
        fake.stop()


def test_render_uses_this_operators_backend_block(tmp_path):
    """The persisted manta block carries the writer's key path (reference quirk Q9); the
    document Terraform < 1.3 runs gets the running operator's."""
    key = make_ssh_key(tmp_path / "id_rsa")
    pk = load_private_key(key)
    class _NoManta:
        def put_directory(self, path):
            pass

    be = MantaBackend("acct", key, pk.fingerprint_md5(), "https://triton", "https://manta.invalid",
                      client=_NoManta())
    st = State("mgr")
    st.set_manager({"source": "github.com/joyent/triton-kubernetes//terraform/modules/bare-metal-rancher?ref=master",
                    "name": "mgr"})
    st.set_terraform_backend_config("terraform.backend.manta", {"account": "acct", "key_material": "/home/alice/k",
                                                                 "key_id": "x", "path": "/triton-kubernetes/mgr"})
    doc = json.loads(render(st, (1, 2, 9), be).body)
    assert doc["terraform"]["backend"]["manta"]["key_material"] == key
    assert json.loads(st.bytes())["terraform"]["backend"]["manta"]["key_material"] == "/home/alice/k"


# --- version pins and older documents ------------------------------------------------------------
def _pinned(ref: str) -> State:
    st = State("mgr")
    st.set_manager({"source": f"tk::terraform/modules/bare-metal-rancher?ref={ref}", "name": "mgr", "host": "h",
                    "rancher_admin_password": PW, "ssh_user": "ubuntu", "key_path": "k"})
    return st


def test_ref_mismatch_is_refused_by_both_executors_until_migrated(tmp_path, monkeypatch):
    log = install_fake_terraform(tmp_path, monkeypatch)
    be = MemoryBackend()
    st = _pinned("v0.0.1")
    be.persist_state(st)
    with pytest.raises(catalog.ModuleRefMismatch) as exc:
        wf.new_cluster(make_ctx(CLUSTER), be)
    msg = str(exc.value)
    assert "module.cluster-manager is pinned to the triton-kubernetes modules v0.0.1" in msg
    assert f"this CLI ships v{__version__}" in msg and "migrate manager" in msg
    assert tf_calls(log) == []  # refused before any question or terraform run
    with pytest.raises(catalog.ModuleRefMismatch):
        DirectExecutor().plan(st)
    from triton_kubernetes_amd.executor.terraform import TerraformExecutor

    with pytest.raises(catalog.ModuleRefMismatch):  # the executor refuses it on its own, before init
        TerraformExecutor().apply(st, be)
    assert [c["argv"][0] for c in tf_calls(log)] == ["version"]
    assert be.state("mgr").module("cluster_baremetal_dev") is None  # nothing persisted

    # migrate re-pins; then the same create goes through
    new, errors, _ = plan_migration(make_ctx({}), st.doc)
    assert not errors and new["cluster-manager"]["source"].endswith(f"?ref=v{__version__}")
    migrate_manager(make_ctx({"cluster_manager": "mgr"}), be)
    assert be.state("mgr").manager()["source"] == f"tk::terraform/modules/bare-metal-rancher?ref=v{__version__}"
    wf.new_cluster(make_ctx(CLUSTER), be)
    assert "dev-w-1" in be.state("mgr").nodes("cluster_baremetal_dev")


def test_unknown_tk_module_is_an_error():
    with pytest.raises(ExecutorError, match="names no module of this CLI"):
        catalog.resolve_source(f"tk::terraform/modules/no-such-module?ref=v{__version__}", "cluster-manager")


def test_absolute_path_document_of_another_install_is_explained_and_migrated(tmp_path, monkeypatch):
    log = install_fake_terraform(tmp_path, monkeypatch)
    be = MemoryBackend()
    st = State("mgr")
    gone = "/opt/venvs/tk-0.8.1/lib/python3.10/site-packages/triton_kubernetes_amd/terraform/modules/bare-metal-rancher"
    st.set_manager({"source": gone, "name": "mgr", "host": "h", "rancher_admin_password": PW,
                    "ssh_user": "ubuntu", "key_path": "k"})
    be.persist_state(st)
    with pytest.raises(TKError) as exc:
        wf.new_cluster(make_ctx(CLUSTER), be)
    assert "another triton-kubernetes install" in str(exc.value) and "migrate manager" in str(exc.value)
    assert tf_calls(log) == []
    ctx = make_ctx({"cluster_manager": "mgr"})
    migrate_manager(ctx, be)
    assert f"{gone} -> tk::terraform/modules/bare-metal-rancher?ref=v{__version__}" in ctx.out.getvalue()
    assert be.read_blob("mgr", "main.tf.json.pre-migrate") is not None
    wf.new_cluster(make_ctx(CLUSTER), be)
    assert be.state("mgr").manager()["source"].startswith("tk::")
