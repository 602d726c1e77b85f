"""Two CLI runs on one cluster manager (a shared state backend): neither overwrites the
other's clusters or nodes (``State.rebase`` under the backend lock, destroy re-reads)."""

import contextlib

import pytest

from helpers import make_ctx
from triton_kubernetes_amd import versions
from triton_kubernetes_amd.backend import MemoryBackend
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.rancher.fake import FakeRancher
from triton_kubernetes_amd.state import State
from triton_kubernetes_amd.state.document import StateError
from triton_kubernetes_amd.workflows import delete_cluster, new_cluster, new_manager


def test_rebase_three_way():
    base = State("m", b'{"module": {"a": {"x": 1}, "b": {"x": 2}}}').mark_base()
    base.set_module("c", {"x": 3})        # ours: added
    base.delete_module("b")               # ours: deleted
    current = State("m", b'{"module": {"a": {"x": 1}, "b": {"x": 2}, "d": {"x": 4}}}')  # theirs: added d
    assert base.rebase(current) == ["d"]
    assert base.modules() == {"a": {"x": 1}, "c": {"x": 3}, "d": {"x": 4}}
    # nobody else wrote: nothing to merge
    mine = State("m", b'{"module": {"a": {"x": 1}}}').mark_base()
    mine.set_module("a", {"x": 9})
    assert mine.rebase(State("m", b'{"module": {"a": {"x": 1}}}')) == []
    assert mine.modules() == {"a": {"x": 9}}
    # both changed one module differently: refused
    mine = State("m", b'{"module": {"a": {"x": 1}}}').mark_base()
    mine.set_module("a", {"x": 2})
    with pytest.raises(StateError, match=r"changed by another triton-kubernetes run \(module.a\)"):
        mine.rebase(State("m", b'{"module": {"a": {"x": 3}}}'))
    # the same change on both sides is not a conflict; the backend block is ours
    mine = State("m", b"{}").mark_base()
    mine.set_module("a", {"x": 1})
    mine.set_terraform_backend_config("terraform.backend.local", {"path": "p"})
    assert mine.rebase(State("m", b'{"module": {"a": {"x": 1}, "z": {}}}')) == ["a", "z"]
    assert mine.doc["terraform"] == {"backend": {"local": {"path": "p"}}} and set(mine.modules()) == {"a", "z"}


class _Interleaved(MemoryBackend):
    """Runs ``hook`` (another CLI run) once, just before this run takes the lock."""

    hook = None

    @contextlib.contextmanager
    def lock(self, name, *a, **kw):
        hook, self.hook = self.hook, None
        if hook is not None:
            hook()
        with super().lock(name, *a, **kw):
            yield


def _cluster_ctx(name, **extra):
    return make_ctx(dict({"executor": "direct", "cluster_manager": "mgr", "cluster_cloud_provider": "baremetal",
                          "name": name, "k8s_version": versions.DEFAULT_K8S_VERSION,
                          "k8s_network_provider": "calico"}, **extra))


@pytest.fixture
def manager():
    fake = FakeRancher.for_manager("mgr", "s3cret-passw0rd").start()
    backend = _Interleaved()
    new_manager(make_ctx({"executor": "direct", "manager_cloud_provider": "baremetal", "name": "mgr",
                          "rancher_admin_password": "s3cret-passw0rd", "rancher_bootstrap_password": fake.bootstrap_password, "host": "rancher+" + fake.url,
                          "ssh_user": "ubuntu", "bastion_host": "", "key_path": "k"}), backend)
    yield fake, backend
    fake.stop()


def test_concurrent_creates_keep_both_clusters(manager):
    fake, backend = manager
    backend.hook = lambda: new_cluster(_cluster_ctx("beta"), backend)
    ctx = _cluster_ctx("alpha")
    new_cluster(ctx, backend)
    assert set(backend.state("mgr").clusters()) == {"alpha", "beta"}
    assert "kept changes another run persisted meanwhile (cluster_baremetal_beta)" in ctx.out.getvalue()


def test_same_cluster_from_two_runs_is_refused(manager):
    fake, backend = manager
    backend.hook = lambda: new_cluster(_cluster_ctx("gamma", k8s_network_provider="flannel"), backend)
    with pytest.raises(TKError, match=r"changed by another triton-kubernetes run \(module.cluster_baremetal_gamma\)"):
        new_cluster(_cluster_ctx("gamma"), backend)
    assert backend.state("mgr").module("cluster_baremetal_gamma")["k8s_network_provider"] == "flannel"


def test_destroy_rereads_under_the_lock(manager):
    fake, backend = manager
    new_cluster(_cluster_ctx("alpha"), backend)
    backend.hook = lambda: new_cluster(_cluster_ctx("beta"), backend)
    delete_cluster(make_ctx({"executor": "direct", "cluster_manager": "mgr", "cluster_name": "alpha"}), backend)
    assert set(backend.state("mgr").clusters()) == {"beta"}
