"""Error-string contract tests ported from the reference's Go tests.

Sources: ``create/node_test.go``, ``cmd/version_test.go``,
``util/backend_prompt_test.go``, ``destroy/{cluster,manager,node}_test.go``,
``get/{cluster,manager}_test.go``.  Every expected string is the reference's.
"""

import io

import pytest

from triton_kubernetes_amd.backend import MemoryBackend, prompt_for_backend
from triton_kubernetes_amd.cli.main import version_text
from triton_kubernetes_amd.errors import TKError
from triton_kubernetes_amd.models.common import new_hostnames
from triton_kubernetes_amd.state import State
from triton_kubernetes_amd.workflows import (delete_cluster, delete_manager, delete_node, get_cluster,
                                              get_manager)

from helpers import make_ctx

# --- create/node_test.go --------------------------------------------------------------------
HOSTNAME_CASES = [
    (["test-1", "test-2"], "test", 0, []),
    (["test-1", "test-2"], "test", -10, []),
    (["test-1", "test-2"], "bar", 1, ["bar-1"]),
    (["test"], "test", 1, ["test-1"]),
    (["foo", "bar"], "test", 3, ["test-1", "test-2", "test-3"]),
    (["test"], "test", 3, ["test-1", "test-2", "test-3"]),
    (["test-1", "test-2", "bar-3", "bar-4"], "test", 3, ["test-3", "test-4", "test-5"]),
]


@pytest.mark.parametrize("existing,name,count,expected", HOSTNAME_CASES)
def test_get_new_hostnames(existing, name, count, expected):
    assert new_hostnames(existing, name, count) == expected


def test_hostnames_atoi_semantics():
    assert new_hostnames(["w-+7", "w-1_0", "w- 9"], "w", 1) == ["w-8"]
    # strconv.Atoi refuses a trailing newline and anything outside int64 (a 64-bit build)
    assert new_hostnames(["w-5\n", "w-3"], "w", 1) == ["w-4"]
    assert new_hostnames(["w-9223372036854775808", "w-2"], "w", 1) == ["w-3"]
    assert new_hostnames(["w-9223372036854775806"], "w", 1) == ["w-9223372036854775807"]
    assert new_hostnames(["w--9223372036854775809", "w-0"], "w", 1) == ["w-1"]


# --- cmd/version_test.go ------------------------------------------------------------------------
def test_version():
    assert version_text("beta") == "triton-kubernetes v0.8.2 (beta)\n"


def test_missing_version():
    assert "no version set for this build" in version_text("")


# --- util/backend_prompt_test.go -----------------------------------------------------------------
def _backend_err(values):
    with pytest.raises(TKError) as exc:
        prompt_for_backend(make_ctx(values, non_interactive=values.get("non-interactive", True)))
    return str(exc.value)


def test_backend_unsupported_provider():
    assert _backend_err({"non-interactive": True, "backend_provider": "S3"}) == "Unsupported backend provider 'S3'"


def test_backend_no_triton_account():
    assert _backend_err({"non-interactive": True, "backend_provider": "manta"}) == \
        "triton_account must be specified"


def test_backend_no_triton_key_path():
    assert _backend_err({"non-interactive": True, "backend_provider": "manta", "triton_account": "xyz"}) == \
        "triton_key_path must be specified"


def test_backend_invalid_key_path_interactive():
    vals = {"non-interactive": False, "backend_provider": "manta", "triton_account": "xyz", "triton_key_path": ""}
    with pytest.raises(TKError) as exc:
        prompt_for_backend(make_ctx(vals, non_interactive=False, answers=[]))
    assert str(exc.value) == "Unable to read private key: open : no such file or directory"


def test_no_triton_url_non_interactive():
    assert _backend_err({"non-interactive": True, "backend_provider": "manta", "triton_account": "xyz",
                         "triton_key_path": "", "triton_key_id": ""}) == "triton_url must be specified"


def test_no_manta_url_non_interactive():
    assert _backend_err({"non-interactive": True, "backend_provider": "manta", "triton_account": "xyz",
                         "triton_key_path": "", "triton_key_id": "", "triton_url": "xyz.triton.com"}) == \
        "manta_url must be specified"


# --- destroy/*_test.go ----------------------------------------------------------------------------
MOCK_CLUSTERS = b'''{"module":{"cluster_1":{"name":"dev_cluster"},"cluster_2":{"name":"beta_cluster"},
                      "cluster_3":{"name":"prod_cluster"}}}'''
MOCK_NODE_HOST = b'{"module":{"cluster_triton_dev-cluster":{"name":"dev_cluster"}}}'


def _err(fn, backend, values=None, non_interactive=True):
    ctx = make_ctx(values or {}, non_interactive=non_interactive, answers=[] if not non_interactive else None)
    with pytest.raises(TKError) as exc:
        fn(ctx, backend)
    return str(exc.value)


def _mock(names, state_doc=None):
    states = {"dev-manager": State("dev-manager", state_doc)} if state_doc is not None else {}
    return MemoryBackend(states=states, state_names=names)


def test_delete_cluster_no_cluster_manager():
    assert _err(delete_cluster, _mock([])) == "No cluster managers."


def test_delete_cluster_missing_cluster_manager():
    assert _err(delete_cluster, _mock(["dev-manager", "beta-manager"])) == "cluster_manager must be specified"


def test_delete_cluster_manager_not_exist():
    assert _err(delete_cluster, _mock(["dev-manager", "beta-manager"]), {"cluster_manager": "prod-manager"}) == \
        "Selected cluster manager 'prod-manager' does not exist."


def test_delete_cluster_must_specify_cluster_name():
    assert _err(delete_cluster, _mock(["dev-manager", "beta-manager"], MOCK_CLUSTERS),
                {"cluster_manager": "dev-manager"}) == "cluster_name must be specified"


def test_delete_cluster_not_exist():
    assert _err(delete_cluster, _mock(["dev-manager", "beta-manager"], MOCK_CLUSTERS),
                {"cluster_manager": "dev-manager", "cluster_name": "cluster_alpha"}) == \
        "A cluster named 'cluster_alpha', does not exist."


def test_delete_manager_no_cluster_manager():
    assert _err(delete_manager, _mock([])) == \
        "No cluster managers, please create a cluster manager before creating a kubernetes cluster."


def test_delete_manager_missing_cluster_manager():
    assert _err(delete_manager, _mock(["dev-manager", "beta-manager"])) == "cluster_manager must be specified"


def test_delete_manager_not_exist():
    assert _err(delete_manager, _mock(["dev-manager", "beta-manager"]), {"cluster_manager": "prod-cluster"}) == \
        "Selected cluster manager 'prod-cluster' does not exist."


def test_delete_node_no_cluster_manager():
    assert _err(delete_node, _mock([])) == \
        "No cluster managers, please create a cluster manager before creating a kubernetes node."


def test_delete_node_missing_cluster_manager():
    assert _err(delete_node, _mock(["dev-manager", "beta-manager"])) == "cluster_manager must be specified"


def test_delete_node_manager_not_exist():
    assert _err(delete_node, _mock(["dev-manager", "beta-manager"]), {"cluster_manager": "prod-manager"}) == \
        "Selected cluster manager 'prod-manager' does not exist."


def test_delete_node_must_specify_cluster_name():
    assert _err(delete_node, _mock(["dev-manager", "beta-manager"], MOCK_CLUSTERS),
                {"cluster_manager": "dev-manager"}) == "cluster_name must be specified"


def test_delete_node_cluster_not_exist():
    assert _err(delete_node, _mock(["dev-manager", "beta-manager"], MOCK_CLUSTERS),
                {"cluster_manager": "dev-manager", "cluster_name": "cluster_alpha"}) == \
        "A cluster named 'cluster_alpha', does not exist."


def test_delete_node_hostname_must_be_specified():
    assert _err(delete_node, _mock(["dev-manager", "beta-manager"], MOCK_NODE_HOST),
                {"cluster_manager": "dev-manager", "cluster_name": "dev_cluster"}) == "hostname must be specified"


def test_delete_node_not_exist():
    assert _err(delete_node, _mock(["dev-manager", "beta-manager"], MOCK_NODE_HOST),
                {"cluster_manager": "dev-manager", "cluster_name": "dev_cluster", "hostname": "dev_node_host"}) == \
        "A node named 'dev_node_host', does not exist."


# --- get/*_test.go -------------------------------------------------------------------------------------
def test_get_cluster_no_cluster_manager():
    assert _err(get_cluster, _mock([])) == "No cluster managers."


def test_get_cluster_missing_cluster_manager():
    assert _err(get_cluster, _mock(["dev-manager", "test-manager"])) == "cluster_manager must be specified"


def test_get_cluster_unidentified_manager():
    assert _err(get_cluster, _mock(["dev-manager", "test-manager"]), {"cluster_manager": "xyz"}) == \
        "Selected cluster manager 'xyz' does not exist."


def test_get_cluster_no_cluster():
    assert _err(get_cluster, _mock(["dev-manager", "test-manager"], b'{"module":{}}'),
                {"cluster_manager": "dev-manager"}) == "No clusters."


def test_get_cluster_no_cluster_name():
    assert _err(get_cluster, _mock(["dev-manager", "test-manager"], MOCK_CLUSTERS),
                {"cluster_manager": "dev-manager"}) == "cluster_name must be specified"


def test_get_cluster_unidentified_cluster():
    assert _err(get_cluster, _mock(["dev-manager", "test-manager"], MOCK_CLUSTERS),
                {"cluster_manager": "dev-manager", "cluster_name": "cluster_xyz"}) == \
        "A cluster named 'cluster_xyz', does not exist."


def test_get_manager_no_cluster_manager():
    assert _err(get_manager, _mock([])) == "No cluster managers."


def test_get_manager_missing_cluster_manager():
    assert _err(get_manager, _mock(["dev-manager", "beta-manager"])) == "cluster_manager must be specified"


def test_get_manager_not_exists():
    assert _err(get_manager, _mock(["dev-manager", "beta-manager"]), {"cluster_manager": "prod-cluster"}) == \
        "Selected cluster manager 'prod-cluster' does not exist."


def test_settings_do_not_leak_between_contexts():
    """The reference's global viper leaked non-interactive between tests."""
    a = make_ctx({"cluster_manager": "x"})
    b = make_ctx({}, non_interactive=False, answers=[])
    assert a.settings.non_interactive and not b.settings.non_interactive
    assert not b.is_set("cluster_manager")
    assert isinstance(a.out, io.StringIO)
