"""State document tests — port of ``state/state_test.go`` (9 tests) + extensions."""

import json

import pytest

from triton_kubernetes_amd.errors import StateError
from triton_kubernetes_amd.state import State, cluster_key_parts, node_key


def test_get():  # state_test.go:8
    st = State("GetState", b'{"config":{"triton":{"key":"55fd4s","url":"https://api.storage.com"}}}')
    assert st.get("config.triton.key") == "55fd4s"


def test_set_manager():  # state_test.go:20
    st = State("AddState", b"{}")
    st.set_manager({"field": "test"})
    assert st.get("module.cluster-manager.field") == "test"


def test_set_terraform_backend_config():  # state_test.go:36
    st = State("AddState", b"{}")
    st.set_terraform_backend_config("module.path.to.backend", {"field": "test"})
    assert st.get("module.path.to.backend.field") == "test"


def test_add_cluster():  # state_test.go:53
    st = State("AddState", b"{}")
    st.add_cluster("aws", "name", {"field": "test"})
    assert st.get("module.cluster_aws_name.field") == "test"


def test_add_node():  # state_test.go:69
    st = State("AddState", b"{}")
    st.add_node("cluster_aws_cluster-name", "node-name", {"field": "test"})
    assert st.get("module.node_aws_cluster-name_node-name.field") == "test"


def test_delete():  # state_test.go:86
    st = State("DelState", b'{"config":{"triton":{"key":"55fd4s","url":"https://api.storage.com"}}}')
    st.delete("config.triton.key")
    assert st.get("config.triton.key") == ""


def test_get_clusters():  # state_test.go:103
    st = State("ClusterState", b'''{"module":{"cluster_1":{"name":"dev_cluster"},
        "cluster_2":{"name":"beta_cluster"}, "cluster_3":{"name":"prod_cluster"}}}''')
    assert len(st.clusters()) == 3


NODES_DOC = b'''{"module":{
  "node_triton_dev-cluster_1":{"hostname":"dev-worker1"},
  "node_triton_dev-cluster_2":{"hostname":"dev-etcd1"},
  "node_triton_dev-cluster_3":{"hostname":"dev-control1"},
  "node_aws_dev-cluster_1":{"hostname":"dev-control2"},
  "node_aws_dev-cluster_2":{"hostname":"dev-control3"}}}'''


def test_get_nodes():  # state_test.go:127
    key = State("ClusterState", b'{"config":{"triton":{"key":"cluster_triton_dev-cluster"}}}').get("config.triton.key")
    assert len(State("NodeState", NODES_DOC).nodes(key)) == 3


def test_get_nodes_without_cloud_provider():  # state_test.go:158
    with pytest.raises(StateError) as exc:
        State("NodeState", NODES_DOC).nodes("cluster_dev-cluster")
    assert str(exc.value) == ("Could not get cluster key parts, cluster does not follow format "
                              "`cluster_{provider}_{clusterName}` 'cluster_dev-cluster'")


# --- extensions ---------------------------------------------------------------------------------
def test_bytes_is_go_marshalindent_compatible():
    st = State("x", b"{}")
    st.set_manager({"source": "a//b?ref=master", "name": "m", "pw": "<&>"})
    raw = st.bytes().decode()
    assert raw.startswith('{\n\t"module": {\n\t\t"cluster-manager": {')
    assert '"pw": "\\u003c\\u0026\\u003e"' in raw  # Go's HTML-safe escaping
    assert json.loads(raw)["module"]["cluster-manager"]["pw"] == "<&>"


def test_same_session_nodes_visible_q1():
    """Reference quirk Q1: nodes added in-session were invisible until re-parse."""
    st = State("x", b"{}")
    key = st.add_cluster("baremetal", "dev", {"name": "dev"})
    st.add_node(key, "dev-worker-1", {"hostname": "dev-worker-1"})
    assert st.clusters() == {"dev": key}
    assert st.nodes(key) == {"dev-worker-1": "node_baremetal_dev_dev-worker-1"}


def test_hostname_with_dot_does_not_corrupt_document():
    st = State("x", b"{}")
    key = st.add_cluster("baremetal", "dev", {"name": "dev"})
    st.add_node(key, "gpu.rack1", {"hostname": "gpu.rack1"})
    assert "node_baremetal_dev_gpu.rack1" in st.modules()
    assert st.nodes(key) == {"gpu.rack1": "node_baremetal_dev_gpu.rack1"}


def test_key_helpers_and_roundtrip():
    assert cluster_key_parts("cluster_aws_prod") == ("aws", "prod")
    assert node_key("cluster_aws_prod", "w-1") == "node_aws_prod_w-1"
    st = State("x", b"{}")
    st.set_terraform_backend_config("terraform.backend.local", {"path": "/p"})
    again = State("x", st.bytes())
    assert again.backend_block() == ("local", {"path": "/p"})
    with pytest.raises(StateError):
        st.delete("module.nope")
    with pytest.raises(StateError):
        State("bad", b"[1,2]")


def test_dumps_go_memo_matches_plain_encoding():
    from hypothesis import given, settings
    from hypothesis import strategies as st

    from triton_kubernetes_amd.utils.jsonenc import dumps_go, dumps_go_plain

    leaf = st.one_of(st.none(), st.booleans(), st.integers(), st.floats(allow_nan=False),
                     st.text(alphabet="ab<>& é\"\\\n", max_size=6))
    tree = st.recursive(leaf, lambda ch: st.one_of(st.lists(ch, max_size=3),
                                                   st.dictionaries(st.text("xyz<", max_size=3), ch, max_size=3)),
                        max_leaves=12)

    @settings(max_examples=200, deadline=None)
    @given(tree)
    def check(obj):
        for indent in ("\t", "  ", ""):
            assert dumps_go(obj, indent) == dumps_go_plain(obj, indent)
            assert dumps_go(obj, indent) == dumps_go_plain(obj, indent)  # memo hit

    check()
