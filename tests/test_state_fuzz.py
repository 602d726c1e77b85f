"""A manager's ``main.tf.json`` that is damaged -- not JSON, not an object, a ``module`` that
is not a map, a module block that is not an object, fields of the wrong type -- makes every
command end in an exit code and a message, never in a Python traceback (a document is
shared through Manta and edited by hand; Terraform refuses such documents with an error)."""

import io
import json
import os

import yaml
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from triton_kubernetes_amd.cli.main import run

ODD = st.sampled_from([None, 0, 7, True, [], ["a"], {}, {"a": 1}, "", "x", {"source": "x"}, {"name": 3},
                       {"hostname": None}])
GOOD = {"terraform": {"backend": {"local": {"path": "/nonexistent/tfstate"}}},
        "module": {"cluster-manager": {"source": "tk::terraform/modules/bare-metal-rancher?ref=v0.8.2", "name": "m",
                                       "host": "10.0.0.1"},
                   "cluster_baremetal_c": {"source": "tk::terraform/modules/bare-metal-rancher-k8s?ref=v0.8.2",
                                           "name": "c"},
                   "node_baremetal_c_w-1": {"source": "tk::terraform/modules/bare-metal-rancher-k8s-host?ref=v0.8.2",
                                            "hostname": "w-1"}}}
CMDS = [("get", "manager"), ("get", "cluster"), ("get", "nodes"), ("destroy", "cluster"), ("destroy", "node"),
        ("create", "node"), ("create", "cluster")]
CONFIG = {"backend_provider": "local", "cluster_manager": "m", "cluster_name": "c", "hostname": "w-1",
          "executor": "terraform", "terraform_binary": "/nonexistent/terraform", "rancher_host_label": "worker",
          "node_count": 1, "hosts": ["10.0.0.3"], "ssh_user": "u", "bastion_host": "", "key_path": "/nonexistent/k",
          "cluster_cloud_provider": "baremetal", "name": "c2", "k8s_version": "v1.31", "k8s_network_provider": "canal",
          "nodes": [{"rancher_host_label": "worker", "node_count": 1, "hostname": "w", "hosts": ["10.0.0.2"],
                     "ssh_user": "u", "bastion_host": "", "key_path": "/nonexistent/k"}]}


@st.composite
def documents(draw):
    kind = draw(st.sampled_from(["raw", "top", "module", "block", "field"]))
    if kind == "raw":
        return draw(st.sampled_from([b"not json", b"", b"{", b"\xff\xfe", b"[]", b"null", b"3"]))
    doc = json.loads(json.dumps(GOOD))
    if kind == "top":
        doc = draw(ODD)
    elif kind == "module":
        doc["module"] = draw(ODD)
    elif kind == "block":
        doc["module"][draw(st.sampled_from(sorted(GOOD["module"])))] = draw(ODD)
    else:
        key = draw(st.sampled_from(sorted(GOOD["module"])))
        doc["module"][key][draw(st.sampled_from(sorted(GOOD["module"][key])))] = draw(ODD)
    return json.dumps(doc).encode()


@settings(max_examples=120, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(documents(), st.sampled_from(CMDS))
def test_a_damaged_document_never_ends_in_a_traceback(tk_home, tmp_path, raw, cmd):
    d = tk_home / ".triton-kubernetes" / "m"
    d.mkdir(parents=True, exist_ok=True)
    (d / "main.tf.json").write_bytes(raw)
    cfg = os.path.join(str(tmp_path), "c.yaml")
    with open(cfg, "w", encoding="utf-8") as fh:
        fh.write(yaml.safe_dump(CONFIG))
    assert isinstance(run(["--non-interactive", "--config", cfg, *cmd], out=io.StringIO()), int)
