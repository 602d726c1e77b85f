"""The CLI in non-interactive mode over generated silent-install files: whatever a value's
type or text (null, numbers, lists, maps, empty, non-ASCII, path-like), every command ends
in an exit code and a message -- a refusal or a result -- never in a Python traceback.  The
files start from valid manager / cluster / node / get / destroy documents and have one to
three values replaced (the reference's viper coerced types silently; this CLI refuses or
converts them)."""

import io
import os

import pytest
import yaml
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from triton_kubernetes_amd.cli.main import run

VALUES = st.sampled_from([None, 0, 7, -1, True, [], ["a"], {}, {"a": 1}, "", "x", 3.5, "10.0.0.1", "a b", "ü",
                          "-", "../x", "1e9", "99999999999999999999"])
MANAGER = {"backend_provider": "local", "name": "m", "manager_cloud_provider": "baremetal", "host": "10.0.0.1",
           "ssh_user": "u", "bastion_host": "", "key_path": "/nonexistent/k", "rancher_admin_password": "long-enough-pw",
           "executor": "terraform", "terraform_binary": "/nonexistent/terraform"}
NODE = {"rancher_host_label": "worker", "node_count": 1, "hostname": "w", "hosts": ["10.0.0.2"], "ssh_user": "u",
        "bastion_host": "", "key_path": "/nonexistent/k"}
CLUSTER = {"backend_provider": "local", "cluster_manager": "m", "cluster_cloud_provider": "baremetal", "name": "c",
           "k8s_version": "v1.31", "k8s_network_provider": "canal", "executor": "terraform",
           "terraform_binary": "/nonexistent/terraform", "nodes": [NODE]}
DOCS = {("create", "manager"): MANAGER, ("create", "cluster"): CLUSTER,
        ("create", "node"): dict({k: v for k, v in CLUSTER.items() if k != "nodes"}, cluster_name="c", **NODE),
        ("get", "manager"): {"backend_provider": "local", "cluster_manager": "m"},
        ("get", "cluster"): {"backend_provider": "local", "cluster_manager": "m", "cluster_name": "c"},
        ("destroy", "cluster"): {"backend_provider": "local", "cluster_manager": "m", "cluster_name": "c",
                                 "executor": "terraform", "terraform_binary": "/nonexistent/terraform"}}


@st.composite
def configs(draw):
    cmd = draw(st.sampled_from(sorted(DOCS)))
    doc = dict(DOCS[cmd])
    for key in draw(st.lists(st.sampled_from(sorted(doc)), min_size=1, max_size=3, unique=True)):
        doc[key] = draw(VALUES)
    if isinstance(doc.get("nodes"), list) and doc["nodes"] and draw(st.booleans()):
        node = dict(NODE)
        node[draw(st.sampled_from(sorted(NODE)))] = draw(VALUES)
        doc["nodes"] = [node]
    return cmd, doc


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(configs())
def test_no_generated_config_ends_in_a_traceback(tk_home, tmp_path, case):
    cmd, doc = case
    path = os.path.join(str(tmp_path), "c.yaml")
    with open(path, "w", encoding="utf-8") as fh:
        fh.write(yaml.safe_dump(doc))
    code = run(["--non-interactive", "--config", path, *cmd], out=io.StringIO())
    assert isinstance(code, int)


@pytest.mark.parametrize("content,why", [
    ("a: [\n", "is not valid YAML"),
    ("a: !!python/object:os.system x\n", "is not valid YAML"),  # safe_load: no object construction
    ("\t- bad indent\n", "is not valid YAML"),
    ("- a\n- b\n", "must contain a mapping at the top level"),
    (None, "No such file or directory"),
])
def test_config_files_that_cannot_be_used_are_refusals(tk_home, tmp_path, content, why):
    path = tmp_path / "c.yaml"
    if content is not None:
        path.write_text(content)
    out = io.StringIO()
    assert run(["--non-interactive", "--config", str(path), "get", "manager"], out=out) == 1
    assert why in out.getvalue()


OTHER_CMDS = [("wait", "cluster"), ("backup", "cluster"), ("restore", "cluster"), ("userdata", "node"),
              ("migrate", "manager"), ("credentials", "node"), ("health", "cluster"), ("drain", "node"),
              ("upgrade", "cluster"), ("cordon", "node"), ("uncordon", "node"), ("forget", "host-key"),
              ("get", "scrape-config")]
OTHER_KEYS = ["cluster_manager", "cluster_name", "hostname", "namespace", "namespaces", "backup_target", "backup_name",
              "s3_bucket", "health_taint", "max_uncorrectable", "drain_timeout", "force", "k8s_version", "source_url",
              "migrate_drop_unknown", "host", "wait_timeout", "node_exporter_port", "rccl_gate_max_mib",
              "host_retry_backoff", "executor"]
MANAGER_DOC = {"module": {
    "cluster-manager": {"source": "tk::terraform/modules/bare-metal-rancher?ref=v0.8.2", "name": "m", "host": "10.0.0.1"},
    "cluster_baremetal_c": {"source": "tk::terraform/modules/bare-metal-rancher-k8s?ref=v0.8.2", "name": "c"},
    "node_baremetal_c_w-1": {"source": "tk::terraform/modules/bare-metal-rancher-k8s-host?ref=v0.8.2",
                             "hostname": "w-1"}}}


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(st.sampled_from(OTHER_CMDS), st.dictionaries(st.sampled_from(OTHER_KEYS), VALUES, max_size=4))
def test_day2_commands_over_generated_settings_never_end_in_a_traceback(tk_home, tmp_path, cmd, extra):
    """The day-2 commands (wait, backup, restore, userdata, migrate, credentials, health,
    drain, upgrade, cordon, forget, scrape-config) against a manager document that was never
    applied, with generated values for their settings: numbers that are not numbers, a
    ``source_url`` with no modules behind it, a node whose block lacks the cluster's
    outputs."""
    import json

    d = tk_home / ".triton-kubernetes" / "m"
    d.mkdir(parents=True, exist_ok=True)
    (d / "main.tf.json").write_text(json.dumps(MANAGER_DOC))
    doc = {"backend_provider": "local", "cluster_manager": "m", "cluster_name": "c", "hostname": "w-1",
           "executor": "terraform", "terraform_binary": "/nonexistent/terraform", "wait_timeout": 1}
    doc.update(extra)
    path = os.path.join(str(tmp_path), "c.yaml")
    with open(path, "w", encoding="utf-8") as fh:
        fh.write(yaml.safe_dump(doc))
    try:
        code = run(["--non-interactive", "--config", path, *cmd], out=io.StringIO())
    except SystemExit as exc:  # argparse's own refusals
        code = exc.code
    assert isinstance(code, int)
