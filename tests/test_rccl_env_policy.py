"""What a node's RCCL environment may hold (``parallel/rccl_env.py:env_problems``).

``/etc/rccl/rccl.env`` is loaded as root by the node agent's service (``EnvironmentFile=``),
sourced by the Terraform host script and applied by the agent at start.  A setting that
names a library (``NCCL_NET_PLUGIN``, ``HSA_TOOLS_LIB``, ``RCCL_ROCR_PATH``), a file to write
(``NCCL_DEBUG_FILE``, ``HSA_COREDUMP_PATTERN``), or a value carrying a newline or quote
(a line of its own: ``LD_PRELOAD=...``) would run code there.  Each entry point refuses it:
the config check, the file renderer, the agent's plan check, the agent's start, and the
host module's variable validation (HCL input check and planner).
"""

import os

import pytest

from triton_kubernetes_amd.parallel.rccl_env import (default_rccl_env, env_problems, parse_env_file,
                                                      render_env_file, site_env_from_topology)

DENIED_KEYS = ["NCCL_NET_PLUGIN", "NCCL_TUNER_PLUGIN", "NCCL_PROFILER_PLUGIN", "HSA_TOOLS_LIB", "RCCL_ROCR_PATH",
               "NCCL_DEBUG_FILE", "NCCL_CONF_FILE", "NCCL_TOPO_FILE", "NCCL_TOPO_DUMP_FILE",
               "NCCL_GRAPH_DUMP_FILE_RANK",
               "HSA_COREDUMP_PATTERN", "HSA_MODEL_LIB", "HSA_MODEL_MEMFILE", "RCCL_REPLAY_FILE", "HSA_REV_COPY_DIR"]
BAD_VALUES = ["WARN\nLD_PRELOAD=/tmp/x.so", 'WARN"', "$(id)", "`id`", "/tmp/evil.so", "lib/evil.so", "a b",
              "x" * 300, "WARN\\"]
GOOD = {"NCCL_DEBUG": "WARN", "NCCL_DEBUG_SUBSYS": "INIT,NET", "NCCL_SOCKET_IFNAME": "^docker,lo",
        "NCCL_IB_HCA": "=mlx5_0:1,mlx5_1:1", "NCCL_IB_GID_INDEX": "3", "NCCL_IB_ADDR_RANGE": "10.0.0.0/8",
        "NCCL_P2P_DIRECT_DISABLE": "1", "NCCL_IB_DATA_DIRECT": "0", "RCCL_MSCCLPP_ENABLE": "0",
        "HSA_FORCE_FINE_GRAIN_PCIE": "1", "NCCL_NET_GDR_LEVEL": "PHB", "NCCL_MIN_NCHANNELS": "32"}


def test_defaults_site_settings_and_common_overrides_are_accepted():
    assert env_problems(default_rccl_env()) == []
    topo = {"nics": [{"name": "mlx5_0", "port": 1, "link_layer": "Ethernet", "roce_v2_gid_index": 3},
                     {"name": "bnxt_re1", "port": 1, "link_layer": "Ethernet", "roce_v2_gid_index": 3}]}
    assert env_problems(site_env_from_topology(topo)) == []
    assert env_problems(GOOD) == []
    assert parse_env_file(render_env_file(GOOD)) == GOOD


@pytest.mark.parametrize("key", DENIED_KEYS)
def test_settings_naming_code_or_files_are_refused(key):
    bad = env_problems({key: "x"})
    assert len(bad) == 1 and "library, plugin, file or path" in bad[0], bad
    with pytest.raises(ValueError):
        render_env_file({key: "x"})


@pytest.mark.parametrize("key", ["LD_PRELOAD", "PATH", "nccl_debug", "NCCL_DEBUG=1", "NCCL-DEBUG", "MSCCL_ALGO_DIR"])
def test_keys_outside_the_rccl_namespaces_are_refused(key):
    assert "only NCCL_*, RCCL_* and HSA_*" in env_problems({key: "1"})[0]


@pytest.mark.parametrize("value", BAD_VALUES)
def test_values_that_are_not_plain_tokens_are_refused(value):
    bad = env_problems({"NCCL_DEBUG": value})
    assert bad and "comma list" in bad[0], (value, bad)
    with pytest.raises(ValueError):  # the file never gets a line of its own from a value
        render_env_file({"NCCL_DEBUG": value})


def test_config_refuses_a_bad_rccl_env():
    from triton_kubernetes_amd.config import Context, Settings
    from triton_kubernetes_amd.errors import ConfigError
    from triton_kubernetes_amd.models.baremetal import _mi355x_fields

    def cfg(env):
        return _mi355x_fields(Context(settings=Settings({"non-interactive": True, "gpu": "mi355x", "gpu_count": "8",
                                                         "rccl_env": env}, env={})))

    assert cfg({"NCCL_SOCKET_IFNAME": "=bond0"})["rccl_env"]["NCCL_SOCKET_IFNAME"] == "=bond0"
    with pytest.raises(ConfigError, match="NCCL_NET_PLUGIN"):
        cfg({"NCCL_NET_PLUGIN": "/tmp/evil.so"})
    with pytest.raises(ConfigError, match="comma list"):
        cfg({"NCCL_DEBUG": "WARN\nLD_PRELOAD=/tmp/x.so"})
    with pytest.raises(ConfigError, match="map"):
        cfg("NCCL_DEBUG=WARN")


def test_agent_refuses_a_plan_whose_rccl_env_names_a_library(tmp_path):
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.plan import BootstrapPlan, Step

    agent = NodeAgent(name="n", mode="sim", devices=[], root=str(tmp_path))
    try:
        for env in ({"HSA_TOOLS_LIB": "libevil.so"}, {"LD_PRELOAD": "x"}, {"NCCL_DEBUG": "WARN\nLD_PRELOAD=x"}):
            plan = BootstrapPlan(hostname="n", role="worker", rancher_url="https://r", token="t", ca_checksum="c",
                                 steps=[Step("rccl_env", "rccl_env", "", {"env": env})])
            assert agent.refusals(plan), env
            with pytest.raises(PermissionError):
                agent.run_plan(plan)
            assert not (tmp_path / "etc/rccl/rccl.env").exists()
        ok = BootstrapPlan(hostname="n", role="worker", rancher_url="https://r", token="t", ca_checksum="c",
                           steps=[Step("rccl_env", "rccl_env", "", {"env": {"NCCL_DEBUG": "WARN"}})])
        assert agent.refusals(ok) == []
    finally:
        agent.stop()


def test_agent_start_skips_file_settings_it_may_not_apply(tmp_path, monkeypatch):
    """A file written by hand or by an older release: the agent applies the plain settings
    and skips the rest (the unit's ``EnvironmentFile=`` is the operator's own business)."""
    from triton_kubernetes_amd.node.agent import NodeAgent

    env = {k: v for k, v in os.environ.items() if not k.startswith(("NCCL_", "RCCL_", "HSA_"))}
    monkeypatch.setattr(os, "environ", env)
    (tmp_path / "etc/rccl").mkdir(parents=True)
    (tmp_path / "etc/rccl/rccl.env").write_text('NCCL_DEBUG="WARN"\nNCCL_NET_PLUGIN="evil"\nHSA_TOOLS_LIB="x.so"\n'
                                                'NCCL_SOCKET_IFNAME="/tmp/x"\n')
    agent = NodeAgent(name="n", mode="sim", devices=[], root=str(tmp_path))
    try:
        agent.rccl_env_applied = agent.apply_node_rccl_env()
        assert agent.rccl_env_applied == {"NCCL_DEBUG": "WARN"}
        assert sorted(agent.rccl_env_skipped) == ["HSA_TOOLS_LIB", "NCCL_NET_PLUGIN", "NCCL_SOCKET_IFNAME"]
        assert "NCCL_NET_PLUGIN" not in env and "HSA_TOOLS_LIB" not in env
        # and the operator can see it on the agent's API
        import json
        import urllib.request

        url = agent.serve("127.0.0.1")
        req = urllib.request.Request(url + "/v1/info", headers={"X-TK-Agent-Token": agent.token})
        info = json.loads(urllib.request.urlopen(req, timeout=10).read())
        assert info["rccl_env_applied"] == ["NCCL_DEBUG"]
        assert sorted(info["rccl_env_skipped"]) == ["HSA_TOOLS_LIB", "NCCL_NET_PLUGIN", "NCCL_SOCKET_IFNAME"]
    finally:
        agent.stop()


def test_host_module_validates_rccl_env():
    """The same rules as the host module's variable validation: the HCL input check and the
    planner refuse what Terraform would ("Invalid value for variable")."""
    from triton_kubernetes_amd.terraform import hcl
    from triton_kubernetes_amd.terraform.catalog import MODULES_DIR
    from triton_kubernetes_amd.terraform.plan import plan_module

    mod = os.path.join(MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host")
    base = {"hostname": "g", "rancher_api_url": "https://r", "rancher_cluster_registration_token": "t",
            "rancher_cluster_ca_checksum": "c", "rancher_host_labels": {"worker": "true"}, "host": "10.0.0.9"}
    good = dict(base, rccl_env=dict(GOOD))
    assert not [p for p in hcl.check_inputs(mod, good) if "rccl_env" in p]
    assert not [e for e in plan_module(mod, good, check_files=False).errors if "Invalid value" in e]
    for bad in ({"NCCL_NET_PLUGIN": "x"}, {"HSA_TOOLS_LIB": "x"}, {"LD_PRELOAD": "x"},
                {"NCCL_DEBUG": "WARN\nLD_PRELOAD=/tmp/x.so"}, {"NCCL_DEBUG": "$(id)"}, {"NCCL_DEBUG": "/tmp/x"}):
        inputs = dict(base, rccl_env=bad)
        problems = hcl.check_inputs(mod, inputs)
        assert any("rccl_env" in p for p in problems), (bad, problems)
        errors = plan_module(mod, inputs, check_files=False).errors
        assert any("Invalid value for variable 'rccl_env'" in e for e in errors), (bad, errors)


def test_agent_refuses_a_metrics_step_outside_an_absolute_directory(tmp_path):
    """The metrics textfile is written by the agent as root: its directory is checked on the
    node as at create (an absolute path without "..")."""
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.plan import BootstrapPlan, Step

    agent = NodeAgent(name="n", mode="sim", devices=[], root=str(tmp_path))
    try:
        def plan(d):
            return BootstrapPlan(hostname="n", role="worker", rancher_url="https://r", token="t", ca_checksum="c",
                                 steps=[Step("gpu_metrics", "gpu_metrics", "", {"dir": d})])

        for bad in ("relative/dir", "/var/../etc", "", None):
            assert agent.refusals(plan(bad)), bad
        assert agent.refusals(plan("/var/lib/node_exporter/textfile")) == []
    finally:
        agent.stop()


def test_numeric_gpu_settings_are_written_plainly_and_validated():
    """The link floors and the busbw gate go into the host script's argv: the config writes
    them as plain numbers (the form the module's validation accepts) and refuses the rest."""
    from triton_kubernetes_amd.config import Context, Settings
    from triton_kubernetes_amd.errors import ConfigError
    from triton_kubernetes_amd.models.baremetal import _mi355x_fields
    from triton_kubernetes_amd.terraform import hcl
    from triton_kubernetes_amd.terraform.catalog import MODULES_DIR

    def cfg(**kw):
        return _mi355x_fields(Context(settings=Settings(dict({"non-interactive": True, "gpu": "mi355x",
                                                              "gpu_count": "8"}, **kw), env={})))

    got = cfg(rccl_min_busbw="1e3", gpu_link_min_gbps="38.50", gpu_link_min_frac=".5")
    assert (got["rccl_min_busbw"], got["gpu_link_min_gbps"], got["gpu_link_min_frac"]) == ("1000", "38.5", "0.5")
    for key, bad in (("rccl_min_busbw", "nan"), ("rccl_min_busbw", "-1"), ("gpu_link_min_gbps", "inf"),
                     ("gpu_link_min_frac", "1.5"), ("gpu_link_min_gbps", "1; id")):
        with pytest.raises(ConfigError, match=key):
            cfg(**{key: bad})
    mod = os.path.join(MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host")
    base = {"hostname": "g", "rancher_api_url": "https://r", "rancher_cluster_registration_token": "t",
            "rancher_cluster_ca_checksum": "c", "rancher_host_labels": {"worker": "true"}, "host": "10.0.0.9"}
    assert not [p for p in hcl.check_inputs(mod, dict(base, rccl_min_busbw=got["rccl_min_busbw"],
                                                      gpu_link_min_gbps=got["gpu_link_min_gbps"],
                                                      gpu_link_min_frac=got["gpu_link_min_frac"])) if "min" in p]
    for key, bad in (("rccl_min_busbw", "1; id"), ("gpu_link_min_gbps", "-3"), ("gpu_link_min_frac", "2")):
        assert any(key in p for p in hcl.check_inputs(mod, dict(base, **{key: bad}))), key


def test_discovered_ports_with_odd_names_are_left_to_rccl():
    topo = {"nics": [{"name": "mlx5_0", "port": 1, "link_layer": "InfiniBand"},
                     {"name": "x\nLD_PRELOAD=/tmp/y", "port": 1, "link_layer": "InfiniBand"},
                     {"name": "mlx5_1", "port": 0, "link_layer": "InfiniBand"}]}
    env = site_env_from_topology(topo)
    assert env == {"NCCL_IB_HCA": "=mlx5_0:1"} and env_problems(env) == []
