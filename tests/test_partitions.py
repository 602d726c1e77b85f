"""MI355X partition modes (``node/partition.py``).

Fixture sysfs trees for an SPX/NPS1 node (8 GPUs) and a CPX/NPS2 node (8 GPUs x 8 compute
partitions = 64 KFD nodes / render nodes; only each GPU's first partition carries the
``current_*_partition`` files, its partitions share the PCI function) drive the labeller
(native and Python), preflight (shell and agent), the readiness waiter's expectations and
the webhook's xGMI placement.
"""

import json
import os
import subprocess

import pytest

from triton_kubernetes_amd.errors import ConfigError
from triton_kubernetes_amd.node import partition
from triton_kubernetes_amd.node.labels import labels_from_topology
from triton_kubernetes_amd.ops import topo
from triton_kubernetes_amd.ops.native import NativeUnavailable

VRAM = 294896 << 20


def _write(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        fh.write(text)


def make_tree(root, ngpu=8, compute="SPX", memory="NPS1"):
    parts = partition.COMPUTE_PARTITIONS[compute.lower()]
    mparts = partition.MEMORY_PARTITIONS[memory.lower()]
    nodes = os.path.join(root, "sys/class/kfd/kfd/topology/nodes")
    _write(f"{nodes}/0/properties", "cpu_cores_count 96\nsimd_count 0\nmem_banks_count 1\n")
    _write(os.path.join(root, "opt/rocm/.info/version"), "7.2.0-43\n")
    kfd = 0
    for g in range(ngpu):
        for p in range(parts):
            kfd += 1
            minor = 128 + (kfd - 1)
            props = {"cpu_cores_count": 0, "simd_count": 1024 // parts, "simd_per_cu": 4, "gfx_target_version": 90500,
                     "vendor_id": 4098, "device_id": 0x75A3, "location_id": (0x05 + 0x10 * g) << 8, "domain": 0,
                     "drm_render_minor": minor, "hive_id": 0x9CD4905654BB148F, "unique_id": 0x7D74AFAB5AA15265 + kfd,
                     "local_mem_size": 0}
            _write(f"{nodes}/{kfd}/properties", "".join(f"{k} {v}\n" for k, v in props.items()))
            _write(f"{nodes}/{kfd}/name", "gfx950\n")
            _write(f"{nodes}/{kfd}/mem_banks/0/properties",
                   f"heap_type 1\nsize_in_bytes {VRAM // mparts}\nwidth 8192\n")
            # xGMI: each GPU's first partition to the other GPUs' first partitions (SPX: the full mesh)
            links = [(0, 2)]
            if p == 0:
                links += [(1 + h * parts, 11) for h in range(ngpu) if h != g]
            for n, (to, typ) in enumerate(links):
                _write(f"{nodes}/{kfd}/io_links/{n}/properties", f"type {typ}\nnode_from {kfd}\nnode_to {to}\n"
                                                                 "weight 15\n")
            dev = os.path.join(root, f"sys/class/drm/renderD{minor}/device")
            if p == 0:  # the PCI function's own attributes; partitions 1.. are xcp platform devices
                _write(f"{dev}/current_compute_partition", compute + "\n")
                _write(f"{dev}/current_memory_partition", memory + "\n")
                _write(f"{dev}/mem_info_vram_total", f"{VRAM}\n")
                for attr, val in (("current_link_width", "16"), ("max_link_width", "16"),
                                  ("vbios_version", "113-M355-01-1K1-020F"),
                                  ("hwmon/hwmon3/power1_cap", "1400000000"),
                                  ("hwmon/hwmon3/power1_cap_default", "1400000000"),
                                  ("current_link_speed", "32.0 GT/s PCIe"), ("max_link_speed", "32.0 GT/s PCIe")):
                    _write(f"{dev}/{attr}", val + "\n")
            else:
                os.makedirs(dev, exist_ok=True)
            _write(os.path.join(root, f"dev/dri/renderD{minor}"), "")
    _write(os.path.join(root, "sys/module/amdgpu/version"), "6.12.12\n")
    return root


@pytest.fixture(scope="module")
def native_ok():
    try:
        topo.native_topology("sysfs", "/nonexistent")
    except NativeUnavailable as exc:
        pytest.skip(f"native labeller not buildable here: {exc}")


@pytest.fixture
def spx(tmp_path):
    return make_tree(str(tmp_path / "spx"))


@pytest.fixture
def cpx(tmp_path):
    return make_tree(str(tmp_path / "cpx"), compute="CPX", memory="NPS2")


def test_modes_policy():
    assert partition.normalize(None, None) == ("spx", "nps1")
    assert partition.normalize("CPX", "NPS2") == ("cpx", "nps2")
    with pytest.raises(ConfigError, match="gpu_compute_partition must be one of spx, dpx, qpx, cpx"):
        partition.normalize("tpx", "nps1")
    with pytest.raises(ConfigError, match="needs at least 2 compute partitions"):
        partition.normalize("spx", "nps2")
    assert partition.logical_gpus({"gpu_count": 8, "gpu_compute_partition": "cpx"}) == 64
    assert partition.logical_gpus({"gpu_count": "2"}) == 2
    assert partition.compute_share("qpx") == 0.25 and partition.memory_share("cpx", "nps2") == 0.25
    from triton_kubernetes_amd.ops.probe import Thresholds

    th = Thresholds.for_partition("cpx", "nps2")
    assert th.share == 0.125 and th.mem_share == 0.25 and th.min_cus == 32


def test_labeller_spx_nps1(spx, native_ok):
    doc = topo.native_topology("sysfs", spx)
    native = topo.native_labels("sysfs", spx)
    assert native == labels_from_topology(doc)
    assert native["amd.com/gpu.count"] == "8" and native["amd.com/gpu.logical-count"] == "8"
    assert native["amd.com/gpu.partitions-per-gpu"] == "1" and native["amd.com/gpu.cu-count"] == "256"
    assert native["amd.com/gpu.compute-partition"] == "spx" and native["amd.com/gpu.memory-partition"] == "nps1"
    assert native["amd.com/xgmi.fully-connected"] == "true"
    assert partition.physical_count(doc) == 8


def test_labeller_cpx_nps2(cpx, native_ok):
    doc = topo.native_topology("sysfs", cpx)
    assert len(doc["gpus"]) == 64 and partition.physical_count(doc) == 8
    native = topo.native_labels("sysfs", cpx)
    assert native == labels_from_topology(doc)
    assert native["amd.com/gpu.count"] == "8" and native["amd.com/gpu.logical-count"] == "64"
    assert native["amd.com/gpu.partitions-per-gpu"] == "8" and native["amd.com/gpu.cu-count"] == "32"
    assert native["amd.com/gpu.compute-partition"] == "cpx" and native["amd.com/gpu.memory-partition"] == "nps2"
    # a partition is not a whole GPU with its own links: no full-mesh claim
    assert native["amd.com/xgmi.fully-connected"] == "false"


def test_preflight_modes_from_sysfs_and_topology(spx, cpx, native_ok):
    assert partition.sysfs_modes(spx) == ("spx", "nps1")
    assert partition.sysfs_modes(cpx) == ("cpx", "nps2")
    assert partition.topology_modes(topo.native_topology("sysfs", cpx)) == ("cpx", "nps2")
    assert partition.check(("spx", "nps1"), ("spx", "nps1")) is None
    msg = partition.check(("spx", "nps1"), ("cpx", "nps2"))
    assert "compute partition is CPX, the cluster expects SPX" in msg and "memory partition is NPS2" in msg
    assert partition.check(("cpx", "nps2"), (None, None)) is None  # not reported: not held against it


@pytest.mark.parametrize("cfg_modes,tree,ok", [(("spx", "nps1"), "spx", True), (("cpx", "nps2"), "cpx", True),
                                               (("spx", "nps1"), "cpx", False), (("cpx", "nps2"), "spx", False)])
def test_shell_preflight_on_fixture_trees(tmp_path, cfg_modes, tree, ok):
    """The rendered preflight step (SSH path) against a fixture tree: render-node count of
    the logical GPUs and the sysfs partition modes."""
    from triton_kubernetes_amd.node.plan import build_host_plan

    root = make_tree(str(tmp_path / tree), compute=tree.upper(), memory="NPS2" if tree == "cpx" else "NPS1")
    cfg = {"hostname": "g", "rancher_host_labels": {"worker": "true"}, "gpu_count": 8, "gpu_burnin": "off",
           "gpu_compute_partition": cfg_modes[0], "gpu_memory_partition": cfg_modes[1]}
    plan = build_host_plan(cfg, "https://r", "t", "s", mi355x=True)
    step = next(s for s in plan.steps if s.name == "gpu_preflight")
    body = (step.shell.replace("lsmod | grep '^amdgpu' >/dev/null ||", "true ||").replace("test -c /dev/kfd", "true")
            .replace("/dev/", f"{root}/dev/").replace("/sys/", f"{root}/sys/").replace("/etc/", f"{root}/etc/")
            .replace("sudo ", ""))
    bindir = tmp_path / "bin"
    bindir.mkdir(exist_ok=True)
    (bindir / "usermod").write_text("#!/bin/sh\nexit 0\n")
    (bindir / "usermod").chmod(0o755)
    p = subprocess.run(["bash", "-c", "f() {\n" + body + "\n}\nf"], capture_output=True, text=True,
                       env=dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}"))
    assert (p.returncode == 0) == ok, p.stderr
    if not ok:
        assert "partition is" in p.stderr or "expected 64 GPUs" in p.stderr


def test_agent_preflight_checks_the_modes(cpx, native_ok, tmp_path):
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.plan import build_host_plan

    doc = topo.native_topology("sysfs", cpx)
    agent = NodeAgent(name="n", mode="sim", devices=list(range(64)), token="t" * 24, root=str(tmp_path / "r"),
                      topology_override=doc, burnin_override=lambda d, lvl: {"ok": True})
    try:
        base = {"hostname": "g", "rancher_host_labels": {"worker": "true"}, "gpu_count": 8, "gpu_burnin": "quick"}
        good = agent.run_plan(build_host_plan(dict(base, gpu_compute_partition="cpx", gpu_memory_partition="nps2"),
                                              "http://127.0.0.1:9", "t", "s", mi355x=True))
        pre = next(s for s in good["steps"] if s["name"] == "gpu_preflight")
        assert pre["ok"] and pre["detail"]["partition"] == {"compute": "cpx", "memory": "nps2"}
        assert pre["detail"]["gpus"] == 64
        bad = agent.run_plan(build_host_plan(base, "http://127.0.0.1:9", "t", "s", mi355x=True))
        assert not bad["ok"] and "compute partition is CPX, the cluster expects SPX" in bad["error"]
    finally:
        agent.stop()


def test_waiter_expects_logical_gpus():
    from triton_kubernetes_amd.backend import MemoryBackend
    from triton_kubernetes_amd.models.baremetal import addons_key
    from triton_kubernetes_amd.readiness.waiter import spec_from_state
    from triton_kubernetes_amd.state import State
    from triton_kubernetes_amd.terraform.catalog import MODULES_DIR, module_source

    st = State("m", {})
    st.set_manager({"source": module_source(MODULES_DIR, "bare-metal-rancher", "")})
    key = st.add_cluster("baremetal", "c", {"source": module_source(MODULES_DIR, "bare-metal-rancher-k8s", ""),
                                            "name": "c"})
    st.set_module(addons_key("c"), {"source": module_source(MODULES_DIR, "rancher-k8s-mi355x-addons", "")})
    for i, (c, m) in enumerate((("cpx", "nps2"), ("spx", "nps1"))):
        st.add_node(key, f"g-{i}", {"source": module_source(MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host", ""),
                                    "hostname": f"g-{i}", "host": f"agent+http://h{i}:1", "gpu_count": 8,
                                    "gpu_compute_partition": c, "gpu_memory_partition": m})
    be = MemoryBackend()
    be.write_tfstate("m", json.dumps({"module_outputs": {
        "cluster-manager": {"rancher_url": "http://r", "rancher_access_key": "a", "rancher_secret_key": "s"},
        key: {"rancher_cluster_id": "c-1"}}}).encode())
    _, spec = spec_from_state(st, be, key, rccl_gate=True)
    assert spec.gpu_nodes == {"g-0": 64, "g-1": 8}
    assert spec.rccl_ndev == [64, 8]


def _node_matches(affinity, labels):
    """Required node affinity (ORed terms of ANDed In expressions) against node labels."""
    req = ((affinity or {}).get("nodeAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution")
    if not req:
        return True
    return any(all(labels.get(e["key"]) in e["values"] for e in t.get("matchExpressions") or [])
               for t in req["nodeSelectorTerms"])


def test_webhook_placement_keeps_multi_gpu_pods_off_partitioned_nodes(spx, cpx, native_ok):
    from triton_kubernetes_amd.k8s import webhook

    spx_labels = topo.native_labels("sysfs", spx)
    cpx_labels = topo.native_labels("sysfs", cpx)

    def pod(gpus):
        return {"metadata": {"name": "p"}, "spec": {"containers": [{"name": "c", "image": "x", "resources": {
            "limits": {"amd.com/gpu": str(gpus)}}}]}}

    for gpus, on_spx, on_cpx in ((8, True, False), (2, True, False), (1, True, True)):
        p = pod(gpus)
        out = webhook.apply_patch(p, webhook.patch_for_pod(p, {}))
        aff = out["spec"].get("affinity")
        assert _node_matches(aff, spx_labels) is on_spx, gpus
        assert _node_matches(aff, cpx_labels) is on_cpx, gpus


def test_provider_and_module_accept_the_modes():
    from triton_kubernetes_amd.models.baremetal import _mi355x_fields
    from triton_kubernetes_amd.terraform import hcl
    from triton_kubernetes_amd.terraform.catalog import MODULES_DIR

    from helpers import make_ctx

    out = _mi355x_fields(make_ctx({"gpu_compute_partition": "CPX", "gpu_memory_partition": "nps2"}))
    assert out["gpu_compute_partition"] == "cpx" and out["gpu_memory_partition"] == "nps2"
    assert "gpu_compute_partition" not in _mi355x_fields(make_ctx({}))  # module defaults: spx / nps1
    with pytest.raises(ConfigError):
        _mi355x_fields(make_ctx({"gpu_compute_partition": "spx", "gpu_memory_partition": "nps2"}))
    mod = os.path.join(MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host")
    assert hcl.check_inputs(mod, {"gpu_compute_partition": "cpx", "gpu_memory_partition": "nps2", "host": "h",
                                  "hostname": "h", "rancher_api_url": "https://r",
                                  "rancher_cluster_registration_token": "t",
                                  "rancher_cluster_ca_checksum": "c", "rancher_host_labels": {"worker": "true"}}) == []
    assert hcl.check_inputs(mod, {"gpu_compute_partition": "tpx"})


def test_shell_preflight_without_render_nodes_says_so(tmp_path):
    """Under the script's ``set -euo pipefail``, ``ls renderD* | wc -l`` fails when there is
    no render node; the count must still come out as 0 and the step name the problem."""
    import glob

    from triton_kubernetes_amd.node.plan import build_host_plan

    root = make_tree(str(tmp_path / "none"))
    for f in glob.glob(f"{root}/dev/dri/renderD*"):
        os.remove(f)
    cfg = {"hostname": "g", "rancher_host_labels": {"worker": "true"}, "gpu_count": 8, "gpu_burnin": "off"}
    step = next(s for s in build_host_plan(cfg, "https://r", "t", "s", mi355x=True).steps if s.name == "gpu_preflight")
    body = (step.shell.replace("lsmod | grep '^amdgpu' >/dev/null ||", "true ||").replace("test -c /dev/kfd", "true")
            .replace("/dev/", f"{root}/dev/").replace("/sys/", f"{root}/sys/").replace("/etc/", f"{root}/etc/")
            .replace("sudo ", ""))
    p = subprocess.run(["bash", "-c", "set -euo pipefail\nf() {\n" + body + "\n}\n( set -e; f )"], capture_output=True,
                       text=True)
    assert p.returncode == 1 and "found 0 render nodes" in p.stderr, (p.returncode, p.stderr)
