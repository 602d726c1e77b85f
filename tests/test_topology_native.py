"""Native labeller (csrc/tk_topo.cpp) sysfs collector against a fixture tree — runs on CPU.

The tree mimics an 8xMI355X node: KFD topology (one CPU node + 8 GPU nodes, a
full xGMI mesh as io_links type 11) and the DRM device attributes the
collector joins in.  The native labels must equal the Python spec
(node/labels.py) applied to the native JSON.
"""

import json
import os
import subprocess

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from triton_kubernetes_amd.node.labels import labels_from_topology
from triton_kubernetes_amd.ops import topo
from triton_kubernetes_amd.ops.native import NativeUnavailable, executable

VRAM = 294896 << 20


def _write(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        fh.write(text)


def make_tree(root, ngpu=8, hive=0x9CD4905654BB148F, partition="SPX", mesh=True, ue=None):
    nodes = os.path.join(root, "sys/class/kfd/kfd/topology/nodes")
    _write(f"{nodes}/0/properties", "cpu_cores_count 96\nsimd_count 0\nmem_banks_count 1\n")
    for i in range(ngpu):
        kfd = i + 1
        minor = 128 + i
        props = {"cpu_cores_count": 0, "simd_count": 1024, "simd_per_cu": 4, "gfx_target_version": 90500,
                 "vendor_id": 4098, "device_id": 0x75A3, "location_id": (0x05 + 0x10 * i) << 8, "domain": 0,
                 "drm_render_minor": minor, "hive_id": hive, "unique_id": 0x7D74AFAB5AA15265 + i,
                 "local_mem_size": 0}
        _write(f"{nodes}/{kfd}/properties", "".join(f"{k} {v}\n" for k, v in props.items()))
        _write(f"{nodes}/{kfd}/name", "gfx950\n")
        _write(f"{nodes}/{kfd}/mem_banks/0/properties", f"heap_type 1\nsize_in_bytes {VRAM}\nwidth 8192\n")
        links = [(0, 2)] + ([(j + 1, 11) for j in range(ngpu) if j != i] if mesh else [])
        for n, (to, typ) in enumerate(links):
            _write(f"{nodes}/{kfd}/io_links/{n}/properties", f"type {typ}\nnode_from {kfd}\nnode_to {to}\nweight 15\n")
        dev = os.path.join(root, f"sys/class/drm/renderD{minor}/device")
        _write(f"{dev}/current_compute_partition", partition + "\n")
        _write(f"{dev}/current_memory_partition", "NPS1\n")
        _write(f"{dev}/mem_info_vram_total", f"{VRAM}\n")
        _write(f"{dev}/numa_node", f"{i // 4}\n")
        _write(f"{dev}/ras/umc_err_count", f"ue: {(ue or {}).get(i, 0)}\nce: 3\n")
    _write(os.path.join(root, "sys/module/amdgpu/version"), "6.12.12\n")
    return root


@pytest.fixture(scope="module")
def native_ok():
    try:
        topo.native_topology("sysfs", "/nonexistent")
    except NativeUnavailable as exc:
        pytest.skip(f"native labeller not buildable here: {exc}")


def test_sysfs_collector_document(tmp_path, native_ok):
    doc = topo.native_topology("sysfs", make_tree(str(tmp_path)))
    assert doc["status"] == 0 and doc["source"] == "sysfs"
    assert doc["driver"] == {"name": "amdgpu", "version": "6.12.12"}
    gpus = doc["gpus"]
    assert len(gpus) == 8
    g = gpus[0]
    assert g["hip_id"] == 0 and g["drm_render"] == 128 and g["bdf"] == "0000:05:00.0"
    assert g["device_id"] == "0x75a3" and g["vendor_id"] == "0x1002" and g["market_name"] == "AMD Instinct MI355X"
    assert g["compute_units"] == 256 and g["target_graphics_version"] == "gfx950"
    assert g["vram_mb"] == 294896 and g["numa_node"] == 0 and gpus[7]["numa_node"] == 1
    assert g["compute_partition"] == "SPX" and g["memory_partition"] == "NPS1"
    assert g["xgmi_hive_id"] == "0x9cd4905654bb148f"
    assert g["ecc_correctable"] == 3 and g["ecc_uncorrectable"] == 0
    assert sorted(lk["peer"] for lk in g["links"]) == list(range(1, 8))
    assert all(lk["type"] == "XGMI" and lk["p2p"] for lk in g["links"])


def test_native_labels_equal_python_spec(tmp_path, native_ok):
    root = make_tree(str(tmp_path), ue={3: 2})
    native = topo.native_labels("sysfs", root)
    spec = labels_from_topology(topo.native_topology("sysfs", root))
    assert native == spec
    assert native["amd.com/gpu.product-name"] == "MI355X"
    assert native["amd.com/gpu.vram"] == "288G"
    assert native["amd.com/gpu.count"] == "8" and native["amd.com/gpu.cu-count"] == "256"
    assert native["amd.com/xgmi.fully-connected"] == "true" and native["amd.com/xgmi.links-per-gpu"] == "7"
    assert native["amd.com/gpu.ecc-uncorrectable"] == "2"


@pytest.mark.parametrize("kw,key,want", [
    ({"mesh": False}, "amd.com/xgmi.fully-connected", "false"),
    ({"partition": "CPX"}, "amd.com/gpu.compute-partition", "cpx"),
    ({"ngpu": 1}, "amd.com/xgmi.fully-connected", "false"),
])
def test_label_variants(tmp_path, native_ok, kw, key, want):
    root = make_tree(str(tmp_path), **kw)
    native = topo.native_labels("sysfs", root)
    assert native[key] == want
    assert native == labels_from_topology(topo.native_topology("sysfs", root))


def test_python_kfd_reader_agrees_on_topology(tmp_path, native_ok):
    root = make_tree(str(tmp_path))
    py = topo.kfd_topology(os.path.join(root, "sys/class/kfd/kfd/topology/nodes"))
    nat = topo.native_topology("sysfs", root)
    for a, b in zip(py["gpus"], nat["gpus"]):
        assert a["compute_units"] == b["compute_units"] and a["bdf"] == b["bdf"]
        assert sorted(lk["peer"] for lk in a["links"]) == sorted(lk["peer"] for lk in b["links"])


def test_executable_sysfs_root(tmp_path, native_ok):
    root = make_tree(str(tmp_path))
    exe = executable("amdgpu-topo-labeller")
    proc = subprocess.run([exe, "--labels", "--source", "sysfs", "--sysfs-root", root], capture_output=True,
                          text=True, timeout=60)
    assert proc.returncode == 0, proc.stderr
    assert "amd.com/gpu.product-name=MI355X" in proc.stdout.splitlines()
    proc = subprocess.run([exe, "--source", "sysfs", "--sysfs-root", root], capture_output=True, text=True,
                          timeout=60)
    assert json.loads(proc.stdout)["source"] == "sysfs"
    bad = subprocess.run([exe, "--source", "nope"], capture_output=True, text=True, timeout=60)
    assert bad.returncode == 64
    empty = subprocess.run([exe, "--labels", "--source", "sysfs", "--sysfs-root", str(tmp_path / "none")],
                           capture_output=True, text=True, timeout=60)
    assert empty.returncode == 2 and "no KFD topology" in empty.stderr


@pytest.mark.parametrize("flag,value", [("--max-uncorrectable", "abc"), ("--max-uncorrectable", "3x"),
                                        ("--max-uncorrectable", ""), ("--max-uncorrectable", " 2"),
                                        ("--max-uncorrectable", "99999999999999999999"),
                                        ("--max-bad-pages", "lots"), ("--max-bad-pages", "auto2")])
def test_health_thresholds_must_be_whole_numbers(tmp_path, native_ok, flag, value):
    """A threshold that is not a whole number is a usage error (64), not 0: `atoll("abc")`
    made every uncorrectable error count as too many, or none of them."""
    root = make_tree(str(tmp_path))
    exe = executable("amdgpu-topo-labeller")
    bad = subprocess.run([exe, "--health", "--source", "sysfs", "--sysfs-root", root, flag, value],
                         capture_output=True, text=True, timeout=60)
    assert bad.returncode == 64 and "usage:" in bad.stderr
    for good in (["--max-uncorrectable", "2", "--max-bad-pages", "auto"], ["--max-bad-pages", "-1"],
                 ["--max-bad-pages", "10"]):
        ok = subprocess.run([exe, "--health", "--source", "sysfs", "--sysfs-root", root] + good,
                            capture_output=True, text=True, timeout=60)
        assert ok.returncode == 0 and json.loads(ok.stdout)["status"] == "healthy", ok.stderr


# a RoCE port's GID table as mlx5 fills it: link-local IPv6 as RoCE v1 / v2 (0, 1), then
# the interface's IPv4 address, IPv4-mapped, as v1 / v2 (2, 3); empty slots read as zeros
ROCE_GIDS = [("IB/RoCE v1", "fe80:0000:0000:0000:0a00:00ff:fe00:0001"),
             ("RoCE v2", "fe80:0000:0000:0000:0a00:00ff:fe00:0001"),
             ("IB/RoCE v1", "0000:0000:0000:0000:0000:ffff:0a00:0001"),
             ("RoCE v2", "0000:0000:0000:0000:0000:ffff:0a00:0001"),
             (None, "0000:0000:0000:0000:0000:0000:0000:0000")]


def add_gids(port_dir, table):
    for i, (kind, gid) in enumerate(table):
        _write(f"{port_dir}/gids/{i}", gid + "\n")
        if kind is not None:
            _write(f"{port_dir}/gid_attrs/types/{i}", kind + "\n")


def add_rdma(root, nics, gids=ROCE_GIDS):
    """RDMA devices under sys/class/infiniband: (name, state, link_layer, rate, netdev, numa)."""
    for name, state, layer, rate, netdev, numa in nics:
        dev = os.path.join(root, "sys/class/infiniband", name)
        _write(f"{dev}/ports/1/state", f"{state}\n")
        _write(f"{dev}/ports/1/link_layer", f"{layer}\n")
        _write(f"{dev}/ports/1/rate", f"{rate}\n")
        if layer == "Ethernet" and gids:
            add_gids(f"{dev}/ports/1", gids)
        pci = os.path.join(root, "sys/devices/pci0000:00", f"0000:{0x1a + len(name):02x}:00.0")
        _write(f"{pci}/numa_node", f"{numa}\n")
        os.makedirs(f"{pci}/net/{netdev}", exist_ok=True)
        os.symlink(pci, f"{dev}/device")
    return root


RDMA = [("mlx5_0", "4: ACTIVE", "Ethernet", "400 Gb/sec (4X NDR)", "ens1f0np0", 0),
        ("mlx5_1", "1: DOWN", "Ethernet", "400 Gb/sec (4X NDR)", "ens1f1np1", 0),
        ("mlx5_2", "4: ACTIVE", "Ethernet", "200 Gb/sec (4X HDR)", "ens2f0np0", 1)]


def test_rdma_nics_python_reader_labels_and_rccl_env(tmp_path):
    from triton_kubernetes_amd.parallel.rccl_env import site_env_from_topology

    root = add_rdma(make_tree(str(tmp_path), ngpu=2), RDMA)
    nics = topo.rdma_nics(root)
    assert [n["name"] for n in nics] == ["mlx5_0", "mlx5_1", "mlx5_2"]
    assert [n["port"] for n in nics] == [1, 0, 1] and [n["active"] for n in nics] == [True, False, True]
    assert nics[0]["rate_gbps"] == 400 and nics[0]["netdev"] == "ens1f0np0" and nics[2]["numa_node"] == 1
    assert nics[0]["bdf"].startswith("0000:")
    labels = labels_from_topology({"gpus": [], "nics": nics})
    assert labels["amd.com/rdma.count"] == "2"
    assert labels["amd.com/rdma.link-layer"] == "ethernet" and labels["amd.com/rdma.rate-gbps"] == "200"
    env = site_env_from_topology({"nics": nics})
    assert nics[0]["roce_v2_gid_index"] == 3 and "roce_v2_gid_index" not in nics[1]  # a DOWN port: not read
    assert env == {"NCCL_IB_HCA": "=mlx5_0:1,mlx5_2:1", "NCCL_IB_GID_INDEX": "3"}
    assert site_env_from_topology({"nics": []}) == {}
    ib = [dict(n, link_layer="InfiniBand") for n in nics]
    assert site_env_from_topology({"nics": ib}) == {"NCCL_IB_HCA": "=mlx5_0:1,mlx5_2:1"}


@pytest.mark.parametrize("case", ["ipv6-only", "differ", "no-gids"])
def test_roce_gid_discovery(tmp_path, native_ok, case):
    """The RoCE v2 GID index is read from the ports' GID tables, not assumed: IPv4-mapped
    first, else IPv6; NCCL_IB_GID_INDEX only when every RoCE port agrees (else RCCL picks
    per port itself)."""
    from triton_kubernetes_amd.parallel.rccl_env import site_env_from_topology

    gids = {"ipv6-only": ROCE_GIDS[:2], "differ": ROCE_GIDS, "no-gids": None}[case]
    root = add_rdma(make_tree(str(tmp_path), ngpu=2), RDMA, gids=gids)
    if case == "differ":  # mlx5_2's IPv4 address sits at another index
        add_gids(os.path.join(root, "sys/class/infiniband/mlx5_2/ports/1"),
                 ROCE_GIDS[:2] + [(None, "0" * 4 + ":0000" * 7)] * 3 + ROCE_GIDS[2:4])
    doc = topo.native_topology("sysfs", root)
    assert doc["nics"] == topo.rdma_nics(root)
    want = {"ipv6-only": [1, 1], "differ": [3, 6], "no-gids": [None, None]}[case]
    active = [n for n in doc["nics"] if n["active"]]
    assert [n.get("roce_v2_gid_index") for n in active] == want
    env = topo.native_rccl_env(root)
    assert env == site_env_from_topology(doc)
    assert env.get("NCCL_IB_GID_INDEX") == ("1" if case == "ipv6-only" else None)


def test_rdma_native_matches_python(tmp_path, native_ok):
    """C++ NIC collector, its labels and its RCCL env equal the Python mirror."""
    from triton_kubernetes_amd.parallel.rccl_env import site_env_from_topology

    root = add_rdma(make_tree(str(tmp_path), ngpu=8), RDMA)
    doc = topo.native_topology("sysfs", root)
    assert doc["status"] == 0
    assert doc["nics"] == topo.rdma_nics(root)
    labels = topo.native_labels("sysfs", root)
    assert labels == labels_from_topology(doc)
    assert labels["amd.com/rdma.count"] == "2"
    assert topo.native_rccl_env(root) == site_env_from_topology(doc)
    exe = executable("amdgpu-topo-labeller")
    out = subprocess.run([exe, "--rccl-env", "--sysfs-root", root], capture_output=True, text=True, check=True).stdout
    assert out.splitlines() == ['NCCL_IB_HCA="=mlx5_0:1,mlx5_2:1"', 'NCCL_IB_GID_INDEX="3"']


def test_agent_rccl_env_merges_discovered_nics(tmp_path):
    """The agent writes the discovered RDMA settings; an explicit rccl_env key wins."""
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.labels import synthetic_topology
    from triton_kubernetes_amd.node.plan import build_host_plan
    from triton_kubernetes_amd.parallel.rccl_env import parse_env_file

    nics = topo.rdma_nics(add_rdma(str(tmp_path / "sys"), RDMA))
    topology = dict(synthetic_topology(1), nics=nics)
    agent = NodeAgent("n1", "sim", devices=[0], root=str(tmp_path / "node"), token="t",
                      topology_override=topology, burnin_override=lambda d, lvl: {"ok": True})
    cfg = {"hostname": "gpu-1", "rancher_host_labels": {"worker": "true"}, "gpu_count": 1,
           "rccl_env": {"NCCL_IB_GID_INDEX": "5", "NCCL_DEBUG": "INFO"}}
    plan = build_host_plan(cfg, "http://127.0.0.1:9", "t", "s", mi355x=True)
    plan.steps = [s for s in plan.steps if s.action != "agent"]
    res = agent.run_plan(plan)
    assert res["ok"], res
    env = parse_env_file((tmp_path / "node/etc/rccl/rccl.env").read_text())
    assert env["NCCL_IB_HCA"] == "=mlx5_0:1,mlx5_2:1"
    assert env["NCCL_IB_GID_INDEX"] == "5" and env["NCCL_DEBUG"] == "INFO"
    assert res["labels"]["amd.com/rdma.count"] == "2"
    step = next(s for s in res["steps"] if s["name"] == "rccl_env")
    assert step["detail"]["discovered"] == ["NCCL_IB_GID_INDEX", "NCCL_IB_HCA"]


# the harness may preload a library of its own: ASan is told not to insist on coming first
# rather than the child's environment being changed
ASAN_ENV = {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
            "UBSAN_OPTIONS": "print_stacktrace=1"}


@pytest.fixture(scope="module")
def asan_labeller(tmp_path_factory):
    import shutil

    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    src = os.path.join(os.path.dirname(topo.__file__), "csrc", "tk_topo.cpp")
    exe = str(tmp_path_factory.mktemp("asan") / "labeller-asan")
    build = subprocess.run([gxx, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                            "-fno-sanitize-recover=all", "-DTK_TOPO_MAIN", src, "-o", exe],
                           capture_output=True, text=True)
    assert build.returncode == 0, build.stderr[-2000:]
    return exe


def _asan_run(exe, argv):
    run = subprocess.run([exe] + argv, capture_output=True, text=True, env=dict(os.environ, **ASAN_ENV), timeout=60)
    assert "Sanitizer" not in run.stderr and "runtime error" not in run.stderr, run.stderr[-3000:]
    return run


def test_labeller_clean_under_asan_ubsan(tmp_path, asan_labeller):
    """Race/memory-safety check of the native labeller's host code (the
    reference has none): the sysfs collector built with AddressSanitizer + UBSan runs the
    JSON, --labels and --rccl-env paths over the fixture tree (GPUs + RDMA NICs) with no
    sanitizer report and the same output as the regular build."""
    root = add_rdma(make_tree(str(tmp_path / "root"), ngpu=8, ue={3: 2}), RDMA)
    ref = executable("amdgpu-topo-labeller") if os.path.exists(os.path.join(
        os.path.dirname(topo.__file__), "lib", "amdgpu-topo-labeller")) else None
    for args in ([], ["--labels"], ["--rccl-env"]):
        argv = args + (["--source", "sysfs"] if args != ["--rccl-env"] else []) + ["--sysfs-root", root]
        run = _asan_run(asan_labeller, argv)
        assert run.returncode == 0, run.stderr[-3000:]
        if ref:
            want = subprocess.run([ref] + argv, capture_output=True, text=True).stdout
            assert run.stdout == want


def _corrupt(root, how):
    """One damage to a fixture tree, as a failing disk, a half-written driver attribute or
    an odd kernel would leave sysfs."""
    nodes = os.path.join(root, "sys/class/kfd/kfd/topology/nodes")
    dev = os.path.join(root, "sys/class/drm/renderD129/device")
    ib = os.path.join(root, "sys/class/infiniband/mlx5_0/ports/1")
    if how == "empty-properties":
        _write(f"{nodes}/2/properties", "")
    elif how == "garbage-values":
        _write(f"{nodes}/2/properties", "simd_count abc\nsimd_per_cu -4\ndrm_render_minor zz\nhive_id -1\n"
                                        "location_id 0x\nunique_id 1e9\ngfx_target_version \n")
    elif how == "huge-numbers":
        _write(f"{nodes}/2/properties", "".join(f"{k} {'9' * 40}\n" for k in (
            "simd_count", "simd_per_cu", "gfx_target_version", "location_id", "domain", "drm_render_minor",
            "hive_id", "unique_id", "vendor_id", "device_id")))
        _write(f"{nodes}/2/mem_banks/0/properties", f"heap_type 1\nsize_in_bytes {'9' * 40}\n")
    elif how == "zero-cu":
        _write(f"{nodes}/2/properties", "simd_count 1024\nsimd_per_cu 0\nvendor_id 4098\ndrm_render_minor 129\n")
    elif how == "links-nowhere":
        for n, to in enumerate((999, -1, 2, 18446744073709551615)):
            _write(f"{nodes}/2/io_links/{n}/properties", f"type 11\nnode_from 2\nnode_to {to}\n")
    elif how == "long-line":
        _write(f"{nodes}/2/properties", "simd_count " + "1" * 200000 + "\nx" * 5000)
        _write(f"{nodes}/2/name", "g" * 100000)
    elif how == "binary-bytes":
        with open(f"{nodes}/2/name", "wb") as fh:
            fh.write(bytes(range(256)))
        with open(f"{dev}/current_compute_partition", "wb") as fh:
            fh.write(b"\xff\xfe\x00SPX\n")
    elif how == "property-is-a-directory":
        os.remove(f"{nodes}/2/properties")
        os.makedirs(f"{nodes}/2/properties")
        os.remove(f"{dev}/mem_info_vram_total")
        os.makedirs(f"{dev}/mem_info_vram_total")
    elif how == "drm-missing":
        import shutil

        shutil.rmtree(os.path.dirname(dev))
    elif how == "ras-garbage":
        _write(f"{dev}/ras/umc_err_count", "ue: \nce: -7\nue: 99999999999999999999999\n")
        _write(f"{dev}/numa_node", "-1\n")
        _write(f"{dev}/current_compute_partition", "\n")
    elif how == "no-gpu-nodes":
        import shutil

        for n in range(1, 9):
            shutil.rmtree(f"{nodes}/{n}")
    elif how == "rdma-garbage":
        _write(f"{ib}/state", "")
        _write(f"{ib}/rate", "fast\n")
        _write(f"{ib}/gids/0", "zz:" * 40 + "\n")
        _write(f"{ib}/gid_attrs/types/0", "\x00" * 10)
        os.remove(os.path.join(root, "sys/class/infiniband/mlx5_0/device"))
        os.symlink("/nonexistent/device", os.path.join(root, "sys/class/infiniband/mlx5_0/device"))
    return root


CORRUPTIONS = ["empty-properties", "garbage-values", "huge-numbers", "zero-cu", "links-nowhere", "long-line",
               "binary-bytes", "property-is-a-directory", "drm-missing", "ras-garbage", "no-gpu-nodes",
               "rdma-garbage"]


@pytest.mark.parametrize("how", CORRUPTIONS)
def test_labeller_clean_under_asan_ubsan_over_damaged_sysfs(tmp_path, asan_labeller, how):
    """The sanitizer build over damaged trees: each run ends with no AddressSanitizer or
    UBSan report and with a documented status (0, or 2 when no GPU is left to label), and
    what it prints is a JSON document or key=value lines."""
    root = _corrupt(add_rdma(make_tree(str(tmp_path / "root"), ngpu=8), RDMA), how)
    for args in ([], ["--labels"], ["--rccl-env"], ["--health"], ["--health", "--labels"], ["--prom", "--node", "n1"]):
        argv = args + (["--source", "sysfs"] if args != ["--rccl-env"] else []) + ["--sysfs-root", root]
        run = _asan_run(asan_labeller, argv)
        # --health: 3 is its verdict "a GPU is unhealthy"
        assert run.returncode in ((0, 2, 3) if "--health" in args else (0, 2)), \
            (how, args, run.returncode, run.stderr[-3000:])
        if run.returncode in (0, 3) and args in ([], ["--health"]):
            json.loads(run.stdout)
        elif run.returncode == 0 and args[0] == "--prom":
            assert all(ln.startswith("#") or " " in ln for ln in run.stdout.splitlines()), run.stdout[:500]
        elif run.returncode == 0:
            assert all("=" in line for line in run.stdout.splitlines()), run.stdout[:500]


def test_rdma_port_with_an_odd_name_stays_out_of_the_rccl_env(tmp_path, native_ok):
    """A port name that is not a plain device name is left to RCCL's own detection by both
    renderers (the file is loaded as root): the C++ labeller and the Python mirror agree."""
    from triton_kubernetes_amd.parallel.rccl_env import site_env_from_topology

    odd = [("mlx5_0", "4: ACTIVE", "InfiniBand", "400 Gb/sec (4X NDR)", "ib0", 0),
           ("x$(id)", "4: ACTIVE", "InfiniBand", "400 Gb/sec (4X NDR)", "ib1", 0)]
    root = add_rdma(make_tree(str(tmp_path), ngpu=2), odd)
    doc = topo.native_topology("sysfs", root)
    assert sorted(n["name"] for n in doc["nics"]) == ["mlx5_0", "x$(id)"]
    assert topo.native_rccl_env(root) == site_env_from_topology(doc) == {"NCCL_IB_HCA": "=mlx5_0:1"}


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(ngpu=st.integers(1, 8), partition=st.sampled_from(["SPX", "DPX", "QPX", "CPX"]), mesh=st.booleans(),
       hive=st.integers(1, 2 ** 63 - 1), ue=st.dictionaries(st.integers(0, 7), st.integers(0, 50), max_size=3))
def test_native_labels_equal_python_spec_over_generated_nodes(native_ok, ngpu, partition, mesh, hive, ue):
    """The C++ labeller and the Python spec (node/labels.py) over generated nodes: GPU count,
    partition mode, xGMI mesh or none, hive id, uncorrectable-error counts."""
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        root = make_tree(d, ngpu=ngpu, hive=hive, partition=partition, mesh=mesh, ue=ue)
        native = topo.native_labels("sysfs", root)
        assert native == labels_from_topology(topo.native_topology("sysfs", root))
        assert native["amd.com/gpu.count"] == str(ngpu)


K8S_LABEL_VALUE = r"(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?"


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(version=st.text(alphabet=st.characters(blacklist_categories=("Cs",), blacklist_characters="\x00"),
                       min_size=1, max_size=90))
def test_free_text_becomes_the_same_valid_label_value_in_both(native_ok, version):
    """Free text the node reports (here its ROCm version file) turns into the same label value
    in the C++ labeller and in the Python spec, and that value is a valid Kubernetes label
    value (at most 63 characters, alphanumeric at both ends) -- long, non-ASCII and
    punctuation-heavy text included."""
    import re
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        root = make_tree(d, ngpu=1)
        _write(os.path.join(root, "opt/rocm/.info/version"), version)
        native = topo.native_labels("sysfs", root)
        doc = topo.native_topology("sysfs", root)
        assert native == labels_from_topology(doc)
        for v in native.values():
            assert len(v) <= 63 and re.fullmatch(K8S_LABEL_VALUE, v), (version, v)


@pytest.mark.parametrize("how", CORRUPTIONS)
def test_in_process_readers_over_damaged_sysfs(tmp_path, native_ok, how):
    """The in-process library and the Python KFD reader over the same damaged trees: a
    document (or NativeUnavailable for a tree with no GPU left), never a decode error --
    bytes that are not UTF-8 come through as U+FFFD on both sides."""
    root = _corrupt(add_rdma(make_tree(str(tmp_path / "root"), ngpu=8), RDMA), how)
    doc = topo.native_topology("sysfs", root)
    assert doc["status"] in (0, 2)
    py = topo.kfd_topology(os.path.join(root, "sys/class/kfd/kfd/topology/nodes"))
    assert isinstance(py["gpus"], list)
    if how == "binary-bytes":
        names = [g["market_name"] for g in py["gpus"]]
        assert any("�" in n for n in names)
        assert json.loads(json.dumps(doc)) == doc
    if doc["status"] == 0:
        assert topo.native_labels("sysfs", root) == labels_from_topology(doc)


def test_prom_text_stays_utf8_over_a_node_name_that_is_not(tmp_path, native_ok):
    """The exposition format is UTF-8 (node_exporter drops a textfile that is not): a node
    name with bytes that are not comes out with U+FFFD, quotes and backslashes escaped."""
    root = make_tree(str(tmp_path), ngpu=2)
    out = subprocess.run([executable("amdgpu-topo-labeller"), "--prom", "--source", "sysfs", "--sysfs-root", root,
                          "--node", os.fsdecode(b'n\xff\xfe"x\\')], capture_output=True, timeout=60).stdout
    text = out.decode("utf-8")
    assert 'tk_gpu_healthy{node="n��\\"x\\\\",gpu="0"' in text
