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
