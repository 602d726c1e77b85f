"""Node GPU topology (N1): the native labeller ``csrc/tk_topo.cpp``.

``discover()`` returns its JSON document.  Sources, in the order tried:

1. ``sysfs`` in-process (``libtk_topo.so``): KFD topology + DRM attributes,
   plain file reads (~1 ms) — the default on the bootstrap critical path;
2. ``amdsmi`` out of process (``amdgpu-topo-labeller``): amd_smi's own view,
   kept in a child process so its library state never shares an address
   space with HIP/RCCL (tens of ms, mostly ``amdsmi_init``);
3. the pure-Python KFD reader below when no native build is present.

The GPU tests assert that sources 1 and 2 yield identical node labels.
"""

import ctypes
import glob
import json
import os
import subprocess
from typing import Any, Dict, List, Optional

from .native import NativeUnavailable, executable, load

KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"
# io_link type values in KFD (kfd_topology.h): 11 = XGMI, 2 = PCIe
_KFD_LINK_TYPES = {11: "XGMI", 2: "PCIE"}
GFX_TARGETS = {90500: "gfx950", 90400: "gfx942", 90402: "gfx942", 90010: "gfx90a"}


def amdsmi_topology(timeout: float = 60.0, source: str = "amdsmi") -> Dict[str, Any]:
    """Run the ``amdgpu-topo-labeller`` executable (amd_smi in its own process).

    Kept out of process on purpose: amd_smi's library state and teardown then
    never share an address space with the HIP runtime / RCCL of the caller.
    """
    exe = executable("amdgpu-topo-labeller")
    proc = subprocess.run([exe, "--source", source], capture_output=True, text=True, timeout=timeout,
                          check=False)
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    if not lines:
        raise NativeUnavailable(f"amdgpu-topo-labeller produced no JSON (rc={proc.returncode}): {proc.stderr[-500:]}")
    doc = json.loads(lines[-1])
    doc["status"] = proc.returncode
    return doc


def amdsmi_labels(timeout: float = 60.0, source: str = "amdsmi", sysfs_root: str = "") -> Dict[str, str]:
    """``amdgpu-topo-labeller --labels``: the node labels computed natively."""
    exe = executable("amdgpu-topo-labeller")
    argv = [exe, "--labels", "--source", source] + (["--sysfs-root", sysfs_root] if sysfs_root else [])
    proc = subprocess.run(argv, capture_output=True, text=True, timeout=timeout, check=False)
    if proc.returncode != 0:
        raise NativeUnavailable(f"amdgpu-topo-labeller --labels failed (rc={proc.returncode}): {proc.stderr[-500:]}")
    out: Dict[str, str] = {}
    for ln in proc.stdout.splitlines():
        if ln.startswith("amd.com/") and "=" in ln:
            k, v = ln.split("=", 1)
            out[k] = v
    return out


def _native_call(fn_name: str, source: str, root: str) -> "tuple[int, str]":
    lib = load("libtk_topo.so")
    fn = getattr(lib, fn_name)
    fn.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    fn.restype = ctypes.c_int
    size = 1 << 16
    while True:
        buf = ctypes.create_string_buffer(size)
        rc = fn(source.encode(), root.encode(), buf, size)
        if rc < 0:
            size = -rc + 1
            continue
        return rc, buf.value.decode()


def native_topology(source: str = "sysfs", sysfs_root: str = "") -> Dict[str, Any]:
    """The labeller's JSON document, in-process (sysfs collector; the library
    is built without amd_smi, which runs in a child: :func:`amdsmi_topology`)."""
    rc, text = _native_call("tkt_topology_json_src", source, sysfs_root)
    doc = json.loads(text)
    doc["status"] = rc
    return doc


def native_rccl_env(sysfs_root: str = "") -> Dict[str, str]:
    """The labeller's inter-node RCCL settings (``amdgpu-topo-labeller --rccl-env``), in-process."""
    from ..parallel.rccl_env import parse_env_file

    lib = load("libtk_topo.so")
    fn = lib.tkt_rccl_env_src
    fn.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    fn.restype = ctypes.c_int
    buf = ctypes.create_string_buffer(1 << 14)
    rc = fn(sysfs_root.encode(), buf, len(buf))
    if rc != 0:
        raise NativeUnavailable(f"tkt_rccl_env_src failed ({rc})")
    return parse_env_file(buf.value.decode())


def native_labels(source: str = "sysfs", sysfs_root: str = "") -> Dict[str, str]:
    rc, text = _native_call("tkt_topology_labels_src", source, sysfs_root)
    if rc != 0:
        raise NativeUnavailable(f"native labeller ({source}) failed with status {rc}")
    return dict(ln.split("=", 1) for ln in text.splitlines() if "=" in ln)


def native_health(source: str = "sysfs", sysfs_root: str = "", max_uncorrectable: int = 0,
                  max_bad_pages: int = -1) -> Dict[str, Any]:
    """The labeller's GPU health verdict (``amdgpu-topo-labeller --health``), in-process."""
    lib = load("libtk_topo.so")
    fn = lib.tkt_health_src
    fn.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_int,
                   ctypes.c_char_p, ctypes.c_size_t]
    fn.restype = ctypes.c_int
    size = 1 << 16
    while True:
        buf = ctypes.create_string_buffer(size)
        rc = fn(source.encode(), sysfs_root.encode(), max_uncorrectable, max_bad_pages, 0, buf, size)
        if rc < 0:
            size = -rc + 1
            continue
        if rc != 0:
            raise NativeUnavailable(f"native labeller ({source}) failed with status {rc}")
        return json.loads(buf.value.decode())


def _read_props(path: str) -> Dict[str, int]:
    props: Dict[str, int] = {}
    try:
        with open(path, "r", encoding="utf-8", errors="replace") as fh:
            for line in fh:
                parts = line.split()
                if len(parts) == 2:
                    try:
                        props[parts[0]] = int(parts[1])
                    except ValueError:
                        pass
    except OSError:
        pass
    return props


def kfd_topology(root: str = KFD_TOPOLOGY) -> Dict[str, Any]:
    """GPU nodes (``simd_count > 0``) and their io_links from KFD sysfs."""
    nodes = []
    for node_dir in sorted(glob.glob(os.path.join(root, "*")), key=lambda p: int(os.path.basename(p))
                           if os.path.basename(p).isdigit() else 1 << 30):
        props = _read_props(os.path.join(node_dir, "properties"))
        if props.get("simd_count", 0) <= 0:
            continue
        name = ""
        try:
            with open(os.path.join(node_dir, "name"), "r", encoding="utf-8", errors="replace") as fh:
                name = fh.read().strip()
        except OSError:
            pass
        links = []
        for link in sorted(glob.glob(os.path.join(node_dir, "io_links", "*"))):
            lp = _read_props(os.path.join(link, "properties"))
            links.append({"kfd_to": lp.get("node_to", -1), "type": _KFD_LINK_TYPES.get(lp.get("type", -1), "OTHER"),
                          "weight": lp.get("weight", 0)})
        nodes.append({"kfd_node": int(os.path.basename(node_dir)), "name": name, "props": props, "links": links})
    kfd_to_index = {n["kfd_node"]: i for i, n in enumerate(nodes)}
    gpus: List[Dict[str, Any]] = []
    for i, n in enumerate(nodes):
        p = n["props"]
        simd_per_cu = p.get("simd_per_cu", 4) or 4
        gfx = GFX_TARGETS.get(p.get("gfx_target_version", 0), "")
        gpu: Dict[str, Any] = {
            "index": i,
            "kfd_node": n["kfd_node"],
            "market_name": n["name"],
            "device_id": hex(p.get("device_id", 0)),
            "compute_units": p.get("simd_count", 0) // simd_per_cu,
            "numa_node": max(0, p.get("numa_node", 0) if "numa_node" in p else 0),
            "xgmi_hive_id": hex(p.get("hive_id", 0)) if p.get("hive_id") else "0x0",
            "links": [],
        }
        if gfx:
            gpu["target_graphics_version"] = gfx
        if "domain" in p or "location_id" in p:
            loc = p.get("location_id", 0)
            gpu["bdf"] = f"{p.get('domain', 0):04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"
        for lk in n["links"]:
            if lk["kfd_to"] in kfd_to_index:
                gpu["links"].append({"peer": kfd_to_index[lk["kfd_to"]], "type": lk["type"],
                                     "hops": 1, "p2p": lk["type"] == "XGMI"})
        gpus.append(gpu)
    return {"source": "kfd", "gpus": gpus}


def _read_text(path: str) -> Optional[str]:
    try:
        with open(path, "r", encoding="utf-8", errors="replace") as fh:
            return fh.read().strip()
    except OSError:
        return None


def roce_v2_gid(port_dir: str) -> int:
    """The port's RoCE v2 GID index: the first IPv4-mapped one, else the first IPv6 one,
    -1 when it has none (mirror of ``csrc/tk_topo.cpp:roce_v2_gid``)."""
    try:
        idx = sorted(int(i) for i in os.listdir(os.path.join(port_dir, "gid_attrs", "types")) if i.isdigit())
    except OSError:
        return -1
    v6 = -1
    for i in idx:
        if _read_text(os.path.join(port_dir, "gid_attrs", "types", str(i))) != "RoCE v2":
            continue
        gid = _read_text(os.path.join(port_dir, "gids", str(i))) or ""
        if not gid.strip("0:"):
            continue  # an empty slot
        if gid.startswith("0000:0000:0000:0000:0000:ffff:"):
            return i
        if v6 < 0:
            v6 = i
    return v6


def rdma_nics(root: str = "") -> List[Dict[str, Any]]:
    """RDMA devices under ``<root>/sys/class/infiniband`` (the inter-node RCCL fabric).

    Mirror of ``csrc/tk_topo.cpp:collect_nics``: the first ACTIVE port of each device,
    its link layer (``InfiniBand`` / ``Ethernet`` = RoCE) and rate, the netdev and PCI
    function behind it, and its NUMA node."""
    base = os.path.join(root or "/", "sys/class/infiniband")
    try:
        names = sorted(n for n in os.listdir(base) if not n.startswith("."))
    except OSError:
        return []
    out: List[Dict[str, Any]] = []
    for name in names:
        dev = os.path.join(base, name)
        nic: Dict[str, Any] = {"name": name, "port": 0, "active": False, "link_layer": "", "rate_gbps": 0}
        ports_dir = os.path.join(dev, "ports")
        try:
            ports = sorted(int(p) for p in os.listdir(ports_dir) if p.isdigit())
        except OSError:
            ports = []
        for port in ports:
            pd = os.path.join(ports_dir, str(port))
            state = _read_text(os.path.join(pd, "state")) or ""
            if "ACTIVE" not in state:
                if not nic["link_layer"]:
                    nic["link_layer"] = _read_text(os.path.join(pd, "link_layer")) or ""
                continue
            nic.update(port=port, active=True, link_layer=_read_text(os.path.join(pd, "link_layer")) or "")
            rate = (_read_text(os.path.join(pd, "rate")) or "").split()
            nic["rate_gbps"] = int(rate[0]) if rate and rate[0].isdigit() else 0
            gid = roce_v2_gid(pd)
            if gid >= 0:
                nic["roce_v2_gid_index"] = gid
            break
        try:
            nets = sorted(n for n in os.listdir(os.path.join(dev, "device", "net")) if not n.startswith("."))
        except OSError:
            nets = []
        if nets:
            nic["netdev"] = nets[0]
        try:
            nic["bdf"] = os.path.basename(os.readlink(os.path.join(dev, "device")))
        except OSError:
            pass
        numa = _read_text(os.path.join(dev, "device", "numa_node"))
        if numa is not None and numa.lstrip("-").isdigit():
            nic["numa_node"] = int(numa)
        out.append(nic)
    return out


def discover(kfd_root: Optional[str] = None, prefer: str = "sysfs") -> Dict[str, Any]:
    """Best-effort topology: native sysfs (or amd_smi), the other native source, Python KFD, empty."""
    if kfd_root is None:
        order = ["sysfs", "amdsmi"] if prefer == "sysfs" else ["amdsmi", "sysfs"]
        for source in order:
            try:
                doc = native_topology("sysfs") if source == "sysfs" else amdsmi_topology()
                if doc.get("status") == 0 and doc.get("gpus"):
                    return doc
            except (NativeUnavailable, OSError, ValueError, subprocess.SubprocessError):
                continue
    root = kfd_root or KFD_TOPOLOGY
    if os.path.isdir(root):
        doc = kfd_topology(root)
        doc["nics"] = rdma_nics("" if kfd_root is None else os.path.join(kfd_root, *[".."] * 6))
        return doc
    return {"source": "none", "gpus": [], "nics": rdma_nics() if kfd_root is None else []}
