"""Kubernetes node labels for AMD GPU nodes, derived from the N1 topology document.

Label keys follow the ROCm k8s node-labeller's ``amd.com/gpu.*`` namespace,
plus xGMI keys used for topology-aware scheduling:

=====================================  =============================================
``amd.com/gpu.present``                ``true``
``amd.com/gpu.count``                  physical GPUs on the node (distinct PCI functions)
``amd.com/gpu.logical-count``          schedulable GPUs: compute partitions (``amd.com/gpu``)
``amd.com/gpu.partitions-per-gpu``     compute partitions per physical GPU (1 in SPX)
``amd.com/gpu.product-name``           e.g. ``MI355X`` (from the market name)
``amd.com/gpu.family``                 ``AI`` for Instinct parts
``amd.com/gpu.device-id``              PCI device id
``amd.com/gpu.cu-count``               CUs per GPU (min over GPUs)
``amd.com/gpu.vram``                   VRAM per GPU, e.g. ``288G``
``amd.com/gpu.target``                 ``gfx950``
``amd.com/gpu.compute-partition``      ``spx`` / ``cpx`` ... (lower-cased)
``amd.com/gpu.memory-partition``       ``nps1`` / ``nps4`` ...
``amd.com/xgmi.hive-id``               hive id shared by the node's GPUs (hex)
``amd.com/xgmi.links-per-gpu``         min xGMI peers over GPUs
``amd.com/xgmi.fully-connected``       every GPU has an xGMI link to every other; only
                                       claimed in SPX (node/partition.py)
``amd.com/gpu.ecc-uncorrectable``      uncorrectable ECC errors, summed over physical GPUs
``amd.com/gpu.bad-pages``              retired VRAM pages (driver bad-page records), summed
``amd.com/gpu.pcie-width``             the narrowest GPU's PCIe link width (lanes)
``amd.com/gpu.vbios``                  the GPUs' VBIOS version (``mixed`` when they differ)
``amd.com/rocm.version``               the node's ROCm userspace (``<ROCM_PATH>/.info/version``)
``amd.com/gpu.power-cap``              the lowest GPU board power cap (W)
``amd.com/gpu.health``                 ``healthy`` / ``unhealthy`` (node/health.py policy)
=====================================  =============================================

Pods that need all 8 GPUs on one xGMI hive use node affinity on
``amd.com/xgmi.fully-connected=true`` + ``amd.com/gpu.count=8``; multi-node jobs
use pod affinity on ``amd.com/xgmi.hive-id`` to stay inside a hive where the
fabric spans nodes (see ``k8s/manifests.py``).
"""

import re
from typing import Any, Dict, List

LABEL_PREFIX = "amd.com/"
_VALUE_RE = re.compile(r"[^A-Za-z0-9._-]")


def _label_value(v: Any) -> str:
    """A Kubernetes label value: at most 63 characters, alphanumeric at both ends (the cut
    can leave a '-', '.' or '_' last, which is trimmed again).  Mirrored in
    ``ops/csrc/tk_topo.cpp:label_value``."""
    s = _VALUE_RE.sub("-", str(v)).strip("-._")
    return s[:63].rstrip("-._")


# PCI device id -> product, for parts whose market name is not the SKU name
# (amd_smi reports an MI355X as "AMD Instinct MI355 OAM").  Mirrored in
# ops/csrc/tk_topo.cpp:product_from_device_id.
DEVICE_PRODUCTS = {"0x75a3": "MI355X", "0x75a0": "MI350X", "0x74a5": "MI325X", "0x74a1": "MI300X"}


def product_name(market_name: str, device_id: str = "") -> str:
    if str(device_id).lower() in DEVICE_PRODUCTS:
        return DEVICE_PRODUCTS[str(device_id).lower()]
    m = re.search(r"(MI\d{3}[A-Z]*)", market_name or "")
    return m.group(1) if m else _label_value(market_name)


def rdma_labels(doc: Dict[str, Any]) -> Dict[str, str]:
    """``amd.com/rdma.*``: the node's active RDMA ports (inter-node RCCL fabric)."""
    active = [n for n in doc.get("nics", []) or [] if n.get("port", 0) > 0]
    labels = {"amd.com/rdma.count": str(len(active))}
    layers = {str(n.get("link_layer", "")).lower() for n in active if n.get("link_layer")}
    if len(layers) == 1:
        labels["amd.com/rdma.link-layer"] = _label_value(layers.pop())
    rates = [int(n["rate_gbps"]) for n in active if n.get("rate_gbps")]
    if rates:
        labels["amd.com/rdma.rate-gbps"] = str(min(rates))
    return labels


def labels_from_topology(doc: Dict[str, Any]) -> Dict[str, str]:
    labels = _gpu_labels(doc)
    labels.update(rdma_labels(doc))
    return labels


def _gpu_labels(doc: Dict[str, Any]) -> Dict[str, str]:
    gpus: List[Dict[str, Any]] = doc.get("gpus") or []
    if not gpus:
        return {"amd.com/gpu.present": "false"}
    physical = len({g.get("bdf") or f"#{i}" for i, g in enumerate(gpus)})  # = node/partition.physical_count
    labels: Dict[str, str] = {
        "amd.com/gpu.present": "true",
        "amd.com/gpu.count": str(physical),
        "amd.com/gpu.logical-count": str(len(gpus)),
    }
    rocm = (doc.get("rocm") or {}).get("version")
    if rocm:
        labels["amd.com/rocm.version"] = _label_value(rocm)
    if len(gpus) % physical == 0:
        labels["amd.com/gpu.partitions-per-gpu"] = str(len(gpus) // physical)
    names = {product_name(g.get("market_name", ""), g.get("device_id", "")) for g in gpus
             if g.get("market_name") or str(g.get("device_id", "")).lower() in DEVICE_PRODUCTS}
    if len(names) == 1:
        name = names.pop()
        labels["amd.com/gpu.product-name"] = _label_value(name)
        if name.startswith("MI"):
            labels["amd.com/gpu.family"] = "AI"
    # a GPU whose KFD node carries no device_id reads as 0x0: unknown, not a different id
    dev_ids = {g.get("device_id") for g in gpus if g.get("device_id") not in (None, "", "0x0")}
    if len(dev_ids) == 1:
        labels["amd.com/gpu.device-id"] = _label_value(dev_ids.pop())
    cus = [int(g["compute_units"]) for g in gpus if g.get("compute_units")]
    if cus:
        labels["amd.com/gpu.cu-count"] = str(min(cus))
    vram = [int(g["vram_mb"]) for g in gpus if g.get("vram_mb")]
    if vram:
        # nearest GiB: the 294896 MiB an MI355X reports reads as 288G
        labels["amd.com/gpu.vram"] = f"{(min(vram) + 512) // 1024}G"
    targets = {g.get("target_graphics_version") for g in gpus if g.get("target_graphics_version")}
    if len(targets) == 1:
        labels["amd.com/gpu.target"] = _label_value(targets.pop())
    cmodes = set()
    for key, label in (("compute_partition", "compute-partition"), ("memory_partition", "memory-partition")):
        vals = {str(g.get(key, "")).lower() for g in gpus if g.get(key)}
        if key == "compute_partition":
            cmodes = set(vals)
        if len(vals) == 1:
            labels[f"amd.com/gpu.{label}"] = _label_value(vals.pop())
    hives = {g.get("xgmi_hive_id") for g in gpus if g.get("xgmi_hive_id") not in (None, "", "0x0")}
    if len(hives) == 1:
        labels["amd.com/xgmi.hive-id"] = _label_value(hives.pop())
    # one VBIOS on every GPU, or "mixed" (a node whose GPUs were flashed apart)
    vbioses = {g["vbios_version"] for g in gpus if g.get("vbios_version")}
    if vbioses:
        labels["amd.com/gpu.vbios"] = _label_value(vbioses.pop()) if len(vbioses) == 1 else "mixed"
    caps = [int(g["power_cap_w"]) for g in gpus if int(g.get("power_cap_w", -1)) > 0]
    if caps:
        labels["amd.com/gpu.power-cap"] = str(min(caps))  # watts, the lowest GPU
    xgmi_peers = []
    for g in gpus:
        peers = {lk["peer"] for lk in g.get("links", []) if lk.get("type") == "XGMI"}
        xgmi_peers.append(len(peers))
    labels["amd.com/xgmi.links-per-gpu"] = str(min(xgmi_peers))
    # a compute partition is not a whole GPU with its own xGMI links: the full-mesh claim
    # (what multi-GPU pods are placed on) holds in SPX only
    whole = cmodes <= {"spx"} and physical == len(gpus)
    labels["amd.com/xgmi.fully-connected"] = "true" if whole and len(gpus) > 1 and \
        min(xgmi_peers) == len(gpus) - 1 else "false"
    # RAS counters per physical GPU (its partitions report the same device's counters)
    from .health import physical_gpus, ras_labels

    phys = physical_gpus(doc)
    labels.update(ras_labels(phys))
    return labels


def burnin_labels(level: str, results: Dict[Any, Dict[str, Any]]) -> Dict[str, str]:
    """Node labels that say what the burn-in covered (same keys and formatting as
    ``gpu-burnin --labels``, the SSH / Terraform path): pass/fail, the level, and the HBM
    the memtest held -- the minimum over the node's GPUs, in GiB and percent of the card.
    ``quick`` memtests 1 GiB (0.3 % of 288 GiB); ``full`` every free byte but 4 GiB."""
    ok = all(r.get("ok", False) for r in results.values()) if results else False
    tested = [int((r.get("memtest") or {}).get("bytes", 0)) for r in results.values()]
    total = [int((r.get("memtest") or {}).get("hbm_bytes", 0)) for r in results.values()]
    lo = min(tested) if tested else 0
    frac = min((t / h for t, h in zip(tested, total) if h), default=0.0)
    return {"amd.com/gpu.burnin": "passed" if ok else "failed",
            "amd.com/gpu.burnin-level": level,
            "amd.com/gpu.burnin-hbm-tested-gib": f"{lo / (1 << 30):.0f}",
            "amd.com/gpu.burnin-hbm-tested-pct": f"{100.0 * frac:.1f}"}


DEFAULT_MIN_LINK_GBPS = 38.0  # = ops/probe.py (half of one xGMI link's ~76.8 GB/s one way)


def link_labels(matrix: Dict[str, Any], min_frac: float = 0.5,
                min_gbps: float = DEFAULT_MIN_LINK_GBPS) -> Dict[str, Any]:
    """Verdict and labels of a node's peer-to-peer link matrix (``ops/probe.py:link_matrix``
    or ``gpu-burnin --p2p``).  A pair is a degraded xGMI link when it is below ``min_frac``
    of the node's median (one bad link) OR below the absolute floor ``min_gbps`` (a
    uniformly slow fabric, whose median looks healthy) OR when the data it delivered did not
    match what was sent (``data_errors``: ``corrupt``); a pair without peer access or whose
    transfer failed is an error.  Returns ``{"labels": {...}, "degraded": [...],
    "below_floor": [...], "corrupt": [...], "status": passed|degraded|error}``."""
    vals = sorted(matrix.get("pairs", {}).values())
    errors = list(matrix.get("errors", []))
    errors += [f"{p}: no peer access" for p, ok in sorted(matrix.get("peer_access", {}).items()) if not ok]
    if not vals:
        return {"labels": {}, "degraded": [], "below_floor": [], "errors": errors,
                "status": "error" if errors else "skipped"}
    median = vals[len(vals) // 2] if len(vals) % 2 else 0.5 * (vals[len(vals) // 2 - 1] + vals[len(vals) // 2])
    below = sorted(p for p, v in matrix["pairs"].items() if v < min_gbps)
    # a link that delivered wrong data is degraded whatever its speed
    corrupt = sorted(p for p, w in (matrix.get("data_errors") or {}).items() if w)
    degraded = sorted(set(p for p, v in matrix["pairs"].items() if v < min_frac * median or v < min_gbps)
                      | set(corrupt))
    status = "error" if errors else ("degraded" if degraded else "passed")
    labels = {"amd.com/xgmi.link-check": status,
              "amd.com/xgmi.p2p-min-gbps": f"{vals[0]:.0f}",
              "amd.com/xgmi.p2p-median-gbps": f"{median:.0f}"}
    if matrix.get("method"):
        labels["amd.com/xgmi.p2p-method"] = str(matrix["method"])
    return {"labels": labels, "degraded": degraded, "below_floor": below, "corrupt": corrupt, "errors": errors,
            "status": status, "floor_gbps": min_gbps}


def merge_link_matrices(a: Dict[str, Any], b: Dict[str, Any]) -> Dict[str, Any]:
    """Two measurements of a node's link matrix as one: each pair's best bandwidth (a
    throughput that read low once is not a slow link), every data error of either (a link
    that corrupted data once stays corrupt), the errors of the later one."""
    pairs = dict(a.get("pairs") or {})
    for p, v in (b.get("pairs") or {}).items():
        pairs[p] = max(v, pairs.get(p, v))
    data = dict(a.get("data_errors") or {})
    for p, w in (b.get("data_errors") or {}).items():
        data[p] = int(data.get(p, 0)) + int(w)
    return dict(a, pairs=pairs, data_errors=data, errors=list(b.get("errors") or []),
                peer_access=dict(b.get("peer_access") or a.get("peer_access") or {}))


LINK_REMEASURE = 2  # extra measurements of a matrix whose only fault is speed (as ops/probe.py:REMEASURE)


def best_link_verdict(measure, min_frac: float = 0.5, min_gbps: float = DEFAULT_MIN_LINK_GBPS,
                      remeasure: int = LINK_REMEASURE) -> Dict[str, Any]:
    """:func:`link_labels` of ``measure()``, measured again (best of up to ``remeasure`` + 1
    per pair) while the verdict is ``degraded`` for speed alone -- the burn-in's rule for
    throughput gates.  A pair that delivered wrong data, or a pair that could not be
    measured, is never retried away.  ``remeasured`` counts the extra measurements."""
    matrix = measure()
    verdict = link_labels(matrix, min_frac, min_gbps)
    tries = 0
    while verdict["status"] == "degraded" and not verdict.get("corrupt") and tries < remeasure:
        matrix = merge_link_matrices(matrix, measure())
        verdict = link_labels(matrix, min_frac, min_gbps)
        tries += 1
    verdict["remeasured"] = tries
    verdict["matrix"] = matrix
    return verdict


def agent_label_flags(labels: Dict[str, str]) -> List[str]:
    """``--label k=v`` arguments for ``rancher/agent``."""
    out: List[str] = []
    for k in sorted(labels):
        out += ["--label", f"{k}={labels[k]}"]
    return out


def synthetic_topology(ngpus: int = 8, hive: str = "0xabc123", product: str = "AMD Instinct MI355X",
                       cus: int = 256, vram_mb: int = 294912) -> Dict[str, Any]:
    """A fully connected 8xMI355X topology document (tests / dry runs)."""
    gpus = []
    for i in range(ngpus):
        gpus.append({
            "index": i, "market_name": product, "device_id": "0x75a3", "compute_units": cus, "vram_mb": vram_mb,
            "target_graphics_version": "gfx950", "compute_partition": "SPX", "memory_partition": "NPS1",
            "xgmi_hive_id": hive, "ecc_uncorrectable": 0, "ecc_correctable": 0, "bad_pages": 0,
            "bad_pages_pending": 0, "pcie_width": 16, "pcie_max_width": 16,
            "links": [{"peer": j, "type": "XGMI", "hops": 1, "p2p": True} for j in range(ngpus) if j != i],
        })
    return {"source": "synthetic", "gpus": gpus}
