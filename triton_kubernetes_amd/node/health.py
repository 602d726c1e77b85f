"""MI355X GPU health policy: RAS counters -> healthy / unhealthy, at bring-up and on demand.

The reference has no notion of GPU health (it joined whatever host it was given,
``terraform/modules/bare-metal-rancher-k8s-host/main.tf:24-42``).  A fleet of MI355X nodes
needs one: a GPU that has logged uncorrectable HBM errors, or has retired more VRAM pages
than the driver's own threshold, should not receive GPU pods.

Inputs are the N1 topology document (``ops/csrc/tk_topo.cpp``: amd_smi or sysfs) -- per
GPU ``ecc_uncorrectable`` / ``ecc_correctable`` (summed over the RAS blocks) and
``bad_pages`` / ``bad_pages_pending`` (the driver's bad-page records,
``ras/gpu_vram_bad_pages`` or ``amdsmi_get_gpu_bad_page_info``).

Rules (mirrored by ``tk_topo.cpp:render_health``; tests compare the two on fixture trees),
judged per **physical** GPU -- compute partitions share the PCI function and report that
device's counters, so the max over a GPU's partitions counts once:

* unhealthy when uncorrectable ECC errors > ``gpu_max_uncorrectable_ecc`` (default 0);
* unhealthy when retired VRAM pages > ``gpu_max_retired_pages``; the default (``auto``,
  -1) is the amdgpu driver's default bad-page threshold, one page per 100 MiB of VRAM
  rounded up (``RAS_BAD_PAGE_COVER`` in ``amdgpu_ras.c``): 2949 pages for 288 GiB;
* unhealthy when its PCIe link to the host trained narrower than the device supports
  (``current_link_width`` < ``max_link_width``: a badly seated card or riser halves host
  transfers; the link *speed* is not judged, power management lowers it at idle);
* a counter the platform does not report is not judged.

What happens to an unhealthy node is the cluster's ``gpu_health`` setting:

``fail`` (default)  its bootstrap fails with the reasons (like a failed burn-in);
``taint``           it joins with :data:`HEALTH_TAINT` (``NoSchedule``): the device plugin
                    (which does not tolerate it) never advertises its GPUs, so no GPU pod
                    lands there; the readiness waiter leaves it out of the GPU and RCCL
                    checks and reports it;
``off``             not checked.

``triton-kubernetes health cluster`` re-reads every MI355X node and (``health_taint``)
adds or removes the taint through Rancher's Kubernetes API (``workflows/health.py``).
"""

from typing import Any, Dict, List, Optional

from ..errors import ConfigError

POLICIES = ("fail", "taint", "off")
HEALTH_TAINT = {"key": "amd.com/gpu-health", "value": "unhealthy", "effect": "NoSchedule"}
HEALTH_LABEL = "amd.com/gpu.health"
BAD_PAGE_COVER_MIB = 100  # amdgpu: "typical ECC bad page rate is 1 bad page per 100MB VRAM"


def policy_of(cfg: Dict[str, Any]) -> str:
    p = str(cfg.get("gpu_health") or "fail").lower()
    if p not in POLICIES:
        raise ConfigError(f"gpu_health must be one of {', '.join(POLICIES)}. Found '{p}'.")
    return p


def limits_of(cfg: Dict[str, Any]) -> "tuple[int, int]":
    """``(max_uncorrectable, max_bad_pages)`` from a node config; -1 bad pages = auto."""
    def num(key: str, default: int, auto: bool = False) -> int:
        raw = cfg.get(key)
        if raw is None or raw == "":
            return default
        if auto and str(raw).lower() == "auto":
            return -1
        try:
            v = int(str(raw))
        except ValueError:
            v = -2
        if v < (-1 if auto else 0):
            raise ConfigError(f"{key} must be a non-negative integer{' or auto' if auto else ''}. Found '{raw}'.")
        return v

    return num("gpu_max_uncorrectable_ecc", 0), num("gpu_max_retired_pages", -1, auto=True)


def physical_gpus(doc: Dict[str, Any]) -> List[Dict[str, Any]]:
    """One entry per physical GPU (distinct PCI function), in order of first appearance;
    counters are the max over its partitions (-1: not reported)."""
    out: List[Dict[str, Any]] = []
    at: Dict[str, int] = {}
    for i, g in enumerate(doc.get("gpus") or []):
        key = g.get("bdf") or f"#{i}"
        if key not in at:
            at[key] = len(out)
            out.append({"bdf": g.get("bdf", ""), "has_ecc": False, "ecc_uncorrectable": 0, "ecc_correctable": 0,
                        "vram_mb": 0, "bad_pages": -1, "bad_pages_pending": -1, "pcie_width": -1,
                        "pcie_max_width": -1})
        p = out[at[key]]
        p["has_ecc"] = p["has_ecc"] or "ecc_uncorrectable" in g
        p["ecc_uncorrectable"] = max(p["ecc_uncorrectable"], int(g.get("ecc_uncorrectable", 0) or 0))
        p["ecc_correctable"] = max(p["ecc_correctable"], int(g.get("ecc_correctable", 0) or 0))
        p["vram_mb"] = max(p["vram_mb"], int(g.get("vram_mb", 0) or 0))
        p["bad_pages"] = max(p["bad_pages"], int(g.get("bad_pages", -1)))
        p["bad_pages_pending"] = max(p["bad_pages_pending"], int(g.get("bad_pages_pending", -1)))
        p["pcie_width"] = max(p["pcie_width"], int(g.get("pcie_width", -1)))
        p["pcie_max_width"] = max(p["pcie_max_width"], int(g.get("pcie_max_width", -1)))
    return out


def bad_page_limit(p: Dict[str, Any], max_bad: int) -> int:
    if max_bad >= 0:
        return max_bad
    return (p["vram_mb"] + BAD_PAGE_COVER_MIB - 1) // BAD_PAGE_COVER_MIB if p["vram_mb"] else -1


def evaluate(doc: Dict[str, Any], max_uncorrectable: int = 0, max_bad_pages: int = -1) -> Dict[str, Any]:
    """The node's health verdict (same document as ``amdgpu-topo-labeller --health``)."""
    reasons: List[str] = []
    gpus: List[Dict[str, Any]] = []
    for i, p in enumerate(physical_gpus(doc)):
        limit = bad_page_limit(p, max_bad_pages)
        who = f"GPU {i}" + (f" ({p['bdf']})" if p["bdf"] else "")
        ok = True
        if p["has_ecc"] and p["ecc_uncorrectable"] > max_uncorrectable:
            reasons.append(f"{who}: {p['ecc_uncorrectable']} uncorrectable ECC errors (max {max_uncorrectable})")
            ok = False
        if p["bad_pages"] >= 0 and limit >= 0 and p["bad_pages"] > limit:
            reasons.append(f"{who}: {p['bad_pages']} retired VRAM pages (max {limit})")
            ok = False
        if 0 < p["pcie_width"] < p["pcie_max_width"]:
            reasons.append(f"{who}: PCIe link trained at x{p['pcie_width']}, the device supports x{p['pcie_max_width']}")
            ok = False
        g: Dict[str, Any] = {"gpu": i, "bdf": p["bdf"], "ok": ok}
        if p["has_ecc"]:
            g.update(ecc_uncorrectable=p["ecc_uncorrectable"], ecc_correctable=p["ecc_correctable"])
        if p["bad_pages"] >= 0:
            g.update(bad_pages=p["bad_pages"], bad_pages_pending=p["bad_pages_pending"])
        if limit >= 0:
            g["bad_page_limit"] = limit
        if p["pcie_width"] >= 0:
            g["pcie_width"] = p["pcie_width"]
        if p["pcie_max_width"] >= 0:
            g["pcie_max_width"] = p["pcie_max_width"]
        gpus.append(g)
    return {"status": "unhealthy" if reasons else "healthy", "max_uncorrectable": max_uncorrectable,
            "max_bad_pages": max_bad_pages if max_bad_pages >= 0 else "auto",
            "unhealthy_gpus": sum(not g["ok"] for g in gpus), "reasons": reasons, "gpus": gpus}


def health_labels(verdict: Dict[str, Any]) -> Dict[str, str]:
    return {HEALTH_LABEL: verdict["status"], "amd.com/gpu.unhealthy-count": str(verdict["unhealthy_gpus"])}


def ras_labels(gpus: List[Dict[str, Any]]) -> Dict[str, str]:
    """The RAS / link labels over physical GPUs -- :func:`physical_gpus` entries or a
    verdict's ``gpus`` (a counter a GPU does not report is absent or -1)."""
    labels = {"amd.com/gpu.ecc-uncorrectable": str(sum(max(0, int(p.get("ecc_uncorrectable", 0))) for p in gpus))}
    if any(int(p.get("bad_pages", -1)) >= 0 for p in gpus):
        labels["amd.com/gpu.bad-pages"] = str(sum(max(0, int(p.get("bad_pages", -1))) for p in gpus))
    widths = [int(p["pcie_width"]) for p in gpus if int(p.get("pcie_width", -1)) > 0]
    if widths:
        labels["amd.com/gpu.pcie-width"] = str(min(widths))  # the narrowest GPU link to the host
    return labels


def has_health_taint(node: Dict[str, Any]) -> bool:
    """A Kubernetes Node object carrying :data:`HEALTH_TAINT`."""
    return any(t.get("key") == HEALTH_TAINT["key"] for t in ((node.get("spec") or {}).get("taints") or []))


def taint_flag(taint: Optional[Dict[str, str]] = None) -> str:
    """``key=value:Effect``: the form the Rancher agents' ``--taints`` take."""
    t = taint or HEALTH_TAINT
    return f"{t['key']}={t['value']}:{t['effect']}"


__all__ = ["POLICIES", "HEALTH_TAINT", "HEALTH_LABEL", "policy_of", "limits_of", "physical_gpus", "evaluate",
           "health_labels", "ras_labels", "has_health_taint", "taint_flag", "bad_page_limit"]
