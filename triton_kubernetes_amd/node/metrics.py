"""Prometheus metrics of an MI355X node: RAS counters, PCIe link, bring-up and burn-in.

The reference has no metrics at all ("None beyond stdout"); a fleet of
MI355X nodes is watched by Prometheus, so each node exposes what its bring-up measured and
what its GPUs report now, in the text exposition format (version 0.0.4):

* the node agent serves it at ``GET /metrics`` (``node/agent_http.py``; the agent token as
  ``Authorization: Bearer`` -- Prometheus' ``authorization`` scrape setting -- or
  ``X-TK-Agent-Token``);
* SSH / Terraform nodes: ``amdgpu-topo-labeller --prom`` prints the GPU families
  (``ops/csrc/tk_topo.cpp``, same names and samples: tests compare both) for
  node_exporter's textfile collector.

GPU families come from the health verdict (``node/health.py:evaluate``), one sample per
**physical** GPU (``gpu`` = its index among physical GPUs, ``bdf`` its PCI address):

=====================================  ======================================================
``tk_gpu_healthy``                     1 healthy, 0 unhealthy (the bring-up policy's rules)
``tk_gpu_ecc_uncorrectable_errors``    uncorrectable ECC errors (RAS blocks summed)
``tk_gpu_ecc_correctable_errors``      correctable ECC errors
``tk_gpu_retired_pages``               retired VRAM pages; ``..._pending``: pending retirement
``tk_gpu_retired_pages_limit``         the bad-page limit the verdict used
``tk_gpu_pcie_link_width``             trained PCIe lanes; ``..._max_width``: the device's
``tk_node_unhealthy_gpus``             unhealthy physical GPUs on the node
=====================================  ======================================================

Bring-up families (agent only, from its last plan): ``tk_bringup_duration_seconds``,
``tk_bringup_success``, ``tk_bringup_step_duration_seconds{step}``,
``tk_bringup_step_success{step}``, ``tk_gpu_burnin{gpu,check,metric}`` (every number the
burn-in measured: HBM GB/s, MFMA / GEMM TFLOP/s, memtest bytes), ``tk_rccl_local_busbw_gbps``
(node all-reduce peak bus bandwidth) and ``tk_xgmi_p2p_{min,median}_gbps`` (link matrix).
"""

import re
from typing import Any, Dict, List, Optional, Tuple

# name -> (type, help); order = exposition order
GPU_FAMILIES: List[Tuple[str, str, str]] = [
    ("tk_gpu_healthy", "gauge", "1 if the GPU passes the node's health rules, else 0"),
    ("tk_gpu_ecc_uncorrectable_errors", "gauge", "Uncorrectable ECC errors, summed over RAS blocks"),
    ("tk_gpu_ecc_correctable_errors", "gauge", "Correctable ECC errors, summed over RAS blocks"),
    ("tk_gpu_retired_pages", "gauge", "Retired VRAM pages (driver bad-page records)"),
    ("tk_gpu_retired_pages_pending", "gauge", "VRAM pages pending retirement"),
    ("tk_gpu_retired_pages_limit", "gauge", "Retired-page limit of the health rules"),
    ("tk_gpu_pcie_link_width", "gauge", "Trained PCIe link width (lanes)"),
    ("tk_gpu_pcie_link_max_width", "gauge", "PCIe link width the device supports (lanes)"),
    ("tk_node_unhealthy_gpus", "gauge", "Unhealthy physical GPUs on the node"),
]
# verdict gpu field -> family
_GPU_FIELDS = [("ecc_uncorrectable", "tk_gpu_ecc_uncorrectable_errors"),
               ("ecc_correctable", "tk_gpu_ecc_correctable_errors"),
               ("bad_pages", "tk_gpu_retired_pages"), ("bad_pages_pending", "tk_gpu_retired_pages_pending"),
               ("bad_page_limit", "tk_gpu_retired_pages_limit"), ("pcie_width", "tk_gpu_pcie_link_width"),
               ("pcie_max_width", "tk_gpu_pcie_link_max_width")]

BRINGUP_FAMILIES: List[Tuple[str, str, str]] = [
    ("tk_agent_info", "gauge", "Node agent (always 1; labels: node, mode)"),
    ("tk_agent_gpu_collect_success", "gauge", "1 if the agent read the GPUs' RAS counters for this scrape"),
    ("tk_node_gpu_info", "gauge", "Always 1; labels: the node's GPU product, VBIOS, ROCm, partition modes, power cap"),
    ("tk_bringup_duration_seconds", "gauge", "Wall time of the node's last bootstrap plan"),
    ("tk_bringup_success", "gauge", "1 if the node's last bootstrap plan succeeded"),
    ("tk_bringup_step_duration_seconds", "gauge", "Wall time of each step of the last bootstrap plan"),
    ("tk_bringup_step_success", "gauge", "1 if the step succeeded"),
    ("tk_gpu_burnin", "gauge", "Burn-in measurements of the last bootstrap (GB/s, TFLOP/s, bytes)"),
    ("tk_rccl_local_busbw_gbps", "gauge", "Peak all-reduce bus bandwidth over the node's GPUs (GB/s)"),
    ("tk_xgmi_p2p_min_gbps", "gauge", "Slowest GPU pair of the peer-to-peer link matrix (GB/s)"),
    ("tk_xgmi_p2p_median_gbps", "gauge", "Median GPU pair of the peer-to-peer link matrix (GB/s)"),
]


def _esc(v: Any) -> str:
    return str(v).replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


def _num(v: float) -> str:
    if isinstance(v, bool):
        return "1" if v else "0"
    if isinstance(v, int) or float(v).is_integer():
        return str(int(v))
    return repr(float(v))


class Exposition:
    """Samples grouped by family, rendered with one HELP/TYPE header per family."""

    def __init__(self, families: List[Tuple[str, str, str]]):
        self.meta = {name: (typ, hlp) for name, typ, hlp in families}
        self.samples: Dict[str, List[Tuple[Dict[str, str], float]]] = {name: [] for name, _, _ in families}

    def add(self, name: str, value: float, **labels: Any) -> None:
        self.samples[name].append(({k: str(v) for k, v in labels.items()}, value))

    def render(self) -> str:
        out = []
        for name, rows in self.samples.items():
            if not rows:
                continue
            typ, hlp = self.meta[name]
            out.append(f"# HELP {name} {hlp}")
            out.append(f"# TYPE {name} {typ}")
            for labels, value in rows:
                lab = ",".join(f'{k}="{_esc(v)}"' for k, v in labels.items())
                out.append(f"{name}{{{lab}}} {_num(value)}" if lab else f"{name} {_num(value)}")
        return "\n".join(out) + ("\n" if out else "")


def gpu_exposition(verdict: Dict[str, Any], node: str) -> Exposition:
    exp = Exposition(GPU_FAMILIES)
    for g in verdict.get("gpus") or []:
        who = {"node": node, "gpu": g["gpu"], "bdf": g.get("bdf", "")}
        exp.add("tk_gpu_healthy", 1 if g.get("ok") else 0, **who)
        for field, family in _GPU_FIELDS:
            if field in g and int(g[field]) >= 0:
                exp.add(family, int(g[field]), **who)
    exp.add("tk_node_unhealthy_gpus", int(verdict.get("unhealthy_gpus", 0)), node=node)
    return exp


def gpu_metrics(verdict: Dict[str, Any], node: str) -> str:
    """The GPU families of a health verdict (what ``amdgpu-topo-labeller --prom`` prints)."""
    return gpu_exposition(verdict, node).render()


def _flatten(prefix: str, obj: Any) -> List[Tuple[str, float]]:
    if isinstance(obj, bool):
        return []
    if isinstance(obj, (int, float)):
        return [(prefix, obj)]
    if isinstance(obj, dict):
        out = []
        for k in sorted(obj):
            out += _flatten(f"{prefix}.{k}" if prefix else str(k), obj[k])
        return out
    return []


# node label -> info-metric label (node/labels.py)
INFO_LABELS = (("amd.com/gpu.product-name", "product"), ("amd.com/gpu.vbios", "vbios"),
               ("amd.com/rocm.version", "rocm"), ("amd.com/gpu.compute-partition", "compute_partition"),
               ("amd.com/gpu.memory-partition", "memory_partition"), ("amd.com/gpu.power-cap", "power_cap_w"))


def bringup_metrics(plan_doc: Optional[Dict[str, Any]], node: str, mode: str = "",
                    gpu_collect_ok: Optional[bool] = None, labels: Optional[Dict[str, str]] = None) -> str:
    """Families of the node's last bootstrap plan (an agent ``run_plan`` result); ``labels``:
    the node labels it set (the info metric)."""
    exp = Exposition(BRINGUP_FAMILIES)
    exp.add("tk_agent_info", 1, node=node, mode=mode)
    if labels and labels.get("amd.com/gpu.present") == "true":
        exp.add("tk_node_gpu_info", 1, node=node, **{m: labels.get(k, "") for k, m in INFO_LABELS})
    if gpu_collect_ok is not None:
        exp.add("tk_agent_gpu_collect_success", 1 if gpu_collect_ok else 0, node=node)
    if not plan_doc:
        return exp.render()
    exp.add("tk_bringup_duration_seconds", float(plan_doc.get("ms", 0.0)) / 1e3, node=node)
    exp.add("tk_bringup_success", 1 if plan_doc.get("ok") else 0, node=node)
    for s in plan_doc.get("steps") or []:
        exp.add("tk_bringup_step_duration_seconds", float(s.get("ms", 0.0)) / 1e3, node=node, step=s["name"])
        exp.add("tk_bringup_step_success", 1 if s.get("ok") else 0, node=node, step=s["name"])
        detail = s.get("detail")
        if not s.get("ok") or not isinstance(detail, dict):
            continue
        name = s["name"]
        if name == "gpu_burnin":
            for gpu, res in sorted(detail.items()):
                if not isinstance(res, dict):
                    continue
                for check in ("hbm", "mfma", "gemm", "gemm_fp8", "memtest"):
                    for metric, v in _flatten("", res.get(check) or {}):
                        exp.add("tk_gpu_burnin", v, node=node, gpu=gpu, check=check, metric=metric)
        elif name == "rccl_local" and "peak_busbw_gbps" in detail:
            exp.add("tk_rccl_local_busbw_gbps", float(detail["peak_busbw_gbps"]), node=node)
        elif name == "gpu_links":
            labels = detail.get("labels") or {}
            for key, family in (("amd.com/xgmi.p2p-min-gbps", "tk_xgmi_p2p_min_gbps"),
                                ("amd.com/xgmi.p2p-median-gbps", "tk_xgmi_p2p_median_gbps")):
                if key in labels:
                    exp.add(family, float(labels[key]), node=node)
    return exp.render()


CONTENT_TYPE = "text/plain; version=0.0.4; charset=utf-8"

__all__ = ["GPU_FAMILIES", "BRINGUP_FAMILIES", "Exposition", "gpu_metrics", "gpu_exposition", "bringup_metrics",
           "CONTENT_TYPE"]


# --- node_exporter textfile collector (SSH / Terraform nodes) ------------------------------
TEXTFILE_NAME = "tk_gpu.prom"
TEXTFILE_UNIT = "tk-gpu-metrics"
_DIR_RE = re.compile(r"^/[A-Za-z0-9._/-]+$")


def textfile_dir_of(cfg: Dict[str, Any]) -> str:
    """``gpu_metrics_textfile``: node_exporter's ``--collector.textfile.directory`` on the
    node ("" = off, the default)."""
    d = str(cfg.get("gpu_metrics_textfile") or "").strip()
    if d and (not _DIR_RE.fullmatch(d) or "/../" in d + "/"):
        from ..errors import ConfigError

        raise ConfigError(f"gpu_metrics_textfile must be an absolute directory path. Found '{d}'.")
    return d.rstrip("/") if d != "/" else d


def textfile_script(tools_dir: str, directory: str, max_ue: str, max_bad: str) -> str:
    """Bash that writes ``<directory>/tk_gpu.prom`` now and installs a systemd timer that
    rewrites it every minute (atomically: node_exporter never reads half a file).  The
    arguments are shell-safe literals or Terraform template expressions."""
    cmd = (f"{tools_dir}/amdgpu-topo-labeller --prom --max-uncorrectable {max_ue} --max-bad-pages {max_bad}"
           f" > {directory}/{TEXTFILE_NAME}.tmp && mv {directory}/{TEXTFILE_NAME}.tmp {directory}/{TEXTFILE_NAME}")
    return f"""sudo mkdir -p {directory}
sudo sh -c '{cmd}'
if command -v systemctl >/dev/null 2>&1 && [ -d /run/systemd/system ]; then
sudo tee /etc/systemd/system/{TEXTFILE_UNIT}.service >/dev/null <<'TK_UNIT_EOF'
[Unit]
Description=MI355X GPU health metrics for the node_exporter textfile collector
[Service]
Type=oneshot
ExecStart=/bin/sh -c '{cmd}'
TK_UNIT_EOF
sudo tee /etc/systemd/system/{TEXTFILE_UNIT}.timer >/dev/null <<'TK_UNIT_EOF'
[Unit]
Description=Refresh {directory}/{TEXTFILE_NAME} every minute
[Timer]
OnBootSec=30s
OnUnitActiveSec=60s
[Install]
WantedBy=timers.target
TK_UNIT_EOF
sudo systemctl daemon-reload && sudo systemctl enable --now {TEXTFILE_UNIT}.timer >/dev/null
else
echo 'gpu metrics: no systemd; {directory}/{TEXTFILE_NAME} is written once' >&2
fi"""


__all__ += ["TEXTFILE_NAME", "TEXTFILE_UNIT", "textfile_dir_of", "textfile_script"]
