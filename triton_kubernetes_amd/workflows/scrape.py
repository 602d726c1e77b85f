"""``get scrape-config``: Prometheus ``scrape_configs`` for a cluster's MI355X nodes.

Each MI355X node exposes its metrics (``node/metrics.py``) one of two ways, and the
generated jobs follow what the node module says:

* a node managed by the node agent (``host: agent+https://...``): ``GET /metrics`` on the
  agent, HTTPS verified against the cluster manager's agent CA, authorised with *that
  node's* token (tokens are per node, so one job per node);
* an SSH / Terraform node with ``gpu_metrics_textfile``: node_exporter's textfile
  collector on the node (``<host>:9100``, ``node_exporter_port``), one job for all of them.

The CA and the tokens are written to ``metrics_secrets_dir`` (files ``0600``; the jobs
reference them through ``ca_file`` / ``credentials_file``, so no secret is printed).  The
YAML goes to stdout after the command's breadcrumb line, or to ``scrape_config_file``,
ready to merge under ``scrape_configs:``.

Settings: ``cluster_manager``, ``cluster_name``, ``metrics_secrets_dir`` (required when the
cluster has agent nodes), ``node_exporter_port`` (9100), ``scrape_config_file``.
"""

import os
import urllib.parse
from typing import Any, Dict, List

from ..backend.base import Backend
from ..config.context import Context
from ..errors import ConfigError
from ..terraform.catalog import module_from_source
from .select import select_cluster, select_manager


def _write_secret(path: str, data: str) -> None:
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    with os.fdopen(fd, "w", encoding="utf-8") as fh:
        fh.write(data)
    os.chmod(path, 0o600)


def scrape_config(ctx: Context, backend: Backend) -> List[Dict[str, Any]]:
    import yaml

    from ..node.security import agent_address, load_pki, metrics_token

    managers = backend.states()
    if not managers:
        raise ConfigError("No cluster managers.")
    manager = select_manager(ctx, managers)
    state = backend.state(manager)
    name, key = select_cluster(ctx, state.clusters(), "Cluster to scrape")
    agents, textfile = [], []
    for host, mkey in sorted(state.nodes(key).items()):
        cfg = state.module(mkey) or {}
        info = module_from_source(str(cfg.get("source", "")))
        if info is None or not info.mi355x:
            continue
        addr = str(cfg.get("host", ""))
        if addr.startswith("agent+"):
            agents.append((host, addr[len("agent+"):]))
        elif cfg.get("gpu_metrics_textfile") and addr:
            textfile.append((host, agent_address(addr)))
    jobs: List[Dict[str, Any]] = []
    if agents:
        secrets_dir = ctx.settings.get_string("metrics_secrets_dir")
        if not secrets_dir:
            raise ConfigError("metrics_secrets_dir is required: the agent CA and each node's token are written there")
        secrets_dir = os.path.expanduser(secrets_dir)
        os.makedirs(secrets_dir, mode=0o700, exist_ok=True)
        shared = ctx.settings.get_string("agent_token")  # development clusters with one shared token
        pki = load_pki(backend, manager, create=False)
        if pki is None and not shared:
            raise ConfigError(f"cluster manager '{manager}' has no agent PKI")
        ca_file = os.path.join(secrets_dir, f"{manager}-agent-ca.pem")
        if pki is not None:
            _write_secret(ca_file, pki.ca_cert)
        for host, url in agents:
            u = urllib.parse.urlsplit(url)
            token_file = os.path.join(secrets_dir, f"{manager}-{name}-{host}.token")
            # the node's read-only scrape token, never its agent token (which can post plans)
            _write_secret(token_file, metrics_token(shared or pki.node_token(agent_address(url))))
            job: Dict[str, Any] = {
                "job_name": f"tk-{name}-{host}", "scheme": u.scheme or "https", "metrics_path": "/metrics",
                "authorization": {"type": "Bearer", "credentials_file": token_file},
                "static_configs": [{"targets": [u.netloc], "labels": {"cluster": name, "tk_node": host}}]}
            if (u.scheme or "https") == "https" and pki is not None:
                job["tls_config"] = {"ca_file": ca_file, "server_name": agent_address(url)}
            jobs.append(job)
    if textfile:
        port = ctx.settings.get_int_or("node_exporter_port", 9100)
        jobs.append({"job_name": f"tk-{name}-node-exporter",
                     "static_configs": [{"targets": [f"{a}:{port}"], "labels": {"cluster": name, "tk_node": h}}
                                        for h, a in textfile]})
    if not jobs:
        ctx.echo(f"# cluster '{name}' has no MI355X node exposing metrics (agent nodes, or gpu_metrics_textfile)")
        return []
    text = yaml.safe_dump(jobs, sort_keys=False)
    dest = ctx.settings.get_string("scrape_config_file")
    if dest:
        with open(os.path.expanduser(dest), "w", encoding="utf-8") as fh:
            fh.write(text)
        ctx.echo(f"wrote {len(jobs)} scrape job(s) to {dest}")
    else:
        ctx.echo(text.rstrip())
    return jobs


__all__ = ["scrape_config"]


# --- alert rules --------------------------------------------------------------------------
ALERTS: List[Dict[str, Any]] = [
    {"alert": "TkGpuUnhealthy", "expr": "tk_gpu_healthy == 0", "for": "5m",
     "labels": {"severity": "critical"},
     "annotations": {"summary": "GPU {{ $labels.gpu }} ({{ $labels.bdf }}) on {{ $labels.node }} fails the health rules",
                     "runbook": "triton-kubernetes health cluster (health_taint: true) fences the node"}},
    {"alert": "TkGpuUncorrectableEcc", "expr": "increase(tk_gpu_ecc_uncorrectable_errors[1h]) > 0",
     "labels": {"severity": "critical"},
     "annotations": {"summary": "GPU {{ $labels.gpu }} on {{ $labels.node }} logged uncorrectable ECC errors"}},
    {"alert": "TkGpuRetiredPagesNearLimit", "expr": "tk_gpu_retired_pages > 0.8 * tk_gpu_retired_pages_limit",
     "for": "15m", "labels": {"severity": "warning"},
     "annotations": {"summary": "GPU {{ $labels.gpu }} on {{ $labels.node }} retired over 80% of its VRAM page budget"}},
    {"alert": "TkGpuPcieLinkDegraded", "expr": "tk_gpu_pcie_link_width < tk_gpu_pcie_link_max_width", "for": "5m",
     "labels": {"severity": "warning"},
     "annotations": {"summary": "GPU {{ $labels.gpu }} on {{ $labels.node }} runs x{{ $value }} below its PCIe width"}},
    {"alert": "TkNodeBringupFailed", "expr": "tk_bringup_success == 0", "labels": {"severity": "warning"},
     "annotations": {"summary": "the last bootstrap of {{ $labels.node }} failed"}},
    {"alert": "TkAgentGpuReadFailing", "expr": "tk_agent_gpu_collect_success == 0", "for": "10m",
     "labels": {"severity": "warning"},
     "annotations": {"summary": "the node agent on {{ $labels.node }} cannot read its GPUs' RAS counters"}},
]


def alert_rules(ctx: Context, backend: Backend) -> Dict[str, Any]:
    """``get alert-rules``: a Prometheus rule file over the node metrics (no cluster state
    needed; ``alert_rules_file`` writes it to a file)."""
    import yaml

    doc = {"groups": [{"name": "triton-kubernetes-mi355x", "rules": ALERTS}]}
    text = yaml.safe_dump(doc, sort_keys=False)
    dest = ctx.settings.get_string("alert_rules_file")
    if dest:
        with open(os.path.expanduser(dest), "w", encoding="utf-8") as fh:
            fh.write(text)
        ctx.echo(f"wrote {len(ALERTS)} alert rule(s) to {dest}")
    else:
        ctx.echo(text.rstrip())
    return doc


__all__ += ["alert_rules", "ALERTS"]
