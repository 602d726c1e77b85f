"""``get manager|cluster`` (reference ``get/manager.go``, ``get/cluster.go``),
plus ``get nodes``.

``manager`` / ``cluster`` print the module outputs: ``rancher_url`` /
``rancher_access_key`` / ``rancher_secret_key`` for the manager, the cluster id /
registration token / CA checksum (+ provider network ids) for a cluster.  With
Terraform < 0.12 this is exactly ``terraform output -module <key>``; otherwise the
executor reads the root outputs it rendered, or the DirectExecutor's tfstate.

``nodes`` (new) lists the cluster's Kubernetes nodes as the cluster sees them, read
through Rancher's Kubernetes API with the manager's keys: Ready, roles, and for MI355X
nodes the GPUs (allocatable ``amd.com/gpu`` of the labeller's count), product and
partition mode, burn-in level, xGMI link check and GPU health (taint) -- one table, or
one JSON object per node with ``output: json``.
"""

import json
from typing import Any, Dict, List

from ..backend.base import Backend
from ..config.context import Context
from ..errors import ConfigError
from ..state import MANAGER_KEY
from .select import executor_for, select_cluster, select_manager

NODE_COLUMNS = ("NAME", "READY", "ROLES", "VERSION", "GPUS", "PRODUCT", "PARTITION", "BURN-IN", "XGMI", "PCIE", "UE/PAGES",
                "HEALTH")


def get_manager(ctx: Context, backend: Backend) -> None:
    managers = backend.states()
    if not managers:
        raise ConfigError("No cluster managers.")
    manager = select_manager(ctx, managers)
    state = backend.state(manager)
    executor_for(ctx, state, backend).print_outputs(state, backend, MANAGER_KEY, ctx.out)


def get_cluster(ctx: Context, backend: Backend) -> None:
    managers = backend.states()
    if not managers:
        raise ConfigError("No cluster managers.")
    manager = select_manager(ctx, managers)
    state = backend.state(manager)
    clusters = state.clusters()
    if not clusters:
        raise ConfigError("No clusters.")
    _, key = select_cluster(ctx, clusters, "Cluster to view")
    executor_for(ctx, state, backend).print_outputs(state, backend, key, ctx.out)


def _node_row(item: Dict[str, Any]) -> Dict[str, str]:
    from ..node.health import HEALTH_LABEL, HEALTH_TAINT, has_health_taint

    meta, status = item.get("metadata") or {}, item.get("status") or {}
    labels = meta.get("labels") or {}
    ready = next((c.get("status") for c in status.get("conditions") or [] if c.get("type") == "Ready"), "Unknown")
    roles = sorted(k.rsplit("/", 1)[1] for k, v in labels.items()
                   if k.startswith("node-role.kubernetes.io/") and v in ("true", ""))
    gpu = labels.get("amd.com/gpu.present") == "true"
    row = {"NAME": meta.get("name", ""), "READY": "Ready" if ready == "True" else "NotReady",
           "ROLES": ",".join(roles) or "-",
           "VERSION": (status.get("nodeInfo") or {}).get("kubeletVersion") or "-"}
    if gpu:
        alloc = (status.get("allocatable") or {}).get("amd.com/gpu", "0")
        row["GPUS"] = f"{alloc}/{labels.get('amd.com/gpu.logical-count', labels.get('amd.com/gpu.count', '?'))}"
        row["PRODUCT"] = labels.get("amd.com/gpu.product-name", "-")
        row["PARTITION"] = "/".join(x for x in (labels.get("amd.com/gpu.compute-partition"),
                                                 labels.get("amd.com/gpu.memory-partition")) if x) or "-"
        row["BURN-IN"] = (f"{labels.get('amd.com/gpu.burnin', '-')}({labels['amd.com/gpu.burnin-level']})"
                          if "amd.com/gpu.burnin-level" in labels else labels.get("amd.com/gpu.burnin", "-"))
        row["XGMI"] = labels.get("amd.com/xgmi.link-check") or (
            "mesh" if labels.get("amd.com/xgmi.fully-connected") == "true" else "-")
        row["PCIE"] = f"x{labels['amd.com/gpu.pcie-width']}" if "amd.com/gpu.pcie-width" in labels else "-"
        row["UE/PAGES"] = (f"{labels.get('amd.com/gpu.ecc-uncorrectable', '-')}/"
                           f"{labels.get('amd.com/gpu.bad-pages', '-')}")
        health = labels.get(HEALTH_LABEL, "-")
        effects = [t.get("effect") for t in (item.get("spec") or {}).get("taints") or []
                   if t.get("key") == HEALTH_TAINT["key"]]
        row["HEALTH"] = health + (",tainted" if has_health_taint(item) else "") + (
            ",evicting" if "NoExecute" in effects else "")
    else:
        row.update({c: "-" for c in NODE_COLUMNS[4:]})
    return row


def get_nodes(ctx: Context, backend: Backend) -> List[Dict[str, str]]:
    managers = backend.states()
    if not managers:
        raise ConfigError("No cluster managers.")
    manager = select_manager(ctx, managers)
    state = backend.state(manager)
    clusters = state.clusters()
    if not clusters:
        raise ConfigError("No clusters.")
    name, key = select_cluster(ctx, clusters, "Cluster to view")
    executor = executor_for(ctx, state, backend)
    mgr, cl = executor.outputs(state, backend, MANAGER_KEY), executor.outputs(state, backend, key)
    if not mgr.get("rancher_url") or not cl.get("rancher_cluster_id"):
        raise ConfigError(f"Cluster '{name}' has no Rancher outputs yet (was it applied?)")
    from ..rancher import trust

    factory = ctx.extras.get("rancher_factory") or (  # verified against the pinned CA (rancher/trust.py)
        lambda url, ak="", sk="": trust.client(backend, state.name, url, ak, sk))
    client = factory(mgr["rancher_url"], mgr.get("rancher_access_key", ""), mgr.get("rancher_secret_key", ""))
    items = sorted(client.k8s_nodes(cl["rancher_cluster_id"]), key=lambda i: (i.get("metadata") or {}).get("name", ""))
    rows = [_node_row(i) for i in items]
    if (ctx.settings.get_string("output") or "").lower() == "json":
        for r in rows:
            ctx.echo(json.dumps(r, sort_keys=True))
        return rows
    widths = {c: max([len(c)] + [len(r[c]) for r in rows]) for c in NODE_COLUMNS}
    ctx.echo("  ".join(c.ljust(widths[c]) for c in NODE_COLUMNS).rstrip())
    for r in rows:
        ctx.echo("  ".join(r[c].ljust(widths[c]) for c in NODE_COLUMNS).rstrip())
    from ..readiness.waiter import gpu_mismatch

    labels = {(i.get("metadata") or {}).get("name", ""): (i.get("metadata") or {}).get("labels") or {} for i in items}
    for key, by in sorted(gpu_mismatch(labels).items()):
        ctx.echo(f"warning: MI355X nodes differ in {key}: "
                 + "; ".join(f"{v}: {', '.join(ns)}" for v, ns in sorted(by.items())))
    return rows
