"""``health cluster``: re-read every MI355X node's GPU health and (optionally) fence it.

Day-2 side of the bring-up health policy (``node/health.py``).  For each MI355X node of
the cluster, with the limits its node module was created with (``gpu_max_uncorrectable_ecc``,
``gpu_max_retired_pages``; the same settings given here override them):

* agent nodes (``agent+URL``): ``GET /v1/health`` on the node agent;
* SSH / Terraform nodes: ``amdgpu-topo-labeller --health`` over the host transport (exit 3
  means unhealthy, not a transport failure).

The verdicts are printed as one JSON line per node, then a summary.  With
``health_taint: true`` the CLI also reconciles each node through Rancher's Kubernetes API:
an unhealthy node gets :data:`~..node.health.HEALTH_TAINT` (``NoSchedule``: no new GPU
pods; a device plugin already running there keeps running, as Kubernetes does for
``NoSchedule``) and the ``amd.com/gpu.health`` label; a node that is healthy again has the
taint removed.  The RAS labels the bootstrap labeller set (``amd.com/gpu.ecc-uncorrectable``,
``.bad-pages``, ``.pcie-width``, ``.unhealthy-count``) are refreshed from the same verdict.  ``triton-kubernetes health cluster`` exits 0 either way; the verdict is
in the output (``unhealthy: N``).

``health_taint_effect: NoExecute`` (default ``NoSchedule``) also evicts the pods already
running on an unhealthy node -- GPU jobs and the device plugin, so the node's
``amd.com/gpu`` drops to 0 -- for a GPU that started logging uncorrectable errors under a
running job; pods that tolerate the taint stay.

``health_labels: true`` refreshes the health and RAS labels only (no taint is added or
removed), for clusters whose taints another controller owns.

Settings: ``cluster_manager``, ``cluster_name``, ``health_taint`` (default false), ``health_labels``,
``health_taint_effect`` (``NoSchedule`` | ``NoExecute``),
``gpu_max_uncorrectable_ecc`` / ``gpu_max_retired_pages`` (override the node modules').
"""

import json
import shlex
from typing import Any, Dict, List

from ..backend.base import Backend
from ..config.context import Context
from ..errors import ConfigError, TKError
from ..node.health import HEALTH_TAINT, has_health_taint, health_labels, limits_of, ras_labels
from ..node.plan import TOOLS_DIR
from ..parallel.transport import HostRef
from ..terraform.catalog import module_from_source
from .select import select_cluster, select_manager


def _limits(ctx: Context, cfg: Dict[str, Any]) -> "tuple[int, int]":
    merged = dict(cfg)
    for k in ("gpu_max_uncorrectable_ecc", "gpu_max_retired_pages"):
        if ctx.is_set(k):
            merged[k] = ctx.get_string(k)
    return limits_of(merged)


def _probe(ctx: Context, state, host: str, cfg: Dict[str, Any]) -> Dict[str, Any]:
    max_ue, max_bad = _limits(ctx, cfg)
    addr = str(cfg.get("host", ""))
    if addr.startswith("agent+"):
        from ..readiness.waiter import agent_transport_for

        doc = agent_transport_for(ctx, state.name).get(HostRef(addr), "/v1/health",
                                                          {"max_uncorrectable": max_ue, "max_bad_pages": max_bad})
    else:
        from ..parallel.transport import TransportRouter

        transport = ctx.extras.get("transport") or TransportRouter()
        tools = ctx.get_string("node_tools_dir") or TOOLS_DIR
        bad = "auto" if max_bad < 0 else str(max_bad)
        script = (f"{shlex.quote(tools + '/amdgpu-topo-labeller')} --health --max-uncorrectable {max_ue} "
                  f"--max-bad-pages {bad}; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ]")
        ref = HostRef(addr, cfg.get("ssh_user") or "ubuntu", cfg.get("key_path") or "", cfg.get("bastion_host") or "")
        out = transport.run_script(ref, script, timeout=120)
        line = next((ln for ln in reversed(out.splitlines()) if ln.startswith("{")), "")
        if not line:
            raise TKError(f"{host}: the labeller printed no health verdict")
        doc = json.loads(line)
    doc["node"] = host
    return doc


EFFECTS = ("NoSchedule", "NoExecute")


def _effect(ctx: Context) -> str:
    raw = ctx.get_string("health_taint_effect") if ctx.is_set("health_taint_effect") else "NoSchedule"
    match = {e.lower(): e for e in EFFECTS}.get(str(raw).lower())
    if match is None:
        raise ConfigError(f"health_taint_effect must be one of {', '.join(EFFECTS)}. Found '{raw}'.")
    return match


CONFLICT_RETRIES = 5


def _reconcile(client, cluster_id: str, node: Dict[str, Any], verdict: Dict[str, Any],
               effect: str = "NoSchedule", fence: bool = True) -> str:
    """Add / remove the health taint (``fence``) and set the labels; returns what changed
    ('' = nothing).

    ``spec.taints`` can only be replaced whole, so the patch carries the node's
    ``metadata.resourceVersion``: a taint another controller added since the node was read
    (the node-lifecycle controller's ``node.kubernetes.io/unreachable``, another operator's)
    makes the API server answer 409, and the node is read again and the taints recomputed
    from it, instead of being silently dropped."""
    from ..cloud.http import HTTPError

    name = node["metadata"]["name"]
    for _ in range(CONFLICT_RETRIES):
        try:
            return _reconcile_once(client, cluster_id, node, verdict, effect, fence)
        except HTTPError as exc:
            if exc.status != 409:
                raise
            fresh = next((n for n in client.k8s_nodes(cluster_id) if n["metadata"]["name"] == name), None)
            if fresh is None:
                raise TKError(f"node {name} is gone from the cluster") from exc
            node = fresh
    raise TKError(f"node {name} kept changing while its health taint was updated; run health cluster again")


def _reconcile_once(client, cluster_id: str, node: Dict[str, Any], verdict: Dict[str, Any],
                    effect: str, fence: bool) -> str:
    name = node["metadata"]["name"]
    want = health_labels(verdict)
    want.update(ras_labels(verdict.get("gpus") or []))
    have = (node.get("metadata") or {}).get("labels") or {}
    if not fence:
        if all(have.get(k) == v for k, v in want.items()):
            return ""
        client.patch_node(cluster_id, name, {"metadata": {"labels": want}})
        return "labelled"
    current = [t for t in (node.get("spec") or {}).get("taints") or [] if t.get("key") == HEALTH_TAINT["key"]]
    taints = [t for t in (node.get("spec") or {}).get("taints") or [] if t.get("key") != HEALTH_TAINT["key"]]
    unhealthy = verdict["status"] != "healthy"
    if unhealthy:
        taints.append(dict(HEALTH_TAINT, effect=effect))
    tainted = has_health_taint(node)
    same_effect = not unhealthy or [t.get("effect") for t in current] == [effect]
    if tainted == unhealthy and same_effect and all(have.get(k) == v for k, v in want.items()):
        return ""
    meta: Dict[str, Any] = {"labels": want}
    rv = (node.get("metadata") or {}).get("resourceVersion")
    if rv:
        meta["resourceVersion"] = rv  # a precondition: 409 if the node changed since it was read
    client.patch_node(cluster_id, name, {"metadata": meta, "spec": {"taints": taints}})
    if tainted and unhealthy and not same_effect:
        return f"tainted {effect}"
    if tainted == unhealthy:
        return "labelled"
    return "tainted" if unhealthy else "untainted"


def cluster_health(ctx: Context, backend: Backend) -> List[Dict[str, Any]]:
    managers = backend.states()
    if not managers:
        raise ConfigError("No cluster managers.")
    state = backend.state(select_manager(ctx, managers))
    name, key = select_cluster(ctx, state.clusters(), "Cluster to check")
    nodes = state.nodes(key)
    gpu_hosts = {}
    for host in sorted(nodes):
        cfg = state.module(nodes[host]) or {}
        info = module_from_source(str(cfg.get("source", "")))
        if info is not None and info.mi355x:
            gpu_hosts[host] = cfg
    if not gpu_hosts:
        ctx.echo(f"cluster '{name}' has no MI355X nodes")
        return []
    from ..parallel.fanout import shared_pool

    futs = {h: shared_pool("tk-health", 32).submit(_probe, ctx, state, h, cfg) for h, cfg in gpu_hosts.items()}
    verdicts = []
    for h, f in futs.items():
        try:
            verdicts.append(f.result())
        except Exception as exc:  # noqa: BLE001 - an unreachable node is reported, not fatal
            verdicts.append({"node": h, "status": "unknown", "reasons": [f"{type(exc).__name__}: {exc}"],
                             "gpus": []})
    fence = ctx.settings.get_bool("health_taint") if ctx.is_set("health_taint") else False
    relabel = ctx.settings.get_bool("health_labels") if ctx.is_set("health_labels") else False
    if fence or relabel:
        effect = _effect(ctx) if fence else "NoSchedule"
        from ..readiness.waiter import spec_from_state

        client, spec = spec_from_state(state, backend, key)
        k8s = {n["metadata"]["name"]: n for n in client.k8s_nodes(spec.cluster_id)}
        for v in verdicts:
            if v["status"] == "unknown" or v["node"] not in k8s:
                v["taint"] = "skipped"
                continue
            v["taint"] = _reconcile(client, spec.cluster_id, k8s[v["node"]], v, effect, fence) or "unchanged"
    for v in verdicts:
        ctx.echo(json.dumps({k: v.get(k) for k in ("node", "status", "reasons", "taint") if k in v}, sort_keys=True))
    bad = [v["node"] for v in verdicts if v["status"] == "unhealthy"]
    unknown = [v["node"] for v in verdicts if v["status"] == "unknown"]
    ctx.echo(f"cluster '{name}': {len(verdicts)} MI355X node(s), unhealthy: {len(bad)}"
             + (f" ({', '.join(bad)})" if bad else "") + (f", unreachable: {', '.join(unknown)}" if unknown else ""))
    return verdicts


__all__ = ["cluster_health"]
