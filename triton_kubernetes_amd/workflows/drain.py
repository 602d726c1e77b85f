"""Drain a node before it is destroyed (``destroy node`` with ``drain: true``).

The reference destroys a node's VM/host module and leaves whatever ran there to die with
it (``destroy/node.go:167-168``; its Rancher node object is not even removed).  Replacing
an MI355X node that runs training or serving jobs needs the ``kubectl drain`` sequence,
done through Rancher's Kubernetes API:

1. cordon: ``spec.unschedulable = true`` (no new pods);
2. evict every pod bound to the node through the Eviction API (``policy/v1``), so
   PodDisruptionBudgets are honoured: a 429 answer is retried with back-off until
   ``drain_timeout`` (default 600 s).  DaemonSet pods (the ROCm device plugin, CNI) and
   static mirror pods are left, as ``kubectl drain --ignore-daemonsets`` does;
3. wait until none of the evicted pods is bound to the node any more.

As with ``kubectl drain``, a pod no controller manages (no ``ownerReferences``) would be
gone for good once evicted: such pods stop the drain (after the cordon) unless
``drain_force: true``.

A drain that does not finish in time fails the destroy *before* anything is destroyed
(the node stays cordoned, its module and host are untouched) and names the pods left.

The same steps are day-2 commands on their own: ``drain node`` (cordon + evict, e.g. before
a firmware update), ``cordon node`` and ``uncordon node`` (back into scheduling).
"""

import time
from typing import Any, Callable, Dict, List

from ..errors import TKError

MIRROR_ANNOTATION = "kubernetes.io/config.mirror"


def _evictable(pod: Dict[str, Any]) -> bool:
    meta = pod.get("metadata") or {}
    if MIRROR_ANNOTATION in (meta.get("annotations") or {}):
        return False
    return not any(o.get("kind") == "DaemonSet" for o in meta.get("ownerReferences") or [])


def _ident(pod: Dict[str, Any]) -> str:
    meta = pod.get("metadata") or {}
    return f"{meta.get('namespace', 'default')}/{meta.get('name', '')}"


def drain_node(client: Any, cluster_id: str, name: str, timeout: float = 600.0,
               echo: Callable[[str], None] = lambda s: None, force: bool = False) -> Dict[str, Any]:
    """Cordon ``name`` and evict its pods; returns ``{"evicted": [...], "kept": [...],
    "refusals": N, "seconds": S}``.  Raises :class:`TKError` when pods remain at the deadline."""
    t0 = time.time()
    deadline = t0 + timeout
    client.cordon(cluster_id, name)
    pods = client.node_pods(cluster_id, name)
    kept = sorted(_ident(p) for p in pods if not _evictable(p))
    bare = sorted(_ident(p) for p in pods if _evictable(p) and not (p.get("metadata") or {}).get("ownerReferences"))
    if bare and not force:
        raise TKError(f"{name} runs pods no controller manages (they would not come back): {', '.join(bare)}; "
                      "set drain_force: true to evict them anyway (the node stays cordoned)")
    evicted: List[str] = []
    refusals = 0
    delay = 0.05
    while True:
        left = [p for p in client.node_pods(cluster_id, name) if _evictable(p)]
        if not left:
            break
        if time.time() >= deadline:
            raise TKError(f"drain of {name} timed out after {timeout:g}s; pods still on the node: "
                          + ", ".join(sorted(_ident(p) for p in left))
                          + f" (the node stays cordoned; nothing was destroyed)")
        for p in left:
            ns, pod = _ident(p).split("/", 1)
            code = client.evict_pod(cluster_id, ns, pod)
            if code == 429:
                refusals += 1
            elif _ident(p) not in evicted:
                evicted.append(_ident(p))
        time.sleep(min(delay, max(0.0, deadline - time.time())))
        delay = min(delay * 2, 5.0)
    out = {"evicted": sorted(evicted), "kept": kept, "refusals": refusals, "seconds": round(time.time() - t0, 3)}
    echo(f"Drained {name}: evicted {len(evicted)} pod(s)"
         + (f", {refusals} eviction(s) refused by disruption budgets and retried" if refusals else "")
         + (f"; kept {len(kept)} DaemonSet/mirror pod(s)" if kept else ""))
    return out


def _target(ctx, backend):
    from ..errors import ConfigError
    from .destroy import _rancher_client
    from .select import select_cluster, select_manager, select_node

    managers = backend.states()
    if not managers:
        raise ConfigError("No cluster managers.")
    state = backend.state(select_manager(ctx, managers))
    _, key = select_cluster(ctx, state.clusters(), "Cluster of the node", sort=False)
    hostname, _ = select_node(ctx, state.nodes(key), "Node")
    client, cid = _rancher_client(ctx, backend, state, key)
    if client is None:
        raise ConfigError(f"the cluster of {hostname} has no Rancher outputs yet (was it applied?)")
    return client, cid, hostname


def drain_command(ctx, backend) -> Dict[str, Any]:
    """``drain node``: cordon + evict, the node stays in the cluster (cordoned)."""
    client, cid, hostname = _target(ctx, backend)
    return drain_node(client, cid, hostname, ctx.settings.get_float("drain_timeout", 600), ctx.echo,
                      ctx.settings.get_bool("drain_force"))


def cordon_command(ctx, backend, unschedulable: bool) -> None:
    """``cordon node`` / ``uncordon node``."""
    client, cid, hostname = _target(ctx, backend)
    client.cordon(cid, hostname, unschedulable)
    ctx.echo(f"{hostname} {'cordoned' if unschedulable else 'uncordoned'}")


__all__ = ["drain_node", "drain_command", "cordon_command"]
