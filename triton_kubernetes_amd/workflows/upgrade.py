"""``upgrade cluster``: move a cluster to a newer Kubernetes release through Rancher.

The reference has no upgrade path: a cluster keeps the ``k8s_version`` it was created
with (``create/cluster.go:349-356``), and re-applying its module does not touch a running
cluster.  Here:

1. the target release (``k8s_version``: a full release, or ``vX.Y`` for the server's
   release of that minor) must be of the cluster's distribution, offered by the Rancher
   server, not older than the running one, and at most **one minor** ahead -- the
   Kubernetes version-skew policy upgrades the control plane one minor at a time;
2. Rancher is told (RKE2: the provisioning cluster's ``spec.kubernetesVersion``; RKE1: its
   ``rancherKubernetesEngineConfig``) and its controllers roll the nodes;
3. the cluster module's ``k8s_version`` in the document is updated under the backend lock,
   so the document describes the running cluster;
4. with ``wait`` (default true) the CLI waits until Rancher reports the new release and
   the cluster ``active``, every node's kubelet runs it, then runs the readiness waiter
   (nodes Ready, ``amd.com/gpu`` allocatable again on every MI355X node, the RCCL gate
   with ``rccl_gate: true``): GPU pods lose their devices while a node's kubelet restarts.

Settings: ``cluster_manager``, ``cluster_name``, ``k8s_version``, ``wait`` (true),
``wait_timeout`` (3600).
"""

import re
import time
from typing import Any, Dict, Tuple

from ..backend.base import Backend
from ..config.context import Context
from ..errors import ConfigError, TKError
from ..rancher.client import wait_until
from ..utils.trace import span
from ..versions import distribution_of, k8s_minor, resolve_distribution, running_version
from .select import select_cluster, select_manager


def _key(v: str) -> Tuple[int, ...]:
    return tuple(int(x) for x in re.findall(r"\d+", v.split("+")[0].split("-")[0]))


def check_upgrade(current: str, target: str) -> None:
    """Raise ConfigError unless ``current`` -> ``target`` is a same-distribution upgrade of at
    most one minor."""
    cur_dist, new_dist = distribution_of(current), distribution_of(target)
    if cur_dist and new_dist and cur_dist != new_dist:
        raise ConfigError(f"{target} is an {new_dist.upper()} release; the cluster runs {cur_dist.upper()} "
                          f"({current}). A cluster cannot change distribution.")
    if _key(target) < _key(current):
        raise ConfigError(f"cannot downgrade the cluster from {current} to {target}")
    cm, tm = _key(current)[:2], _key(target)[:2]
    if tm[0] != cm[0] or tm[1] > cm[1] + 1:
        raise ConfigError(f"upgrade one minor at a time: the cluster runs {k8s_minor(current)}, "
                          f"so the next release is v{cm[0]}.{cm[1] + 1}; {target} skips minors")


def upgrade_cluster(ctx: Context, backend: Backend) -> Dict[str, Any]:
    from .destroy import _rancher_client

    managers = backend.states()
    if not managers:
        raise ConfigError("No cluster managers.")
    manager = select_manager(ctx, managers)
    state = backend.state(manager)
    name, key = select_cluster(ctx, state.clusters(), "Cluster to upgrade")
    requested = ctx.settings.get_string("k8s_version")
    if not requested:
        raise ConfigError("k8s_version is required: the Kubernetes release to upgrade to")
    client, cid = _rancher_client(ctx, backend, state, key)
    if client is None:
        raise ConfigError(f"Cluster '{name}' has no Rancher outputs yet (was it applied?)")
    current = client.cluster_version(cid)
    dist = "rke2" if cid.startswith("c-m-") else "rke1"
    try:
        resolve_distribution(requested, dist)
    except ValueError as exc:
        raise ConfigError(str(exc)) from None
    target = client.resolve_k8s_version(requested, dist)
    if getattr(client, "last_version_note", ""):
        ctx.echo(client.last_version_note)
    # what Rancher and the kubelets will report once the cluster runs the target (RKE1: the
    # upstream version, without -rancherN-N)
    want = running_version(target, dist)
    if want == running_version(current, dist):
        ctx.echo(f"cluster '{name}' already runs {current}")
        return {"from": current, "to": target, "changed": False}
    check_upgrade(current, target)
    if not ctx.confirm(f'Upgrade "{name}" from {current} to {target}', f'Upgrade "{name}"'):
        ctx.echo("Upgrade cluster canceled.")
        return {"from": current, "to": target, "changed": False}
    t0 = time.time()
    with span("upgrade.request", cluster=cid, to=target):
        client.upgrade_cluster(cid, target)
    with backend.lock(manager):
        state = backend.state(manager)
        mod = state.module(key)
        if mod is None:
            raise TKError(f"module.{key} was removed by another triton-kubernetes run.")
        state.set_module(key, dict(mod, k8s_version=target))
        backend.persist_state(state)
    ctx.echo(f"cluster '{name}': {current} -> {target} requested")
    out: Dict[str, Any] = {"from": current, "to": target, "changed": True}
    wait = ctx.settings.get_bool("wait") if ctx.is_set("wait") else True
    if wait:
        timeout = ctx.settings.get_float("wait_timeout", 3600)

        def upgraded() -> bool:
            if client.cluster_version(cid) != want or client.cluster_state(cid) != "active":
                return False
            return all((n.get("status") or {}).get("nodeInfo", {}).get("kubeletVersion") == want
                       for n in client.k8s_nodes(cid))

        with span("upgrade.rollout", cluster=cid):
            wait_until(upgraded, timeout, f"cluster {cid} to run {target}")
        out["rollout_s"] = round(time.time() - t0, 3)
        from ..readiness.waiter import wait_after_create

        rep = wait_after_create(ctx, backend, state, key, start=t0)
        out["ready_s"] = round(rep.ready_seconds, 3)
        ctx.echo(f"cluster '{name}' runs {target}")
    return out


__all__ = ["upgrade_cluster", "check_upgrade"]
