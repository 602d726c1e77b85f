"""``destroy manager|cluster|node`` (reference ``destroy/*.go``).

* manager — destroy the whole document, then delete the backend state;
* cluster — ``-target=module.<cluster>`` plus one target per node (and the
  MI355X add-on module if present), then drop those modules and persist;
* node    — ``-target=module.<node>``, drop it, persist.

The document is read again under the backend lock before anything is destroyed, so
nodes another run added meanwhile are destroyed with their cluster and its clusters
are kept in the persisted document.

Host teardown (on by default for bare metal: ``node_cleanup``): every
destroyed bare-metal host is taken out of its cluster -- its rancher-system-agent and RKE2
(or RKE1 containers) uninstalled, their state removed (``node/cleanup.py``) -- so the same
host can join the next cluster.  The DirectExecutor does it over SSH or through the node
agent; the Terraform host modules with a destroy-time provisioner.  A host whose cleanup
failed is listed; its join record refuses the next join until it is cleaned.

Extension (opt-in via ``rancher_cleanup: true``): also
remove the cluster object (``destroy cluster``) or the node's object (``destroy node``:
the Rancher node with that hostname, which also drops it from the Kubernetes node list)
from Rancher after the destroy.

``destroy node`` with ``drain: true`` first cordons the node and evicts its pods through
the Eviction API (``workflows/drain.py``; ``drain_timeout`` seconds, default 600): the jobs
on a GPU node being replaced are rescheduled before its host goes away.
"""

from ..backend.base import Backend
from ..config.context import Context
from ..errors import ConfigError
from ..models.baremetal import addons_key
from ..state import cluster_key_parts
from ..utils.trace import span
from .create import NO_MANAGERS
from .select import executor_for, select_cluster, select_manager, select_node


def delete_manager(ctx: Context, backend: Backend) -> None:
    managers = backend.states()
    if not managers:
        raise ConfigError(NO_MANAGERS)
    manager = select_manager(ctx, managers, sort=True)
    state = backend.state(manager)
    if not ctx.confirm(f'Are you sure you want to destroy "{manager}"', f'Destroy "{manager}"'):
        ctx.echo("Destroy manager canceled.")
        return
    with backend.lock(manager):
        state = backend.state(manager)
        with span("destroy", scope="manager"):
            executor = executor_for(ctx, state, backend)
            executor.destroy(state, backend, [])
        _report_cleanup(ctx, executor)
        backend.delete_state(manager)


def delete_cluster(ctx: Context, backend: Backend) -> None:
    managers = backend.states()
    if not managers:
        raise ConfigError("No cluster managers.")
    manager = select_manager(ctx, managers)
    state = backend.state(manager)
    name, key = select_cluster(ctx, state.clusters(), "Cluster to delete")
    if not ctx.confirm(f'Are you sure you want to destroy "{name}"', f'Destroy "{name}"'):
        ctx.echo("Destroy cluster canceled.")
        return
    with backend.lock(manager):
        state = _reread(backend, manager, key)
        nodes = state.nodes(key)
        targets = [key] + [nodes[h] for h in sorted(nodes)]
        _, cluster_name = cluster_key_parts(key)
        addon = addons_key(cluster_name)
        if state.module(addon) is not None:
            targets.insert(0, addon)
        cleanup = _rancher_cleanup_info(ctx, backend, state, key)
        with span("destroy", scope="cluster", targets=len(targets)):
            executor = executor_for(ctx, state, backend)
            executor.destroy(state, backend, [f"module.{t}" for t in targets])
        _report_cleanup(ctx, executor)
        for t in targets:
            state.delete_module(t)
        backend.persist_state(state)
    if cleanup:
        cleanup()


def delete_node(ctx: Context, backend: Backend) -> None:
    managers = backend.states()
    if not managers:
        raise ConfigError("No cluster managers, please create a cluster manager before creating a kubernetes node.")
    manager = select_manager(ctx, managers)
    state = backend.state(manager)
    _, key = select_cluster(ctx, state.clusters(), "Cluster to delete", sort=False)
    hostname, node_key = select_node(ctx, state.nodes(key))
    if not ctx.confirm(f'Are you sure you want to destroy "{hostname}"', f'Destroy "{hostname}"'):
        ctx.echo("Destroy node canceled.")
        return
    if ctx.settings.get_bool("drain"):
        # before the lock: a drain waits on disruption budgets, the document is not touched
        client, cid = _rancher_client(ctx, backend, state, key)
        if client is None:
            raise ConfigError(f"drain: cluster of {hostname} has no Rancher outputs yet (was it applied?)")
        from .drain import drain_node

        timeout = ctx.settings.get_float("drain_timeout", 600)
        with span("destroy.drain", node=hostname):
            drain_node(client, cid, hostname, timeout, ctx.echo, ctx.settings.get_bool("drain_force"))
    with backend.lock(manager):
        state = _reread(backend, manager, node_key)
        cleanup = _rancher_node_cleanup_info(ctx, backend, state, key, hostname)
        with span("destroy", scope="node"):
            executor = executor_for(ctx, state, backend)
            executor.destroy(state, backend, [f"module.{node_key}"])
        _report_cleanup(ctx, executor)
        state.delete_module(node_key)
        backend.persist_state(state)
    if cleanup:
        cleanup()


def _report_cleanup(ctx: Context, executor) -> None:
    """One line per host the destroy took out of its cluster (the DirectExecutor's report;
    Terraform prints its provisioners' output itself)."""
    for key, rep in sorted((getattr(executor, "last_cleanup", None) or {}).items()):
        host = rep.get("hostname", key)
        if rep.get("ok"):
            done = [a["what"].rsplit("/", 1)[-1] for a in rep.get("actions", []) if a.get("status") == "ok"]
            ctx.echo(f"Cleaned up host {host}" + (f" ({', '.join(done)})" if done else ""))
        else:
            ctx.echo(f"WARNING: cleanup of host {host} failed: {rep.get('error', 'unknown error')}; "
                     f"it cannot join another cluster until it is cleaned up")


def _reread(backend: Backend, manager: str, key: str):
    """The persisted document (under the lock); ``key`` must still be in it."""
    state = backend.state(manager)
    if state.module(key) is None:
        raise ConfigError(f"module.{key} was removed by another triton-kubernetes run.")
    return state


def _rancher_client(ctx: Context, backend: Backend, state, cluster_key: str):
    """``(RancherClient, cluster id)`` from the executor's recorded outputs, or ``(None, "")``."""
    from ..executor.base import outputs_from_tfstate
    from ..rancher import trust
    from ..state import MANAGER_KEY

    raw = backend.read_tfstate(state.name)
    mgr = outputs_from_tfstate(raw, MANAGER_KEY)
    cid = outputs_from_tfstate(raw, cluster_key).get("rancher_cluster_id")
    if not mgr.get("rancher_url") or not cid:
        return None, ""

    factory = ctx.extras.get("rancher_factory") or (  # verified against the pinned CA (rancher/trust.py)
        lambda url, ak="", sk="": trust.client(backend, state.name, url, ak, sk))
    return factory(mgr["rancher_url"], mgr.get("rancher_access_key", ""), mgr.get("rancher_secret_key", "")), cid


def _rancher_node_cleanup_info(ctx: Context, backend: Backend, state, cluster_key: str, hostname: str):
    """Return a callable deleting the node's Rancher object (opt-in), or ``None``."""
    if not ctx.settings.get_bool("rancher_cleanup"):
        return None
    from ..executor.base import outputs_from_tfstate
    from ..rancher import trust
    from ..state import MANAGER_KEY

    raw = backend.read_tfstate(state.name)
    mgr = outputs_from_tfstate(raw, MANAGER_KEY)
    cid = outputs_from_tfstate(raw, cluster_key).get("rancher_cluster_id")
    if not mgr.get("rancher_url") or not cid:
        return None

    def _cleanup():
        client = trust.client(backend, state.name, mgr["rancher_url"], mgr.get("rancher_access_key", ""),
                              mgr.get("rancher_secret_key", ""))
        gone = [n["id"] for n in client.nodes(cid)
                if hostname in (n.get("hostname"), n.get("nodeName"), n.get("requestedHostname"))]
        for nid in gone:
            client.delete_node(nid)
        ctx.echo(f"Removed Rancher node {', '.join(gone)} ({hostname})" if gone else
                 f"No Rancher node named {hostname} in cluster {cid}")

    return _cleanup


def _rancher_cleanup_info(ctx: Context, backend: Backend, state, cluster_key: str):
    """Return a callable deleting the Rancher cluster object (opt-in), or ``None``."""
    if not ctx.settings.get_bool("rancher_cleanup"):
        return None
    from ..executor.base import outputs_from_tfstate
    from ..rancher import trust
    from ..state import MANAGER_KEY

    raw = backend.read_tfstate(state.name)
    mgr = outputs_from_tfstate(raw, MANAGER_KEY)
    cl = outputs_from_tfstate(raw, cluster_key)
    if not mgr.get("rancher_url") or not cl.get("rancher_cluster_id"):
        return None

    def _cleanup():
        client = trust.client(backend, state.name, mgr["rancher_url"], mgr.get("rancher_access_key", ""),
                              mgr.get("rancher_secret_key", ""))
        client.delete_cluster(cl["rancher_cluster_id"])
        ctx.echo(f"Removed Rancher cluster {cl['rancher_cluster_id']}")

    return _cleanup
