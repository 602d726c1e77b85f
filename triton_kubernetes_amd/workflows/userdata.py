"""``userdata node``: cloud-init user-data for a node module instead of SSH delivery.

For bare-metal fleets provisioned by PXE / MAAS / image-based installs, the node's
bootstrap plan can be shipped as cloud-init user-data: the RCCL environment is
written by ``write_files`` before first boot completes, and ``runcmd`` runs the
same plan the SSH path would (node/plan.py:render_cloud_init).  The cluster's
registration token and CA checksum come from the applied cluster module's
outputs (tfstate), exactly as the host module receives them.
"""

from ..backend.base import Backend
from ..config.context import Context
from ..errors import ConfigError, TKError
from ..executor.base import outputs_from_tfstate
from ..executor.direct import resolve
from ..node.plan import build_host_plan, render_cloud_init
from ..terraform.catalog import module_from_source
from .select import select_cluster, select_manager, select_node


def node_userdata(ctx: Context, backend: Backend) -> str:
    managers = backend.states()
    if not managers:
        raise ConfigError("No cluster managers.")
    manager = select_manager(ctx, managers)
    state = backend.state(manager)
    clusters = state.clusters()
    if not clusters:
        raise ConfigError("No clusters.")
    _, cluster_key = select_cluster(ctx, clusters, "Cluster")
    nodes = state.nodes(cluster_key)
    if not nodes:
        raise ConfigError("No nodes.")
    hostname, node_key = select_node(ctx, nodes)
    cfg = state.module(node_key) or {}
    info = module_from_source(str(cfg.get("source", "")))
    raw = backend.read_tfstate(manager)
    outputs = {k: outputs_from_tfstate(raw, k) for k in state.modules()}
    try:
        resolved = resolve(cfg, outputs)
    except Exception as exc:  # noqa: BLE001 - unapplied cluster
        raise TKError(f"node '{hostname}': cluster outputs are not available yet (apply the cluster first): {exc}")
    missing = [k for k in ("rancher_api_url", "rancher_cluster_registration_token", "rancher_cluster_ca_checksum")
               if not isinstance(resolved.get(k), str)]
    if missing:
        raise TKError(f"node '{hostname}': its module block lacks {', '.join(missing)} (not a host module of a "
                      "cluster of this manager?)")
    plan = build_host_plan(resolved, resolved["rancher_api_url"], resolved["rancher_cluster_registration_token"],
                           resolved["rancher_cluster_ca_checksum"], mi355x=bool(info and info.mi355x),
                           sequential=True)
    text = render_cloud_init(plan, resolved.get("rccl_env") if info and info.mi355x else None)
    ctx.out.write(text)
    return text


__all__ = ["node_userdata"]
