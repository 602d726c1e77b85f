"""``get manager|cluster`` (reference ``get/manager.go``, ``get/cluster.go``).

Prints the module outputs: ``rancher_url`` / ``rancher_access_key`` /
``rancher_secret_key`` for the manager, the cluster id / registration token /
CA checksum (+ provider network ids) for a cluster.  With Terraform < 0.12 this
is exactly ``terraform output -module <key>``; otherwise the executor reads the
root outputs it rendered, or the DirectExecutor's tfstate.
"""

from ..backend.base import Backend
from ..config.context import Context
from ..errors import ConfigError
from ..state import MANAGER_KEY
from .select import executor_for, select_cluster, select_manager


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
