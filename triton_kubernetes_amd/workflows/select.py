"""Selection helpers shared by the create / destroy / get workflows."""

from typing import Dict, List, Optional, Tuple

from ..backend.base import Backend
from ..config.context import Context
from ..errors import ConfigError
from ..state import State


def select_manager(ctx: Context, managers: List[str], label: str = "Cluster Manager",
                   sort: bool = False) -> str:
    items = sorted(managers) if sort else list(managers)
    selected = ctx.resolve_choice("cluster_manager", label, items)
    if selected not in managers:
        raise ConfigError(f"Selected cluster manager '{selected}' does not exist.")
    return selected


def select_cluster(ctx: Context, clusters: Dict[str, str], label: str, sort: bool = True) -> Tuple[str, str]:
    """Return ``(cluster name, cluster key)``."""
    if ctx.is_set("cluster_name"):
        name = ctx.get_string("cluster_name")
        if name not in clusters:
            raise ConfigError(f"A cluster named '{name}', does not exist.")
        return name, clusters[name]
    if ctx.non_interactive:
        raise ConfigError("cluster_name must be specified")
    names = sorted(clusters) if sort else list(clusters)
    _, name = ctx.prompter.select(label, names)
    return name, clusters[name]


def select_node(ctx: Context, nodes: Dict[str, str], label: str = "Node to delete") -> Tuple[str, str]:
    if ctx.is_set("hostname"):
        hostname = ctx.get_string("hostname")
        if hostname not in nodes:
            raise ConfigError(f"A node named '{hostname}', does not exist.")
        return hostname, nodes[hostname]
    if ctx.non_interactive:
        raise ConfigError("hostname must be specified")
    names = sorted(nodes)
    _, hostname = ctx.prompter.select(label, names)
    return hostname, nodes[hostname]


def executor_for(ctx: Context, state: Optional[State] = None, backend: Optional[Backend] = None):
    """The executor to run a document with (``backend``: the manager's state backend,
    which also holds its node-agent PKI).

    ``executor`` setting: ``terraform`` | ``direct`` | ``auto`` (default).  Auto
    uses Terraform when the binary is on ``PATH``; otherwise the native
    DirectExecutor if every module in the document is one it implements.
    """
    if backend is not None:
        ctx.extras["backend"] = backend
    if ctx.executor_factory is not None:
        return ctx.executor_factory(ctx)
    from ..executor.factory import build_executor

    return build_executor(ctx, state)


def load_state(backend: Backend, name: str) -> State:
    return backend.state(name)
