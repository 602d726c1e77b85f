"""``create manager|cluster|node`` (reference ``create/manager.go``, ``create/cluster.go``,
``create/node.go``).

Flow per command: select/validate -> provider plugin adds module(s) to the
document -> confirmation -> executor apply -> persist.

Failure semantics differ deliberately from the
reference, which persists ``main.tf.json`` only after a successful apply and so
orphans whatever a failed apply created:

* a failed apply still persists the document (so ``destroy`` can reach every
  resource that may exist) and records ``status.json`` = ``{"phase":
  "apply_failed", "modules": [...], "error": ...}`` in the backend;
* ``create manager`` with the name of a manager whose first apply failed
  resumes it instead of failing with "already exists";
* two CLIs working on one manager (a shared Manta backend) do not overwrite each
  other: under the backend lock the run's own changes are replayed onto the document
  persisted meanwhile (``State.rebase``), and a module both changed is an error.
"""

import json
import time
from typing import Dict, List, Optional

from ..backend.base import Backend
from ..config.context import Context, not_blank
from ..errors import Canceled, ConfigError, TKError
from ..models import CLUSTER_CHOICES, CLUSTER_PROVIDERS, MANAGER_CHOICES, MANAGER_PROVIDERS, NODE_ENTRY_KEYS
from ..models import NODE_PROVIDERS
from ..models.common import nodes_added_message
from ..state import MANAGER_KEY, State
from ..terraform.catalog import check_sources
from ..utils.trace import span
from .select import executor_for, select_cluster, select_manager

STATUS_BLOB = "status.json"
NO_MANAGERS = "No cluster managers, please create a cluster manager before creating a kubernetes cluster."


def read_status(backend: Backend, name: str) -> Dict:
    try:
        raw = backend.read_blob(name, STATUS_BLOB)
    except (NotImplementedError, TKError):
        return {}
    return json.loads(raw) if raw else {}


def _write_status(backend: Backend, name: str, status: Dict) -> None:
    try:
        backend.write_blob(name, STATUS_BLOB, json.dumps(status, indent=2).encode())
    except NotImplementedError:
        pass


def apply_and_persist(ctx: Context, backend: Backend, state: State, new_modules: List[str]) -> None:
    """Run the executor, then persist; on failure persist + record status (see module doc)."""
    executor = executor_for(ctx, state, backend)
    with backend.lock(state.name):
        # another run may have persisted clusters / nodes since this one read the document
        others = state.rebase(backend.state(state.name))
        if others:
            ctx.echo(f"note: kept changes another run persisted meanwhile ({', '.join(others)})")
        try:
            with span("apply", executor=executor.name, modules=len(new_modules)):
                executor.apply(state, backend)
        except BaseException as exc:
            ctx.extras["last_apply"] = getattr(executor, "last_report", None)
            backend.persist_state(state)
            _write_status(backend, state.name, {"phase": "apply_failed", "modules": new_modules,
                                                "error": str(exc), "time": time.time()})
            if isinstance(exc, TKError):
                raise TKError(f"{exc}\n(desired state persisted; re-run to resume or destroy to clean up)") \
                    from exc
            raise
        # per-module results (the DirectExecutor's report: node plans' step timings) for callers
        ctx.extras["last_apply"] = getattr(executor, "last_report", None)
        backend.persist_state(state)
        state.mark_base()
        _write_status(backend, state.name, {"phase": "applied", "modules": new_modules, "time": time.time()})


def _apply_then_wait(ctx: Context, backend: Backend, state: State, cluster_key: str,
                     new_modules: List[str]) -> None:
    """Apply + persist, then (``wait``) the readiness waiter.  With ``rccl_gate`` on
    agent-managed GPU nodes the gate's communicator init is started before the
    apply, so it overlaps node bootstrap (readiness/gate.py)."""
    gate = None
    ctx.extras["backend"] = backend
    if ctx.settings.get_bool("wait"):
        from ..readiness.waiter import early_gate

        gate = early_gate(ctx, state, cluster_key)
    try:
        apply_and_persist(ctx, backend, state, new_modules)
        if ctx.settings.get_bool("wait"):
            from ..readiness.waiter import wait_after_create

            wait_after_create(ctx, backend, state, cluster_key, gate=gate)
    finally:
        if gate is not None:
            gate.abort()  # no-op once the gate ran


# --- manager ---------------------------------------------------------------------------
def new_manager(ctx: Context, backend: Backend) -> None:
    provider = ctx.resolve_choice("manager_cloud_provider", "Create Manager in which Cloud Provider",
                                  MANAGER_CHOICES, transform=str.lower)
    name = ctx.resolve("name", "Cluster Manager Name", validate=not_blank("manager name cannot be blank"))
    if not name:
        raise ConfigError("Invalid Cluster Manager Name")
    if name in backend.states():
        if read_status(backend, name).get("phase") != "apply_failed":
            raise ConfigError(f"A Cluster Manager with the name '{name}' already exists.")
        ctx.echo(f"Resuming creation of '{name}' after a failed apply.")
    state = backend.state(name).mark_base()
    fn = MANAGER_PROVIDERS.get(provider)
    if fn is None:
        raise ConfigError(f"Unsupported cloud provider '{provider}', cannot create manager")
    fn(ctx, state, name)
    if not ctx.confirm("Proceed with the manager creation", "Proceed"):
        ctx.echo("Manager creation canceled.")
        return
    mgr = state.module(MANAGER_KEY) or {}
    if str(mgr.get("host", "")).startswith("rancher+"):
        # an adopted Rancher server: its first-login password, if given, and the opt-in for
        # the legacy derived one go to the state backend (rancher/bootstrap_secret.py), never
        # into main.tf.json
        from ..rancher import bootstrap_secret

        given = ctx.get_string("rancher_bootstrap_password") if ctx.is_set("rancher_bootstrap_password") else ""
        legacy = ctx.settings.get_bool("rancher_legacy_bootstrap") if ctx.is_set("rancher_legacy_bootstrap") \
            else False
        bootstrap_secret.save_adopted(backend, name, given, legacy)
    path, obj = backend.state_terraform_config(name)
    state.set_terraform_backend_config(path, obj)
    apply_and_persist(ctx, backend, state, ["cluster-manager"])


# --- cluster ----------------------------------------------------------------------------
def _node_entry_overrides(entry: Dict, provider: str) -> Dict:
    """Settings overrides for one ``nodes:`` entry (Q4 fix: every present key)."""
    if not isinstance(entry, dict):
        raise ConfigError("Could not read node configuration")
    overrides = {str(k): v for k, v in entry.items()}
    for key in NODE_ENTRY_KEYS["common"]:
        overrides.setdefault(key, None)  # per-node keys never leak between entries
    return overrides


def new_cluster(ctx: Context, backend: Backend) -> Optional[str]:
    managers = backend.states()
    if not managers:
        raise ConfigError(NO_MANAGERS)
    manager = select_manager(ctx, managers)
    state = backend.state(manager).mark_base()
    check_sources(state.modules())  # refused before any question is asked
    provider = ctx.resolve_choice("cluster_cloud_provider", "Create Cluster in which Cloud Provider",
                                  CLUSTER_CHOICES, transform=str.lower)
    fn = CLUSTER_PROVIDERS.get(provider)
    if fn is None:
        raise ConfigError(f"Unsupported cloud provider '{provider}', cannot create cluster")
    before = set(state.modules())
    name = fn(ctx, backend, state)
    clusters = state.clusters()
    if name not in clusters:
        raise ConfigError(f"Couldn't find cluster key for cluster '{name}'.\n")
    key = clusters[name]

    if ctx.is_set("nodes"):
        entries = ctx.settings.get("nodes")
        if not isinstance(entries, list):
            raise ConfigError("Could not read 'nodes' configuration")
        for entry in entries:
            saved = ctx.settings.push_overrides(_node_entry_overrides(entry, provider))
            try:
                hostnames = NODE_PROVIDERS[provider](ctx, manager, key, backend, state)
            finally:
                ctx.settings.pop_overrides(saved)
            ctx.echo(nodes_added_message(hostnames))

    if not ctx.non_interactive:
        more = ctx.prompter.yes_no("Would you like to create nodes for this cluster")
        while more:
            hostnames = NODE_PROVIDERS[provider](ctx, manager, key, backend, state)
            ctx.echo(nodes_added_message(hostnames))
            more = ctx.prompter.yes_no("Would you like to create more nodes for this cluster")
        if not ctx.confirm("Proceed with cluster creation", "Proceed"):
            ctx.echo("Cluster creation canceled.")
            return None

    new_modules = sorted(set(state.modules()) - before)
    _apply_then_wait(ctx, backend, state, key, new_modules)
    return name


# --- node -----------------------------------------------------------------------------------
def new_node(ctx: Context, backend: Backend) -> Optional[List[str]]:
    managers = backend.states()
    if not managers:
        raise ConfigError(NO_MANAGERS)
    manager = select_manager(ctx, managers)
    state = backend.state(manager).mark_base()
    check_sources(state.modules())  # refused before any question is asked
    _, key = select_cluster(ctx, state.clusters(), "Cluster to deploy node to")
    parts = key.split("_")
    if len(parts) < 3:
        raise ConfigError(f"Could not determine cloud provider for cluster '{key}'")
    fn = NODE_PROVIDERS.get(parts[1])
    if fn is None:
        raise ConfigError(f"Unsupported cloud provider '{parts[1]}', cannot create node")
    before = set(state.modules())
    hostnames = fn(ctx, manager, key, backend, state)
    if not ctx.confirm("Proceed with the node creation", "Proceed"):
        ctx.echo("Node creation canceled")
        return None
    _apply_then_wait(ctx, backend, state, key, sorted(set(state.modules()) - before))
    return hostnames


__all__ = ["new_manager", "new_cluster", "new_node", "apply_and_persist", "read_status", "Canceled"]
