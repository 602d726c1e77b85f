"""create -> kubectl-ready waiter (new; the reference stops at agent launch,
``create/cluster.go:277-289``, so it never measures or guarantees readiness).

Phases, each time-stamped (the BASELINE.json metric is ``ready - start``):

1. ``cluster_active``   Rancher reports the cluster ``active`` (RKE done);
2. ``nodes_ready``      every expected node is in the Kubernetes node list with
                        condition ``Ready=True`` (read through Rancher's k8s proxy);
3. ``gpus_allocatable`` every MI355X node advertises ``amd.com/gpu`` equal to its
                        expected count (device plugin up);
4. ``rccl_gate``        optional: one RCCL all-reduce sweep across every GPU of
                        the GPU nodes (N2), run by the node agents as one
                        communicator (``gate.py``; its init may already have been
                        started, pipelined with the node bootstrap).

Polling is adaptive (20 ms doubling to 1 s), not the reference's fixed 5 s.
"""

import json
import time
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, List, Optional

from ..errors import TKError
from ..rancher.client import RancherClient, wait_until
from ..utils.trace import span


@dataclass
class ReadinessSpec:
    cluster_id: str
    nodes: List[str]
    gpu_nodes: Dict[str, int] = field(default_factory=dict)  # hostname -> expected amd.com/gpu
    timeout: float = 3600.0
    rccl_gate: bool = False
    rccl_hosts: List[str] = field(default_factory=list)  # agent URLs of GPU nodes, rank order
    rccl_ndev: List[int] = field(default_factory=list)  # GPUs per rccl_hosts entry (default 1 each)
    rccl_sizes: List[int] = field(default_factory=lambda: [1 << 20, 64 << 20])
    rccl_iters: int = 5


@dataclass
class ReadinessReport:
    start: float
    phases: Dict[str, float] = field(default_factory=dict)
    nodes: Dict[str, Dict[str, Any]] = field(default_factory=dict)
    rccl: Optional[Dict[str, Any]] = None

    @property
    def ready_seconds(self) -> float:
        return max(self.phases.values()) - self.start if self.phases else 0.0

    def to_json(self) -> Dict[str, Any]:
        d = asdict(self)
        d["phase_seconds"] = {k: round(v - self.start, 4) for k, v in self.phases.items()}
        d["ready_seconds"] = round(self.ready_seconds, 4)
        return d


def _node_ready(item: Dict[str, Any]) -> bool:
    for c in (item.get("status") or {}).get("conditions", []) or []:
        if c.get("type") == "Ready":
            return c.get("status") == "True"
    return False


def wait_ready(client: RancherClient, spec: ReadinessSpec, start: Optional[float] = None,
               agent_transport: Any = None, gate: Any = None) -> ReadinessReport:
    rep = ReadinessReport(start=start if start is not None else time.time())
    deadline = rep.start + spec.timeout

    def left() -> float:
        return max(1.0, deadline - time.time())

    with span("ready.cluster_active", cluster=spec.cluster_id):
        wait_until(lambda: client.cluster_state(spec.cluster_id) == "active", left(),
                   f"cluster {spec.cluster_id} to become active")
    rep.phases["cluster_active"] = time.time()

    want = set(spec.nodes)

    def nodes_ready() -> Optional[Dict[str, Dict[str, Any]]]:
        items = {i["metadata"]["name"]: i for i in client.k8s_nodes(spec.cluster_id)}
        if not want.issubset(items) or not all(_node_ready(items[n]) for n in want):
            return None
        return items

    with span("ready.nodes", count=len(want)):
        items = wait_until(nodes_ready, left(), f"{len(want)} nodes Ready")
    rep.phases["nodes_ready"] = time.time()

    if spec.gpu_nodes:
        def gpus() -> Optional[Dict[str, Dict[str, Any]]]:
            got = {i["metadata"]["name"]: i for i in client.k8s_nodes(spec.cluster_id)}
            for host, n in spec.gpu_nodes.items():
                alloc = ((got.get(host) or {}).get("status") or {}).get("allocatable", {})
                if str(alloc.get("amd.com/gpu", "0")) != str(n):
                    return None
            return got

        with span("ready.gpus", nodes=len(spec.gpu_nodes)):
            items = wait_until(gpus, left(), "amd.com/gpu allocatable on every GPU node")
        rep.phases["gpus_allocatable"] = time.time()

    for name in want:
        it = items.get(name, {})
        rep.nodes[name] = {"labels": (it.get("metadata") or {}).get("labels", {}),
                           "allocatable": (it.get("status") or {}).get("allocatable", {})}

    if spec.rccl_gate and spec.rccl_hosts:
        if gate is None:
            from .gate import ClusterGate, members_from

            gate = ClusterGate(agent_transport, members_from(spec.rccl_hosts, spec.rccl_ndev or None),
                               spec.rccl_sizes, spec.rccl_iters)
        with span("ready.rccl_gate", world=gate.world, nodes=len(gate.members)):
            rep.rccl = gate.run()
        if not rep.rccl.get("ok"):
            raise TKError(f"RCCL readiness gate failed: {rep.rccl}")
        rep.phases["rccl_gate"] = time.time()
    return rep


def rccl_gate(transport: Any, agent_urls: List[str], sizes: List[int], iters: int = 5,
              ndevs: Optional[List[int]] = None) -> Dict[str, Any]:
    """One RCCL communicator across the GPU node agents (not pipelined; see gate.py)."""
    from .gate import ClusterGate, members_from

    return ClusterGate(transport, members_from(agent_urls, ndevs), sizes, iters).run()


def spec_from_state(state, backend, cluster_key: str, timeout: float = 3600.0, rccl_gate: bool = False):
    """Build the client + spec for a cluster from the document and the executor's tfstate."""
    from ..executor.base import outputs_from_tfstate
    from ..state import MANAGER_KEY
    from ..terraform.catalog import module_from_source

    raw = backend.read_tfstate(state.name)
    mgr = outputs_from_tfstate(raw, MANAGER_KEY)
    cl = outputs_from_tfstate(raw, cluster_key)
    if not mgr.get("rancher_url") or not cl.get("rancher_cluster_id"):
        raise TKError("cluster outputs unavailable; cannot wait for readiness")
    client = RancherClient(mgr["rancher_url"], mgr.get("rancher_access_key", ""), mgr.get("rancher_secret_key", ""))
    nodes = state.nodes(cluster_key)
    from ..models.baremetal import addons_key
    from ..state import cluster_key_parts

    # amd.com/gpu only appears once the device plugin runs, i.e. with the add-on module
    has_plugin = state.module(addons_key(cluster_key_parts(cluster_key)[1])) is not None
    gpu_nodes: Dict[str, int] = {}
    rccl_hosts: List[str] = []
    rccl_ndev: List[int] = []
    for host in sorted(nodes):
        cfg = state.module(nodes[host]) or {}
        info = module_from_source(str(cfg.get("source", "")))
        if info is not None and info.mi355x:
            if has_plugin:
                gpu_nodes[host] = int(cfg.get("gpu_count", 8))
            addr = str(cfg.get("host", ""))
            if addr.startswith("agent+"):
                rccl_hosts.append(addr[len("agent+"):])
                rccl_ndev.append(int(cfg.get("gpu_count", 8) or 8))
    spec = ReadinessSpec(cl["rancher_cluster_id"], sorted(nodes), gpu_nodes, timeout,
                         rccl_gate and bool(rccl_hosts), rccl_hosts, rccl_ndev)
    return client, spec


def gate_sizes(settings) -> List[int]:
    """RCCL gate message sizes: 1 MiB and ``rccl_gate_max_mib`` (default 64 MiB)."""
    mib = int(float(settings.get_string("rccl_gate_max_mib") or 64)) if settings.is_set("rccl_gate_max_mib") else 64
    if mib < 1:
        raise TKError(f"rccl_gate_max_mib must be >= 1. Found '{mib}'.")
    return sorted({1 << 20, mib << 20})


def agent_transport_for(ctx) -> Any:
    transport = ctx.extras.get("agent_transport")
    if transport is None:
        from ..parallel.transport import AgentTransport

        transport = AgentTransport(token=ctx.settings.get_string("agent_token"))
    return transport


def early_gate(ctx, state, cluster_key: str) -> Any:
    """Start the cluster RCCL gate's communicator init now (``wait`` + ``rccl_gate`` with
    agent-managed GPU nodes; ``rccl_pipeline: false`` disables).  Returns the gate or None."""
    s = ctx.settings
    if not (s.get_bool("wait") and s.get_bool("rccl_gate")):
        return None
    if s.is_set("rccl_pipeline") and not s.get_bool("rccl_pipeline"):
        return None
    from .gate import ClusterGate

    gate = ClusterGate.from_state(state, cluster_key, agent_transport_for(ctx), gate_sizes(s))
    return gate.prepare_async() if gate is not None else None


def wait_after_create(ctx, backend, state, cluster_key: str, start: Optional[float] = None,
                      gate: Any = None) -> ReadinessReport:
    s = ctx.settings
    timeout = float(s.get_string("wait_timeout") or 3600)
    client, spec = spec_from_state(state, backend, cluster_key, timeout, s.get_bool("rccl_gate"))
    spec.rccl_sizes = gate_sizes(s)
    transport = agent_transport_for(ctx) if spec.rccl_gate else None
    if gate is not None and (not spec.rccl_gate or gate.world != sum(spec.rccl_ndev or [1] * len(spec.rccl_hosts))):
        gate.abort()  # membership changed since it was prepared
        gate = None
    rep = wait_ready(client, spec, start=start, agent_transport=transport, gate=gate)
    ctx.extras["last_readiness"] = rep  # callers that time phases (bench.py) read it here
    ctx.echo(f"cluster ready in {rep.ready_seconds:.2f}s: " +
             json.dumps(rep.to_json()["phase_seconds"], sort_keys=True))
    return rep


__all__ = ["ReadinessSpec", "ReadinessReport", "wait_ready", "rccl_gate", "spec_from_state", "wait_after_create",
           "early_gate", "agent_transport_for", "gate_sizes"]
