"""create -> kubectl-ready waiter (new; the reference stops at agent launch,
``create/cluster.go:277-289``, so it never measures or guarantees readiness).

Phases, each time-stamped (the BASELINE.json metric is ``ready - start``):

1. ``cluster_active``   Rancher reports the cluster ``active`` (RKE done);
2. ``nodes_ready``      every expected node is in the Kubernetes node list with
                        condition ``Ready=True`` (read through Rancher's k8s proxy);
3. ``gpus_allocatable`` every MI355X node advertises ``amd.com/gpu`` equal to its
                        expected count (device plugin up).  A node that joined with the
                        GPU health taint (``gpu_health: taint``, ``node/health.py``) is
                        left out of this check and of the gate, and listed in the
                        report's ``gpu_unhealthy``;
4. ``rccl_gate``        optional: one RCCL all-reduce sweep across every GPU of
                        the GPU nodes (N2) as one communicator -- run by the node
                        agents (``gate.py``; its init may already have been started,
                        pipelined with the node bootstrap) or, for nodes delivered
                        over SSH / Terraform, by one ``rccl-ready --cluster``
                        process per node (``process_gate.py``).  When the gate
                        cannot run the report says why (``rccl.skipped``).

Polling is adaptive (20 ms doubling to 1 s), not the reference's fixed 5 s.

The report also lists the GPU-node labels that differ across the cluster's MI355X nodes
(``gpu_mismatch``: product, VBIOS, ISA target, partition modes, HBM, CUs, RDMA fabric,
ROCm userspace, power cap):
one RCCL job over nodes flashed or partitioned apart is a classic source of hangs and
uneven bandwidth.  It is a warning, not a failed readiness.
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
    # GPU nodes without an agent: (HostRef, GPU count), gated by rccl-ready processes
    rccl_process_hosts: List[Any] = field(default_factory=list)
    rccl_process_ndev: List[int] = field(default_factory=list)
    rccl_skip_reason: str = ""
    # hostnames of rccl_hosts / rccl_process_hosts (same order): health-tainted ones leave the gate
    rccl_names: List[str] = field(default_factory=list)
    rccl_process_names: List[str] = field(default_factory=list)


@dataclass
class ReadinessReport:
    start: float
    phases: Dict[str, float] = field(default_factory=dict)
    nodes: Dict[str, Dict[str, Any]] = field(default_factory=dict)
    rccl: Optional[Dict[str, Any]] = None
    gpu_unhealthy: List[str] = field(default_factory=list)  # GPU nodes that joined health-tainted
    # label -> value -> GPU nodes, for labels whose value differs across the GPU nodes
    gpu_mismatch: Dict[str, Dict[str, List[str]]] = field(default_factory=dict)

    @property
    def ready_seconds(self) -> float:
        return max(self.phases.values()) - self.start if self.phases else 0.0

    def to_json(self) -> Dict[str, Any]:
        d = asdict(self)
        d["phase_seconds"] = {k: round(v - self.start, 4) for k, v in self.phases.items()}
        d["ready_seconds"] = round(self.ready_seconds, 4)
        return d


# node labels every MI355X node of one cluster should share (node/labels.py)
UNIFORM_LABELS = ("amd.com/gpu.product-name", "amd.com/gpu.vbios", "amd.com/gpu.target",
                  "amd.com/gpu.compute-partition", "amd.com/gpu.memory-partition", "amd.com/gpu.vram",
                  "amd.com/gpu.cu-count", "amd.com/rdma.link-layer", "amd.com/rdma.rate-gbps",
                  "amd.com/rocm.version", "amd.com/gpu.power-cap")


def gpu_mismatch(node_labels: Dict[str, Dict[str, str]]) -> Dict[str, Dict[str, List[str]]]:
    """The :data:`UNIFORM_LABELS` whose values differ across GPU nodes (``amd.com/gpu.present``);
    a node without the label counts as ``"-"`` when another node has it."""
    gpu = {n: lab for n, lab in node_labels.items() if lab.get("amd.com/gpu.present") == "true"}
    out: Dict[str, Dict[str, List[str]]] = {}
    for key in UNIFORM_LABELS:
        by: Dict[str, List[str]] = {}
        for n in sorted(gpu):
            by.setdefault(gpu[n].get(key, "-"), []).append(n)
        if len(by) > 1:
            out[key] = by
    return out


def _node_ready(item: Dict[str, Any]) -> bool:
    for c in (item.get("status") or {}).get("conditions", []) or []:
        if c.get("type") == "Ready":
            return c.get("status") == "True"
    return False


def wait_ready(client: RancherClient, spec: ReadinessSpec, start: Optional[float] = None,
               agent_transport: Any = None, gate: Any = None, host_transport: Any = None,
               tools_dir: Optional[str] = None) -> ReadinessReport:
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

    # GPU nodes that joined with the health taint: no device plugin, no gate ranks
    from ..node.health import has_health_taint

    unhealthy = {n for n in want if has_health_taint(items.get(n) or {})}
    rep.gpu_unhealthy = sorted(unhealthy)
    gpu_nodes = {h: n for h, n in spec.gpu_nodes.items() if h not in unhealthy}
    rccl_hosts, rccl_ndev = _healthy(spec.rccl_hosts, spec.rccl_ndev, spec.rccl_names, unhealthy)
    proc_hosts, proc_ndev = _healthy(spec.rccl_process_hosts, spec.rccl_process_ndev, spec.rccl_process_names,
                                     unhealthy)
    if gate is not None and len(rccl_hosts) != len(spec.rccl_hosts):
        gate.abort()  # prepared over a node that is now out of the gate
        gate = None

    if gpu_nodes:
        def gpus() -> Optional[Dict[str, Dict[str, Any]]]:
            got = {i["metadata"]["name"]: i for i in client.k8s_nodes(spec.cluster_id)}
            for host, n in gpu_nodes.items():
                alloc = ((got.get(host) or {}).get("status") or {}).get("allocatable", {})
                if str(alloc.get("amd.com/gpu", "0")) != str(n):
                    return None
            return got

        with span("ready.gpus", nodes=len(gpu_nodes)):
            items = wait_until(gpus, left(), "amd.com/gpu allocatable on every GPU node")
        rep.phases["gpus_allocatable"] = time.time()

    for name in want:
        it = items.get(name, {})
        rep.nodes[name] = {"labels": (it.get("metadata") or {}).get("labels", {}),
                           "allocatable": (it.get("status") or {}).get("allocatable", {})}
    rep.gpu_mismatch = gpu_mismatch({n: d["labels"] for n, d in rep.nodes.items()})

    if spec.rccl_gate and rccl_hosts:
        if gate is None:
            from .gate import ClusterGate, members_from

            gate = ClusterGate(agent_transport, members_from(rccl_hosts, rccl_ndev or None),
                               spec.rccl_sizes, spec.rccl_iters)
        with span("ready.rccl_gate", world=gate.world, nodes=len(gate.members)):
            rep.rccl = gate.run()
    elif spec.rccl_gate and proc_hosts:
        from ..node.plan import TOOLS_DIR
        from ..parallel.transport import TransportRouter
        from .process_gate import ProcessGate

        pgate = ProcessGate(host_transport or TransportRouter(), proc_hosts, proc_ndev,
                            spec.rccl_sizes, spec.rccl_iters, timeout=left(), tools_dir=tools_dir or TOOLS_DIR,
                            agent_transport=agent_transport)
        with span("ready.rccl_gate", world=pgate.world, nodes=len(proc_hosts), mode="process"):
            rep.rccl = pgate.run()
    elif spec.rccl_skip_reason:
        rep.rccl = {"ok": None, "skipped": spec.rccl_skip_reason}
    elif spec.rccl_gate and unhealthy:
        rep.rccl = {"ok": None, "skipped": "every MI355X node joined with the GPU health taint"}
    if rep.rccl is not None and "skipped" not in rep.rccl:
        if not rep.rccl.get("ok"):
            raise TKError(f"RCCL readiness gate failed: {rep.rccl}")
        rep.phases["rccl_gate"] = time.time()
    return rep


def _healthy(hosts: List[Any], ndev: List[int], names: List[str], unhealthy: set) -> "tuple[List[Any], List[int]]":
    """``hosts`` / ``ndev`` without the entries whose hostname is in ``unhealthy``."""
    if not unhealthy or not names:
        return list(hosts), list(ndev)
    keep = [i for i, n in enumerate(names) if n not in unhealthy]
    return [hosts[i] for i in keep], ([ndev[i] for i in keep] if ndev else [])


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
    from ..rancher import trust

    # verified against the manager's pinned CA (rancher/trust.py)
    client = trust.client(backend, state.name, mgr["rancher_url"], mgr.get("rancher_access_key", ""),
                          mgr.get("rancher_secret_key", ""))
    nodes = state.nodes(cluster_key)
    from ..models.baremetal import addons_key
    from ..state import cluster_key_parts

    # amd.com/gpu only appears once the device plugin runs, i.e. with the add-on module
    has_plugin = state.module(addons_key(cluster_key_parts(cluster_key)[1])) is not None
    from ..parallel.transport import HostRef

    gpu_nodes: Dict[str, int] = {}
    rccl_hosts: List[str] = []
    rccl_ndev: List[int] = []
    rccl_names: List[str] = []
    proc_hosts: List[HostRef] = []
    proc_ndev: List[int] = []
    proc_names: List[str] = []
    from ..node.partition import logical_gpus

    for host in sorted(nodes):
        cfg = state.module(nodes[host]) or {}
        info = module_from_source(str(cfg.get("source", "")))
        if info is not None and info.mi355x:
            # amd.com/gpu and RCCL ranks count logical GPUs: gpu_count x compute partitions
            n = logical_gpus(cfg)
            if has_plugin:
                gpu_nodes[host] = n
            addr = str(cfg.get("host", ""))
            if addr.startswith("agent+"):
                rccl_hosts.append(addr[len("agent+"):])
                rccl_ndev.append(n)
                rccl_names.append(host)
            elif addr:
                proc_hosts.append(HostRef(addr, cfg.get("ssh_user") or "ubuntu", cfg.get("key_path") or "",
                                          cfg.get("bastion_host") or ""))
                proc_ndev.append(n)
                proc_names.append(host)
    skip = ""
    if rccl_gate:
        if rccl_hosts and proc_hosts:
            # mixed delivery: one communicator through the process gate, whose agent members
            # join via their API (process_gate.py); host order is the rank order
            mixed = []
            for host in sorted(nodes):
                cfg = state.module(nodes[host]) or {}
                info = module_from_source(str(cfg.get("source", "")))
                if info is None or not info.mi355x or not cfg.get("host"):
                    continue
                addr = str(cfg["host"])
                ref = HostRef(addr, cfg.get("ssh_user") or "ubuntu", cfg.get("key_path") or "",
                              cfg.get("bastion_host") or "")
                mixed.append((ref, logical_gpus(cfg), host))
            proc_hosts, proc_ndev, proc_names = [m[0] for m in mixed], [m[1] for m in mixed], [m[2] for m in mixed]
            rccl_hosts, rccl_ndev, rccl_names = [], [], []
        elif not (rccl_hosts or proc_hosts):
            skip = "no MI355X nodes in the cluster"
    spec = ReadinessSpec(cl["rancher_cluster_id"], sorted(nodes), gpu_nodes, timeout,
                         rccl_gate and bool(rccl_hosts or proc_hosts), rccl_hosts, rccl_ndev,
                         rccl_process_hosts=proc_hosts, rccl_process_ndev=proc_ndev, rccl_skip_reason=skip,
                         rccl_names=rccl_names, rccl_process_names=proc_names)
    return client, spec


def gate_sizes(settings) -> List[int]:
    """RCCL gate message sizes: 1 MiB and ``rccl_gate_max_mib`` (default 64 MiB)."""
    mib = int(settings.get_float("rccl_gate_max_mib", 64))
    if mib < 1:
        raise TKError(f"rccl_gate_max_mib must be >= 1. Found '{mib}'.")
    return sorted({1 << 20, mib << 20})


def agent_transport_for(ctx, manager: str = "") -> Any:
    """The transport to the node agents: the caller's (``ctx.extras``), else one built on
    the cluster manager's agent PKI (per-node tokens, TLS against the manager's CA;
    ``node/security.py``).  ``agent_token`` (a shared token, development only) overrides."""
    transport = ctx.extras.get("agent_transport")
    if transport is None:
        from ..parallel.transport import AgentTransport

        shared = ctx.settings.get_string("agent_token")
        backend = ctx.extras.get("backend")
        if shared or backend is None or not manager:
            transport = AgentTransport(token=shared)
        else:
            from ..node.security import load_pki

            transport = AgentTransport(pki=load_pki(backend, manager))
        ctx.extras["agent_transport"] = transport
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

    gate = ClusterGate.from_state(state, cluster_key, agent_transport_for(ctx, state.name), gate_sizes(s))
    return gate.prepare_async() if gate is not None else None


def wait_after_create(ctx, backend, state, cluster_key: str, start: Optional[float] = None,
                      gate: Any = None) -> ReadinessReport:
    s = ctx.settings
    timeout = s.get_float("wait_timeout", 3600)
    client, spec = spec_from_state(state, backend, cluster_key, timeout, s.get_bool("rccl_gate"))
    spec.rccl_sizes = gate_sizes(s)
    mixed = any(h.scheme == "agent" for h in spec.rccl_process_hosts)
    transport = agent_transport_for(ctx, state.name) if spec.rccl_gate and (spec.rccl_hosts or mixed) else None
    if gate is not None and (not spec.rccl_hosts or gate.world != sum(spec.rccl_ndev or [1] * len(spec.rccl_hosts))):
        gate.abort()  # membership changed since it was prepared
        gate = None
    rep = wait_ready(client, spec, start=start, agent_transport=transport, gate=gate,
                     host_transport=ctx.extras.get("transport"),
                     tools_dir=s.get_string("node_tools_dir") or None)
    ctx.extras["last_readiness"] = rep  # callers that time phases (bench.py) read it here
    ctx.echo(f"cluster ready in {rep.ready_seconds:.2f}s: " +
             json.dumps(rep.to_json()["phase_seconds"], sort_keys=True))
    if rep.gpu_unhealthy:
        ctx.echo("GPU nodes joined with the health taint (no GPU pods, not in the RCCL gate): "
                 + ", ".join(rep.gpu_unhealthy) + " -- see `triton-kubernetes health cluster`")
    for key, by in sorted(rep.gpu_mismatch.items()):
        ctx.echo(f"warning: MI355X nodes differ in {key}: "
                 + "; ".join(f"{v}: {', '.join(ns)}" for v, ns in sorted(by.items())))
    return rep


__all__ = ["ReadinessSpec", "ReadinessReport", "UNIFORM_LABELS", "gpu_mismatch", "wait_ready", "rccl_gate", "spec_from_state", "wait_after_create",
           "early_gate", "agent_transport_for", "gate_sizes"]
