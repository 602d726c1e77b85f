#!/usr/bin/env python3
"""Headline benchmark: cluster create -> kubectl-ready wall-clock, bare-metal MI355X.

Metric (BASELINE.json): "cluster create->kubectl-ready wall-clock (s),
bare-metal at 1/2/4/8 workers", measured on config #5: "create cluster MI355X
bare-metal N-worker + ROCm device-plugin + xGMI topology labels".

Shape.  ``--gpus N`` is the number of MI355X GPUs the cluster's worker tier owns.  By
default ONE worker node owns all of them -- one node agent with ``devices=0..N-1``, as on a
real 8xMI355X node, so the per-node steps (burn-in of every GPU concurrently, topology
labels) and the RCCL gate (``ndev=N`` grouped communicator init in one agent) run at node
scale.  ``--workers W`` splits the N GPUs over W agents instead.  The launch
(:func:`resolve_gpus`): without a launcher one process drives all N GPUs (fewer visible:
the run fails with its reason, never a smaller measurement); under ``torchrun`` there is
one rank per GPU (``WORLD_SIZE == N``), and when the launcher masks devices per rank (each
rank sees only its own GPU) every rank runs one 1-GPU agent.  :class:`RunBudget` keeps the
run inside the driver's wall-clock limit by shedding untimed secondary work only.

Each timed step is a COLD create:

1. fresh node-agent processes start (``python -m triton_kubernetes_amd.node.agent``:
   HIP/RCCL load, burn-in arena allocation, RCCL unique id -- nothing carried over
   from earlier steps), plus a fresh control-plane agent;
2. ``create cluster`` runs through the framework's real code path -- settings ->
   bare-metal provider -> ``main.tf.json`` -> DirectExecutor DAG -> Rancher client ->
   parallel node bootstrap (per-GPU HBM/MFMA/memtest burn-in and topology labels,
   for real on the MI355X) -> add-ons -> readiness waiter (cluster active, nodes Ready,
   ``amd.com/gpu`` allocatable, cluster-wide RCCL all-reduce gate across all N GPUs);
3. the agents shut down (communicator teardown, HIP release), inside the step.

The GPU node runs the product's default burn-in level (``full``: HBM/MFMA screens plus a
memtest of all free HBM, ``models/baremetal.py`` DEFAULT_BURNIN); ``--burnin quick`` is the
explicit opt-down and the line's ``config.burnin`` names the level.  Before every timed step,
outside the timed region, the bench waits until the kernel driver has finished clearing the
HBM the previous step released (``ops/hbm.py``; ``hbm_settle_s`` in the line): a node
entering service starts with clear HBM, so no step pays its predecessor's ~300 GB release.

Node state carried across steps, as on a real node after its first GPU process: the page
cache and the HIP runtime's code-object cache (ROCm comgr, on by default, ``~/.cache/comgr``),
which the warmup's first RCCL init fills with librccl's unbundled gfx950 code.  A box's very
first RCCL init takes ~5.5 s; later processes ~1.8 s.  On a box whose cache is cold the bench
first loads RCCL's device code once in a throw-away process, as a booted node's agent has
(``config.comgr_cache``: its size before and after the warmup, ``prewarm_s``).

``value`` is the mean create -> kubectl-ready time (agent start to readiness);
``ms_per_step`` is the whole step including the agent shutdown.  A WARM number (the
same create against agents kept resident across steps, round 1's headline) is
reported only as the secondary ``warm_create_to_ready_s``, measured after the timed
region, each create after the same untimed HBM settle as a cold step
(``warm_hbm_settle_s``: the previous create's burn-in release being cleared).

The cluster is an RKE2 custom cluster (``provisioning.cattle.io/v1``, the default
distribution of the pinned Rancher v2.10.3, versions.py).  Simulated
(``config.simulated_phases``): the Rancher server is the in-process fake, so RKE2
provisioning is instantaneous (``rke_provisioning``); the host steps (``runtime_install``:
firewall, hostname) are sim-mode no-ops of the agents, and the node join
(``agent_container``) fetches the server's ``system-agent-install.sh`` and registers as
``rancher-system-agent`` through the fake's connect API instead of running the installer.
The device-plugin DaemonSet's pod is scheduled by the fake's kubelet model (image, kubelet
socket and ``/sys`` mounts, node selector, taints) and registers instantly
(``device_plugin_pod``).  The reference publishes no number for this metric, so ``vs_baseline`` is null.

Rank 0 prints one JSON line (the driver's contract).
"""

import argparse
import json
import math
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import time

_T_START = time.monotonic()  # the run's wall clock starts with this process (the budget's origin)
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "cluster create→kubectl-ready wall-clock (s), bare-metal at 1/2/4/8 workers"
SIMULATED_PHASES = ["rke_provisioning", "runtime_install", "agent_container", "device_plugin_pod"]


def comgr_cache_dir() -> str:
    """Where the HIP runtime's code-object cache lives (ROCm comgr, on by default): unbundled
    and decompressed device code, keyed by its input.  librccl's gfx950 code comes out of a
    13-target bundle; a process finding it here starts its first communicator in ~1.8 s
    instead of ~5.5 s (profiles/round5/README.md)."""
    if os.environ.get("AMD_COMGR_CACHE_DIR"):
        return os.environ["AMD_COMGR_CACHE_DIR"]
    base = os.environ.get("XDG_CACHE_HOME") or os.path.join(os.path.expanduser("~"), ".cache")
    return os.path.join(base, "comgr")


def dir_mib(path: str) -> float:
    total = 0
    for root, _, files in os.walk(path):
        for f in files:
            try:
                total += os.path.getsize(os.path.join(root, f))
            except OSError:
                pass
    return round(total / 2**20, 1)


COMGR_WARM_MIB = 256  # librccl's unbundled gfx950 code is ~540 MiB; less: the cache is cold


def _prewarm_code() -> str:
    return ("import sys, time\n"
            f"sys.path.insert(0, {HERE!r})\n"
            "from triton_kubernetes_amd.ops import rccl\n"
            "rccl.preload_device_code([0])\n"
            "while rccl.preloads_running():\n"
            "    time.sleep(0.01)\n"
            "rccl.exit_now(0)\n")


def prewarm_comgr(timeout: float = 300.0) -> float:
    """The node's first GPU process after boot, before the timed region: load RCCL's device
    code once in a throw-away process (``tkr_preload_device_code``), which fills the HIP
    code-object cache as a booted node's agent does.  Returns its seconds."""
    code = _prewarm_code()
    t0 = time.perf_counter()
    subprocess.run([sys.executable, "-c", code], timeout=timeout, check=False,
                   env=dict(os.environ, PYTHONPATH=HERE + os.pathsep + os.environ.get("PYTHONPATH", "")))
    return round(time.perf_counter() - t0, 2)


def _default_burnin() -> str:
    from triton_kubernetes_amd.models.baremetal import DEFAULT_BURNIN

    return DEFAULT_BURNIN


def _stop_phases(results) -> dict:
    per_step = []
    for r in results:
        docs = [d for name, d in (r.get("agent_stop_ms") or {}).items() if name.startswith("mi355x") and d]
        if docs:
            per_step.append({k: max(float(d.get(k) or 0.0) for d in docs) for k in docs[0]})
    keys = sorted({k for st in per_step for k in st})
    return {k: round(sum(st.get(k, 0.0) for st in per_step) / len(per_step), 1) for k in keys} if per_step else {}


def settle_cards(hbm, cards, floor: list, resident: bool, timeout_s=None) -> dict:
    """One untimed wait for the driver's clearing on ``cards`` (``ops/hbm.py:settle``).
    ``floor[0]`` is the clean used-HBM level, measured by the first wait and kept for the
    next.  ``resident``: agents stay up across the waits and hold HBM of their own, so the
    cold clean level is out of reach; a wait that ends on its quiet window instead records
    the level it ended at as the floor of the later resident waits.  ``timeout_s``: the
    run budget's cap on this wait (:class:`RunBudget`), None for the settle's own limit."""
    got = hbm.settle(cards=cards, floor=floor[0], **({} if timeout_s is None else {"timeout_s": timeout_s}))
    if not resident:
        floor[0] = got["floor_by_card"]  # per card: one card still clearing is waited for
    elif not got.get("reached_floor") and not got.get("timed_out"):
        floor[0] = dict(hbm.vram_used(cards=cards))
    return got


class RunBudget:
    """Keeps one bench run inside the driver's wall-clock limit (its BENCH record shows
    ``timeout_s`` 600) without touching what is measured.

    Untimed work dominates a run: before each cold step the wait for the driver to clear
    the previous step's ~280 GB-per-GPU release (8.4 s per step on one GPU, against a
    2.3 s step), and after the timed region the secondary warm creates.  On an 8-GPU node
    nobody has measured whether the driver clears eight cards in parallel; if it serialises
    them, 25 settles would outlast any limit before the line prints.

    After every step (warmup or timed) :meth:`plan` projects the run's end from what the
    steps so far cost -- the slowest settle and the slowest step of the last few, for each
    step still to come, plus the warm creates -- and, while the projection exceeds
    ``budget_s``, sheds secondary work in this order:

    1. ``warm_creates``: the secondary warm creates are skipped (``warm_create_to_ready_s``
       null);
    2. ``hbm_settle_capped``: each later settle waits at most what is left per remaining
       step, so a step may start before the driver has finished clearing -- the step then
       pays that clearing inside its timed region, which can only make ``value`` worse.

    Every projection decides afresh: a run that caught up (a slow cold first step, then
    ordinary ones) lifts the cap again, and the warm creates run if the time is there when
    the timed steps are done.  ``shed`` reports what was actually given up.  The
    ``--warmup`` and ``--steps`` counts are never cut: the line's ``steps`` and ``warmup``
    are what ran.  ``budget_s`` 0 turns the guard off."""

    TAIL_S = 15.0  # after the last step: the agents' stop, the report, the process exit
    RECENT = 3  # the projection prices each step still to come at the slowest of the last 3

    def __init__(self, budget_s: float, t0: float = None, clock=time.monotonic):
        self.budget_s = float(budget_s or 0.0)
        self.clock = clock
        self.t0 = _T_START if t0 is None else t0
        self.settles = []
        self.steps = []
        self._natural = []  # what each settle would have taken: its wait, or more when cut
        self.caps_used = []  # the cap each capped settle ran under
        self.projected_s = None
        self.settle_cap_s = None
        self.warm_allowed = True

    @property
    def shed(self) -> list:
        return (["warm_creates"] if not self.warm_allowed else []) + (["hbm_settle_capped"] if self.caps_used else [])

    def record(self, settle_s: float, step_s: float, settle_cut: bool = False) -> None:
        """One settle and the step after it; the settle ran under the cap in force now.
        ``settle_cut``: the wait ended at its limit, not on the clearing done, so the clearing
        would have taken longer: the projection keeps pricing settles at what they took
        before rather than at the cut (a cap priced from its own cut waits would lift itself
        and let the next full-length settle overrun the budget)."""
        self.settles.append(float(settle_s))
        self.steps.append(float(step_s))
        nat = float(settle_s)
        if settle_cut and self._natural:
            nat = max(nat, self._natural[-1])
        self._natural.append(nat)
        if self.settle_cap_s is not None:
            self.caps_used.append(self.settle_cap_s)

    def plan(self, cold_left: int, warm_creates: int) -> None:
        """Re-project after a step; ``cold_left`` cold steps (warmup + timed) and
        ``warm_creates`` warm creates (each with its own settle) are still to run."""
        if not self.steps:
            return
        # the slowest of the last few: a cold first step (fresh box) stops counting once the
        # run has settled, a node whose clears grow keeps counting them
        settle, step = max(self._natural[-self.RECENT:]), max(self.steps[-self.RECENT:])
        elapsed = self.clock() - self.t0
        warm = (settle + step) * warm_creates
        base = elapsed + cold_left * (settle + step) + self.TAIL_S
        self.projected_s = round(base + warm, 1)
        if not self.budget_s or base + warm <= self.budget_s:
            self.warm_allowed, self.settle_cap_s = True, None
            return
        self.warm_allowed = not warm  # nothing to shed when no warm create is left
        if base <= self.budget_s or not cold_left:
            self.settle_cap_s = None
            return
        # rounded down: a cap rounded up by 5 ms per settle would add up over a long run
        self.settle_cap_s = math.floor(max(0.0, (self.budget_s - elapsed - self.TAIL_S - cold_left * step) / cold_left)
                                       * 100) / 100

    def report(self) -> dict:
        return {"budget_s": self.budget_s or None, "projected_s": self.projected_s, "shed": self.shed,
                "settle_cap_s": min(self.caps_used) if self.caps_used else None, "capped_settles": len(self.caps_used),
                "elapsed_s": round(self.clock() - self.t0, 1)}


def resolve_gpus(requested: int, world: int, visible: int, sim: bool, masked_env: bool = False) -> dict:
    """How many GPUs the run measures, and how; raises :class:`GpuCountError` rather than
    measuring fewer GPUs than asked.

    * No launcher (``WORLD_SIZE`` unset or 1): ``--gpus N`` means N GPUs of this node, all
      owned by this one process -- one node agent over devices 0..N-1, as a real 8xMI355X
      node runs one agent.  Fewer than N visible is an error.
    * Under ``torchrun``: one rank per GPU, so ``WORLD_SIZE`` must equal ``--gpus``.  A
      launcher that masks each rank to its own GPU (fewer visible than ranks) gets one
      1-GPU agent per rank."""
    if requested < 1:
        raise GpuCountError(f"--gpus {requested}: at least 1 GPU")
    if world > 1 and world != requested:
        raise GpuCountError(f"--gpus {requested} but WORLD_SIZE {world}: launch one rank per GPU")
    if sim:
        visible = requested
    masked = world > 1 and (visible < requested or masked_env)
    if masked and visible < 1:
        raise GpuCountError(f"{requested} GPUs requested, {visible} visible to rank")
    if not masked and visible < requested:
        raise GpuCountError(f"{requested} GPUs requested, {visible} visible")
    return {"n_gpus": requested, "visible": visible, "masked": masked}


class GpuCountError(RuntimeError):
    pass


def _at_least(lo, kind=int):
    """An argparse type: a finite number of ``kind`` >= ``lo`` (``--steps 0`` would time
    nothing and divide by zero; a negative warm-up or budget means nothing)."""
    def parse(text):
        try:
            v = kind(text)
        except ValueError:
            raise argparse.ArgumentTypeError(f"not a{'n integer' if kind is int else ' number'}: {text!r}")
        if not math.isfinite(v) or v < lo:
            raise argparse.ArgumentTypeError(f"must be a finite number >= {lo}: {text!r}")
        return v

    parse.__name__ = kind.__name__
    return parse


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=_at_least(1), default=1)
    ap.add_argument("--steps", type=_at_least(1), default=3)
    ap.add_argument("--warmup", type=_at_least(0), default=1)
    ap.add_argument("--workers", type=_at_least(1), default=1, help="worker nodes the N GPUs are split over")
    # the product's default level (models/baremetal.py DEFAULT_BURNIN, pinned by
    # tests/test_bench_contract.py); quick is the explicit opt-down
    ap.add_argument("--burnin", default=_default_burnin(), choices=["quick", "full", "off"])
    ap.add_argument("--hbm-settle", default="on", choices=["on", "off"],
                    help="on: before each step, outside the timed region, wait until the kernel driver has "
                         "finished clearing the HBM the previous step released (ops/hbm.py), as on a node "
                         "entering service.  off: the A/B (each step pays its predecessor's clearing)")
    ap.add_argument("--no-rccl-gate", action="store_true")
    ap.add_argument("--rccl-mib", type=_at_least(1), default=64, help="largest RCCL gate message (MiB)")
    ap.add_argument("--warm-steps", type=_at_least(0), default=2,
                    help="secondary: creates against resident agents after the timed region (0: skip)")
    ap.add_argument("--agents", default="proc", choices=["proc", "inproc"],
                    help="proc: every agent in its own fresh process (the headline); inproc: agents as "
                         "objects in this process (the graft smoke: native libraries load here)")
    ap.add_argument("--rccl-slim", default="off", choices=["on", "off"],
                    help="on: the node's opt-in single-target gfx950 RCCL copy (ops/rccl_slim.py), prepared and "
                         "verified before the timed region, loaded by the agents (TK_HIP_RUNTIME=slim). Default "
                         "off: the agents load /opt/rocm's HIP runtime and RCCL, the product default")
    ap.add_argument("--gpu-health", default="taint", choices=["fail", "taint", "off"],
                    help="the GPU node's health policy (node/health.py).  taint (bench default): a GPU with "
                         "uncorrectable ECC errors does not abort the run; the node joins tainted and the line "
                         "lists it under gpu_unhealthy_nodes (its GPUs then sit out the GPU and RCCL checks)")
    ap.add_argument("--link-min-gbps", type=_at_least(0.0, float), default=0.0,
                    help="the GPU node's absolute xGMI link floor (gpu_link_min_gbps; the product default is 38). "
                         "The bench records the link matrix (xgmi_links in the line) rather than certifying it: "
                         "0 keeps only the relative check (a link below half the node's median still fails)")
    ap.add_argument("--sim-gpu", action="store_true",
                    help="CPU dry run: synthetic topology, no burn-in kernels; the cluster RCCL gate runs over the "
                         "libtk_rccl ABI stub (ops/csrc/tk_rccl_stub.cpp: every rank of the world joins and sweeps, "
                         "no GPU); never a valid measurement")
    ap.add_argument("--report", default="", help="write a per-step phase report (rank 0) to this file")
    ap.add_argument("--time-budget", type=_at_least(0.0, float), default=480.0,
                    help="wall-clock seconds the whole run should stay within (RunBudget): past it the secondary "
                         "warm creates are shed, then the untimed settle waits are capped; the timed steps never "
                         "are.  0: off")
    return ap.parse_args(argv)


class AgentProc:
    """One node agent in its own process (what systemd runs on a real node), serving TLS
    with the credentials its cluster manager issued for its address (node/security.py)."""

    def __init__(self, name: str, devices, creds_dir: str, address: str, root: str, synthetic: int = 0,
                 client_ctx=None):
        with open(os.path.join(creds_dir, "agent-token"), "r", encoding="utf-8") as fh:
            self.token = fh.read().strip()
        self.client_ctx = client_ctx
        argv = [sys.executable, "-u", "-m", "triton_kubernetes_amd.node.agent", "--mode", "sim",
                "--listen", f"{address}:0", "--name", name, "--credentials", creds_dir, "--root", root,
                "--devices", ",".join(str(d) for d in devices)]
        if synthetic:
            argv += ["--synthetic-gpus", str(synthetic)]
        env = dict(os.environ, PYTHONPATH=HERE + os.pathsep + os.environ.get("PYTHONPATH", ""))
        self.name = name
        self.proc = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=None, text=True, env=env,
                                     start_new_session=True)
        self.url = ""
        self.runtime = ""
        self.startup_ms = {}
        self.signalled = False

    def wait_url(self, timeout: float = 300.0) -> str:
        # the agent prints one JSON line once it serves (native libraries loaded, arena ready)
        import selectors

        sel = selectors.DefaultSelector()
        sel.register(self.proc.stdout, selectors.EVENT_READ)
        deadline = time.monotonic() + timeout
        while not self.url:
            if self.proc.poll() is not None:
                raise RuntimeError(f"agent {self.name} exited {self.proc.returncode} before serving")
            if not sel.select(timeout=max(0.0, deadline - time.monotonic())):
                raise RuntimeError(f"agent {self.name} did not start within {timeout:.0f}s")
            line = self.proc.stdout.readline()
            if line.startswith("{"):
                doc = json.loads(line)
                self.url = doc["listening"]
                self.runtime = doc.get("hip_runtime", "")
                self.startup_ms = doc.get("startup_ms", {})
                self.preload = doc.get("rccl_preload") or {}
        sel.close()
        return self.url

    def signal_stop(self) -> None:
        """Ask the agent to stop (its API; a signal if that fails)."""
        if self.proc.poll() is not None or self.signalled:
            return
        self.signalled = True
        import urllib.request

        try:
            req = urllib.request.Request(self.url + "/v1/shutdown", data=b"{}", method="POST",
                                         headers={"X-TK-Agent-Token": self.token,
                                                  "Content-Type": "application/json"})
            urllib.request.urlopen(req, timeout=10, context=self.client_ctx).read()
        except OSError:
            self.proc.send_signal(signal.SIGTERM)

    def stop(self, timeout: float = 120.0) -> int:
        if self.proc.poll() is None:
            self.signal_stop()
            try:
                self.proc.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                os.killpg(self.proc.pid, signal.SIGKILL)
                self.proc.wait()
        try:  # the agent's last line: where its shutdown's time went
            for ln in self.proc.stdout.read().splitlines():
                if ln.startswith("{") and '"stopped"' in ln:
                    doc = json.loads(ln)
                    self.stop_ms = dict(doc.get("stop_phases_ms") or {}, total=doc.get("stop_ms"))
        except (OSError, ValueError):
            pass
        self.proc.stdout.close()
        return self.proc.returncode


class InprocAgent:
    """Same interface as :class:`AgentProc`, the agent living in this process."""

    def __init__(self, name: str, devices, creds_dir: str, address: str, root: str, synthetic: int = 0):
        from triton_kubernetes_amd.node.agent import NodeAgent
        from triton_kubernetes_amd.node.security import read_credentials

        creds = read_credentials(creds_dir)
        self.name = name
        self.agent = NodeAgent(name=name, mode="sim", devices=list(devices), token=creds["token"], root=root,
                               policy=creds["policy"])
        if synthetic:
            from triton_kubernetes_amd.node.labels import synthetic_topology

            self.agent.topology_override = synthetic_topology(synthetic)
            self.agent.burnin_override = lambda dev, level: {"ok": True, "simulated": True, "level": level}
        self.url = self.agent.serve(address, ssl_context=creds["ssl_context"])
        self.preload = getattr(self.agent, "rccl_preload", None)

    def wait_url(self, timeout: float = 0.0) -> str:
        return self.url

    def signal_stop(self) -> None:
        pass

    def stop(self, timeout: float = 0.0) -> int:
        self.agent.stop()
        return 0


def failure_line(args, n_gpus, workers, gpus_per_worker, visible, error: str, completed: int = 0) -> dict:
    """The line's shape for a run that measured nothing (``value`` null) and why."""
    return {
        "metric": METRIC, "value": None, "unit": "s", "n_gpus": n_gpus, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": None, "higher_is_better": False, "scaling": "weak",
        "vs_baseline": None, "dtype": "n/a", "data": "FAILED: no measurement",
        "config": {"model": "create cluster MI355X bare-metal N-worker + ROCm device-plugin + xGMI topology "
                            "labels", "workers": workers, "gpus_per_worker": gpus_per_worker,
                   "visible_gpus": visible, "global_batch": "n/a", "seq_len": "n/a",
                   "parallelism": f"{workers} worker node(s) x {gpus_per_worker} GPU(s)",
                   "burnin": args.burnin, "rccl_gate": not args.no_rccl_gate},
        "error": error[:2000], "completed_steps": completed}


def main() -> int:
    args = parse_args()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # counting devices does not initialise HIP on this image; set_device below does
    visible = 0 if args.sim_gpu else torch.cuda.device_count()
    try:
        shape = resolve_gpus(args.gpus, world, visible, args.sim_gpu,
                             masked_env=os.environ.get("TK_BENCH_ASSUME_MASKED") == "1")
    except GpuCountError as exc:
        # never measure fewer GPUs than asked: the line says what was wrong, and the run fails
        if rank == 0:
            print(json.dumps(failure_line(args, args.gpus, None, None, visible, str(exc))), flush=True)
        print(f"bench: {exc}", file=sys.stderr)
        return 2
    n_gpus, visible, masked = shape["n_gpus"], shape["visible"], shape["masked"]
    distributed = world > 1
    if distributed:
        # control-plane sync only (CPU); the GPU collectives are the agents' native RCCL gate
        dist.init_process_group("gloo", init_method="env://")
    if args.sim_gpu:
        if not args.no_rccl_gate:
            # the gate over the C ABI stub: the agents (this process's and their children)
            # join one rendezvous directory, shared by every rank
            from triton_kubernetes_amd.ops import native
            from triton_kubernetes_amd.ops.build import build as build_native

            if rank == 0:
                build_native(only=["libtk_rccl_stub.so"])
            where = [tempfile.mkdtemp(prefix="tk-bench-rccl-stub-") if rank == 0 else None]
            if distributed:
                dist.broadcast_object_list(where, src=0)
            os.environ.update(TK_RCCL_LIB=os.path.join(native.LIB_DIR, "libtk_rccl_stub.so"),
                              TK_RCCL_STUB_DIR=where[0], TK_GATE_BACKEND="rccl")
    else:
        torch.cuda.set_device(0 if masked else min(local_rank, visible - 1))

    # which agents this rank owns: (name, devices).  Unmasked (one process, or ranks that
    # all see the node's GPUs): rank 0 owns every worker agent over devices 0..N-1; masked
    # (each rank sees only its own GPU): every rank owns a 1-GPU agent.
    if masked:
        workers = n_gpus
        mine = [(f"mi355x-{rank}", [0])]
    else:
        workers = max(1, min(args.workers, n_gpus))
        if n_gpus % workers:
            if rank == 0:
                print(json.dumps(failure_line(args, n_gpus, workers, None, visible,
                                              f"--workers {workers} does not divide {n_gpus} GPUs")), flush=True)
            return 2
        per = n_gpus // workers
        mine = [(f"mi355x-{w}", list(range(w * per, (w + 1) * per))) for w in range(workers)] if rank == 0 else []
    gpus_per_worker = n_gpus // workers
    budget = RunBudget(args.time_budget)
    if rank == 0:
        print(f"bench: {n_gpus} GPU(s), {workers} worker(s) x {gpus_per_worker}, world {world}"
              f"{' (masked ranks)' if masked else ''}, burn-in {args.burnin}, {args.warmup} warmup + {args.steps} steps",
              file=sys.stderr, flush=True)

    from triton_kubernetes_amd import versions
    from triton_kubernetes_amd import workflows as wf
    from triton_kubernetes_amd.backend import LocalBackend
    from triton_kubernetes_amd.config import Context, Settings
    from triton_kubernetes_amd.utils.trace import TRACER, span

    slim_meta = None
    os.environ.setdefault("TK_HIP_RUNTIME", "system")  # inherited by the agent processes
    if args.rccl_slim == "on" and not args.sim_gpu:
        # the node's opt-in (one-time per RCCL build, cached, verified by a one-rank
        # all-reduce before first use); outside the timed region, like the OS image
        from triton_kubernetes_amd.ops import native, rccl_slim

        if local_rank == 0:
            slim_meta = rccl_slim.prepare(native.SYSTEM_LIB_DIR)
        if distributed:
            dist.barrier()
        os.environ["TK_HIP_RUNTIME"] = "slim"

    work = tempfile.mkdtemp(prefix=f"tk-bench-r{rank}-")
    synthetic = gpus_per_worker if args.sim_gpu else 0
    fake = backend = ctx_base = None
    devnull = open(os.devnull, "w", encoding="utf-8")  # workflow output (one handle for every step)
    if rank == 0:
        from triton_kubernetes_amd.rancher.fake import FakeRancher

        fake = FakeRancher().start()  # a random first-login password, given as rancher_bootstrap_password
        backend = LocalBackend(os.path.join(work, "state"))
        ctx_base = {"backend_provider": "local", "executor": "direct", "non-interactive": True,
                    "cluster_manager": "bench"}
        mgr = dict(ctx_base, manager_cloud_provider="baremetal", name="bench", rancher_admin_password="bench-admin-pw-0123",
                   rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="ubuntu", bastion_host="", key_path="~/.ssh/id_rsa")
        wf.new_manager(Context(settings=Settings(mgr, env={}), out=devnull), backend)

    # node enrollment (install time, before the timed region): the manager's agent PKI
    # issues each node a TLS certificate for its address, its own token and the allow-list
    # (the manager's agent image; its Rancher server, whose RKE2 installer the node runs).  Every simulated node gets its own loopback address.
    from triton_kubernetes_amd.node.security import AgentPKI, load_pki

    pki_doc = [load_pki(backend, "bench").to_json() if rank == 0 else None, fake.url if rank == 0 else None]
    if distributed:
        dist.broadcast_object_list(pki_doc, src=0)
    pki, rancher_url = AgentPKI.from_json(pki_doc[0]), pki_doc[1]
    addresses = {name: f"127.1.{rank}.{2 + k}" for k, (name, _) in enumerate(mine)}
    if rank == 0:
        addresses["control-plane"] = "127.1.0.250"
    creds = {}
    for name, addr in addresses.items():
        creds[name] = os.path.join(work, "creds", name)
        pki.issue(addr, [versions.AGENT_IMAGE], servers=[rancher_url],
                  distributions=[versions.DEFAULT_DISTRIBUTION]).write(creds[name])
    client_ctx = pki.client_context()

    from triton_kubernetes_amd.node.agent_gate import AgentGateMixin

    last_root = {}  # agent name -> its root in the previous step

    def start_agents(tag: str):
        names = [(name, devs) for name, devs in mine] + ([("control-plane", [])] if rank == 0 else [])
        for name, _ in names:
            # what a real node keeps across agent restarts and clusters: the gate footprints
            # its earlier gates measured (the burn-in's headroom, node/agent_gate.py).  Every
            # other file of the root is fresh (a cold step: a new cluster's join, new labels)
            root = os.path.join(work, tag, name)
            prev = os.path.join(last_root.get(name, ""), AgentGateMixin.FOOTPRINT_FILE.lstrip("/"))
            if name in last_root and os.path.exists(prev):
                dst = os.path.join(root, AgentGateMixin.FOOTPRINT_FILE.lstrip("/"))
                os.makedirs(os.path.dirname(dst), exist_ok=True)
                shutil.copyfile(prev, dst)
            last_root[name] = root
        if args.agents == "inproc":
            return [InprocAgent(name, devs, creds[name], addresses[name], os.path.join(work, tag, name),
                                synthetic if devs else 0) for name, devs in names]
        return [AgentProc(name, devs, creds[name], addresses[name], os.path.join(work, tag, name),
                          synthetic if devs else 0, client_ctx) for name, devs in names]

    runtimes = set()
    preloads = set()  # the GPU agents' RCCL device-code preload handle (how:symbol)

    def gather_urls(procs):
        local = [(p.name, p.wait_url()) for p in procs]
        runtimes.update(getattr(p, "runtime", "") or "in-process" for p in procs if p.name != "control-plane")
        preloads.update("{how}:{symbol}".format(**(getattr(p, "preload", None) or {"how": "none", "symbol": "none"}))
                        for p in procs if p.name != "control-plane")
        if distributed:
            every = [None] * world
            dist.all_gather_object(every, local)
            local = [x for part in every for x in part]
        return dict(local)

    def create(i: int, urls) -> dict:
        """rank 0: one ``create cluster --wait`` against the agents at ``urls``."""
        name = f"bench-{i}".replace("--", "-w")
        cp = "agent+" + urls["control-plane"]
        gpu_hosts = ["agent+" + urls[f"mi355x-{w}"] for w in range(workers)]
        cfg = dict(ctx_base, cluster_cloud_provider="baremetal", name=name, k8s_version=versions.DEFAULT_K8S_VERSION,
                   k8s_network_provider="flannel", gpu_addons=True, wait=True,
                   rccl_gate=not args.no_rccl_gate, rccl_gate_max_mib=args.rccl_mib, wait_timeout=600,
                   nodes=[
                       {"rancher_host_label": "control", "node_count": 1, "hostname": f"{name}-cp",
                        "ssh_user": "ubuntu", "bastion_host": "", "key_path": "k", "hosts": [cp]},
                       {"rancher_host_label": "etcd", "node_count": 1, "hostname": f"{name}-etcd",
                        "ssh_user": "ubuntu", "bastion_host": "", "key_path": "k", "hosts": [cp]},
                       {"rancher_host_label": "worker", "node_count": workers, "hostname": f"{name}-gpu",
                        "ssh_user": "ubuntu", "bastion_host": "", "key_path": "k", "hosts": gpu_hosts,
                        "gpu": "mi355x", "gpu_count": gpus_per_worker, "gpu_burnin": args.burnin,
                        "gpu_health": args.gpu_health, "gpu_link_min_gbps": str(args.link_min_gbps)},
                   ])
        # the CLI's own agent transport: per-node tokens + TLS against the manager's CA
        ctx = Context(settings=Settings(cfg, env={}), out=devnull)
        wf.new_cluster(ctx, backend)
        out = {}
        report = ctx.extras.get("last_apply")
        if report is not None:  # the GPU nodes' plan steps as the agents timed them
            steps = {}
            for key, run in report.runs.items():
                detail = run.detail if isinstance(run.detail, dict) else {}
                if run.info.mi355x:
                    for st in detail.get("steps", []) or []:
                        steps[st.get("name")] = max(steps.get(st.get("name"), 0.0), float(st.get("ms") or 0.0))
                        if st.get("name") == "gpu_burnin" and isinstance(st.get("detail"), dict):
                            # each screen's wall time and the memtest's allocation, max over GPUs
                            bp = out.setdefault("burnin_phase_ms", {})
                            for res in st["detail"].values():
                                if not isinstance(res, dict):
                                    continue
                                mt = res.get("memtest") or {}
                                for k, v in list((res.get("phase_ms") or {}).items()) + [
                                        ("memtest.alloc", mt.get("alloc_ms")), ("memtest.test", mt.get("test_ms")),
                                        ("memtest.process", mt.get("process_ms"))]:
                                    if v is not None:
                                        bp[k] = round(max(bp.get(k, 0.0), float(v)), 1)
                        links = st.get("detail") if st.get("name") == "gpu_links" else None
                        if isinstance(links, dict) and links.get("labels"):
                            # the measured xGMI matrix (node/labels.py:link_labels), per worker
                            lab = links["labels"]
                            out.setdefault("xgmi_links", []).append({
                                "status": links.get("status"), "min_gbps": float(lab.get("amd.com/xgmi.p2p-min-gbps", 0)),
                                "median_gbps": float(lab.get("amd.com/xgmi.p2p-median-gbps", 0)),
                                "method": lab.get("amd.com/xgmi.p2p-method"), "floor_gbps": links.get("floor_gbps"),
                                "remeasured": links.get("remeasured", 0)})
            if steps:
                out["gpu_node_step_ms"] = {k: round(v, 1) for k, v in steps.items()}
        rep = ctx.extras.get("last_readiness")
        if rep is not None:
            out["phase_s"] = rep.to_json()["phase_seconds"]
            out["gpu_unhealthy"] = list(rep.gpu_unhealthy)
            ranks = (rep.rccl or {}).get("ranks") or []
            out["rccl_gate_ranks"] = sum(len(r.get("ranks") or []) for r in ranks)
            phases = [r.get("phase_ms") or {} for r in ranks]
            if phases:  # the gate's communicator phases, max over agents
                out["rccl"] = {k: round(max(float(p.get(k, 0.0)) for p in phases), 3)
                               for k in ("init_total", "init_wait", "alloc", "sweep", "footprint_mib",
                                         "footprint_total_mib", "footprint_kind")}
                # 1 when every agent kept its measurement as a footprint (node/agent_gate.py)
                out["rccl"]["footprint_kept"] = min(float(p.get("footprint_kept", 0.0)) for p in phases)
            # an init that ran out of HBM beside the held burn-in spans and was retried
            retried = [r.get("gate_retry") for r in ranks if r.get("gate_retry")]
            if retried or (rep.rccl or {}).get("retry"):
                out["gate_retry"] = retried or ["oom"]
                out["rccl_peak_busbw_gbps"] = rep.rccl.get("min_peak_busbw_gbps")
        return out

    def cold_step(i: int) -> dict:
        """Fresh agents -> create -> readiness -> agents stop (every rank takes part)."""
        t0 = time.perf_counter()
        with span("bench.agents_start"):
            procs = start_agents(f"s{i}")
            urls = gather_urls(procs)
        t_agents = time.perf_counter()
        out = {"step": i, "agent_startup_ms": {p.name: getattr(p, "startup_ms", {}) for p in procs}}
        if rank == 0:
            out.update(create(i, urls))
        t_ready = time.perf_counter()
        if distributed:
            dist.barrier()  # the create is done before any rank stops its agents
        with span("bench.agents_stop"):
            for p in procs:  # every agent shuts down concurrently
                p.signal_stop()
            rcs = [p.stop() for p in procs]
        if any(rcs):
            raise RuntimeError(f"agent exit codes {rcs}")
        out["agent_stop_ms"] = {p.name: getattr(p, "stop_ms", None) for p in procs}
        # what each GPU node keeps for its next burn-in: the gate footprints it measured
        out["gate_footprints"] = {}
        for name, _ in mine:
            kept = os.path.join(last_root[name], AgentGateMixin.FOOTPRINT_FILE.lstrip("/"))
            if os.path.exists(kept):
                with open(kept, "r", encoding="utf-8") as fh:
                    out["gate_footprints"][name] = json.load(fh)
        out.update(agents_start_s=round(t_agents - t0, 4), create_to_ready_s=round(t_ready - t0, 4),
                   step_s=round(time.perf_counter() - t0, 4))
        return out

    def sync():
        if not args.sim_gpu:
            torch.cuda.synchronize()

    def barrier():
        if distributed:
            dist.barrier()
        sync()

    from triton_kubernetes_amd.ops import hbm

    # this node's GPUs of the run, by their DRM cards (a shared host lists other tenants' GPUs
    # too, whose releases must not hold up -- or end -- the wait): devices 0..N-1, or a
    # masked rank's own GPU.  Unmasked, local rank 0 watches them for every rank; masked,
    # every rank watches its own.
    settler = masked or local_rank == 0
    run_devices = [0] if masked else list(range(n_gpus))
    my_cards = [] if args.sim_gpu or not settler else hbm.cards_for_pci(
        (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        for p in (torch.cuda.get_device_properties(i) for i in run_devices))

    floor = [None]  # the node's clean used-HBM level (the first wait measures it)
    warm_floor = [None]  # the same with the warm creates' resident agents up

    def settle(resident: bool = False) -> dict:
        """Outside the timed region: the previous step's released HBM is cleared by the
        driver before the next step starts (a node entering service starts clean).  Every
        rank waits for the ranks that watch cards.

        ``resident``: agents stay up across the waits (the warm creates) and keep HBM of
        their own, so the clean level is above the cold one; the first such wait ends on a
        quiet window and its end level is the floor of the later ones."""
        got = {"waited_s": 0.0, "released_gib": 0.0, "cards": 0, "timed_out": False}
        if args.hbm_settle == "on" and my_cards:
            got = settle_cards(hbm, my_cards, warm_floor if resident else floor, resident,
                               timeout_s=budget.settle_cap_s)
        elif args.sim_gpu and settler and os.environ.get("TK_BENCH_SIM_SETTLE_S"):
            # CPU rehearsal of a slow driver clear (tests): the wait, capped as a real one is
            want = float(os.environ["TK_BENCH_SIM_SETTLE_S"])
            waited = want if budget.settle_cap_s is None else min(want, budget.settle_cap_s)
            time.sleep(waited)
            got = dict(got, waited_s=round(waited, 3), timed_out=waited < want)
        barrier()
        return got

    def replan(cold_left: int, settle_s: float, step_s: float, what: str = "", settle_cut: bool = False) -> None:
        """Rank 0 re-projects the run (RunBudget) and every rank takes its decision."""
        budget.record(settle_s, step_s, settle_cut)
        if rank == 0:
            budget.plan(cold_left, (args.warm_steps + 1) if args.warm_steps > 0 else 0)
            # one progress line per step on stderr (stdout carries only the result line)
            print(f"bench: {what} settle {settle_s:.1f} s, step {step_s:.2f} s, {cold_left} to go, "
                  f"projected {budget.projected_s} s of {budget.budget_s or 'no'} budget"
                  + (f", settle cap {budget.settle_cap_s} s" if budget.settle_cap_s is not None else ""),
                  file=sys.stderr, flush=True)
        if distributed:
            got = [(budget.warm_allowed, budget.settle_cap_s)]
            dist.broadcast_object_list(got, src=0)
            budget.warm_allowed, budget.settle_cap_s = got[0]

    comgr = {"dir": comgr_cache_dir(), "enabled": os.environ.get("AMD_COMGR_CACHE", "1") != "0",
             "mib_at_start": dir_mib(comgr_cache_dir()), "prewarm_s": None}
    if not args.sim_gpu and local_rank == 0 and comgr["enabled"] and comgr["mib_at_start"] < COMGR_WARM_MIB:
        # a fresh box: its first RCCL process takes ~5.5 s instead of ~1.8 s.  A node in
        # service has run its agent since boot; so does this one, untimed, whatever --warmup
        comgr["prewarm_s"] = prewarm_comgr()
    barrier()
    results = []
    settles = []
    try:
        for w in range(args.warmup):
            t_s = time.perf_counter()
            got = settle()
            barrier()
            t_step = time.perf_counter()
            cold_step(-1 - w)
            replan(args.warmup - w - 1 + args.steps, t_step - t_s, time.perf_counter() - t_step, f"warmup {w + 1}",
                   bool(got.get("timed_out")))
        TRACER.reset()
        comgr["mib_before_timed"] = dir_mib(comgr["dir"])
        # the timed region is the K steps, each bracketed by a barrier + synchronize on both
        # sides; the settle wait before each step is outside it (and reported as hbm_settle_s)
        elapsed = 0.0
        for i in range(args.steps):
            t_s = time.perf_counter()
            settles.append(settle())
            barrier()
            t_step = time.perf_counter()
            results.append(cold_step(i))
            barrier()
            took = time.perf_counter() - t_step
            elapsed += took
            replan(args.steps - i - 1, t_step - t_s, took, f"step {i + 1}", bool(settles[-1].get("timed_out")))
    except Exception as exc:
        if rank == 0:
            # a failed run still says what failed, in the line's own shape (value null), before
            # the traceback: the first run on a new node shape must leave a diagnosis
            print(json.dumps(failure_line(args, n_gpus, workers, gpus_per_worker, visible,
                                          f"{type(exc).__name__}: {exc}", len(results))), flush=True)
        raise
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    trace = TRACER.report()

    # secondary: warm creates against agents kept resident (outside the timed region)
    warm, warm_settles, warm_detail = [], [], []
    if args.warm_steps > 0 and budget.warm_allowed:
        procs = start_agents("warm")
        urls = gather_urls(procs)
        for i in range(args.warm_steps + 1):  # the first one warms the agents, untimed
            # as before a cold step: the previous create's burn-in released ~300 GB per GPU,
            # which the driver clears before a node takes its next cluster (untimed)
            warm_settles.append(settle(resident=True))
            barrier()
            t0 = time.perf_counter()
            if rank == 0:
                warm_detail.append(create(1000 + i, urls))
            if distributed:
                dist.barrier()
            if i:
                warm.append(time.perf_counter() - t0)
            if rank == 0:
                # untimed: destroy it again, which takes the resident hosts out of the cluster
                # (node/cleanup.py) -- a host is a node of one cluster at a time
                wf.delete_cluster(Context(settings=Settings(dict(ctx_base, cluster_name=f"bench-{1000 + i}"),
                                                            env={}), out=devnull), backend)
            if distributed:
                dist.barrier()
        for p in procs:
            p.signal_stop()
        for p in procs:
            p.stop()

    if rank == 0:
        ms = elapsed / max(1, args.steps) * 1000.0
        ready = [r["create_to_ready_s"] for r in results]
        phases = {}
        for sp in trace["spans"]:
            if sp["name"].startswith(("ready.", "module.", "direct.apply", "apply", "bench.")):
                phases.setdefault(sp["name"], []).append(sp["duration"])
        phase_ms = {k: round(sum(v) / max(1, args.steps) * 1000.0, 2) for k, v in sorted(phases.items())}
        node_steps = [r["gpu_node_step_ms"] for r in results if "gpu_node_step_ms" in r]
        for name in sorted({k for ns in node_steps for k in ns}):
            phase_ms[f"gpu_node.{name}"] = round(sum(ns.get(name, 0.0) for ns in node_steps) / len(node_steps), 2)
        gate = [r["rccl"] for r in results if "rccl" in r]
        for k in ("init_total", "init_wait", "sweep"):
            if gate:
                phase_ms[f"rccl.{k}_max_rank"] = round(sum(g[k] for g in gate) / len(gate), 2)
        sim = "SIM-GPU DRY RUN (not a measurement); " if args.sim_gpu else ""
        line = {
            "metric": METRIC,
            "value": round(sum(ready) / max(1, len(ready)), 4),
            "unit": "s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": False,
            "scaling": "weak",
            "vs_baseline": None,
            # a provisioning wall-clock: no tensor dtype, batch or sequence applies
            "dtype": "n/a",
            "data": sim + ("synthetic cold create: fresh node-agent processes per step; simulated phases "
                           "rke_provisioning (in-process Rancher v2.10 fake, RKE2 custom cluster, instantaneous "
                           "provisioning), runtime_install (firewall/hostname no-ops) and agent_container (the node "
                           "fetches system-agent-install.sh and registers as rancher-system-agent via the fake's "
                           "connect API instead of running it) and device_plugin_pod (the plugin DaemonSet is "
                           "scheduled by the fake's kubelet model and registers the node's GPUs instantly); "
                           "real on MI355X: "
                           f"native topology + RDMA labels, per-GPU HBM/MFMA/memtest burn-in level={args.burnin}, "
                           f"cluster RCCL all-reduce gate {'off' if args.no_rccl_gate else 'on'} "
                           f"(one communicator over all {n_gpus} GPUs"
                           + (", over the libtk_rccl ABI stub" if args.sim_gpu and not args.no_rccl_gate else "")
                           + ")"
                           + ("; before each timed step, untimed, the bench waits for the driver to clear the HBM "
                              "the previous step released (a node entering service starts clean)"
                              if args.hbm_settle == "on" and not args.sim_gpu else "")
                           + ("; the run budget capped %d of those waits (down to %.1f s), so a step may pay part "
                              "of its predecessor's clearing inside the timed region"
                              % (len(budget.caps_used), min(budget.caps_used)) if budget.caps_used else "")
                           + ("; the secondary warm creates were shed by the run budget"
                              if "warm_creates" in budget.shed else "")
                           + ("; opt-in node install before the timed region: verified single-target gfx950 "
                              "RCCL copy (ops/rccl_slim.py)" if slim_meta else "")),
            "config": {
                "model": "create cluster MI355X bare-metal N-worker + ROCm device-plugin + xGMI topology labels",
                "workers": workers, "gpus_per_worker": gpus_per_worker, "visible_gpus": visible,
                "control_plane_nodes": 2, "global_batch": "n/a", "seq_len": "n/a",
                "parallelism": f"{workers} worker node(s) x {gpus_per_worker} GPU(s)",
                "executor": "direct", "burnin": args.burnin, "rccl_gate": not args.no_rccl_gate,
                "gpu_health": args.gpu_health, "gpu_link_min_gbps": args.link_min_gbps,
                "start": ("cold (fresh agent processes per step)" if args.agents == "proc"
                          else "cold agents in the bench process (fresh NodeAgent objects per step)"),
                "rccl_gate_max_mib": args.rccl_mib,
                "simulated_phases": list(SIMULATED_PHASES),
                "rancher": versions.RANCHER_VERSION, "k8s_distribution": versions.DEFAULT_DISTRIBUTION,
                "k8s_version": versions.DEFAULT_K8S_VERSION,
                # HIP runtime + RCCL the GPU agents ran on (ops/native.py:select_runtime)
                "agent_hip_runtime": sorted(runtimes),
                # the kernel handle each GPU agent's RCCL device-code preload used ("none:none":
                # nothing preloaded; the gate's first init then loads the code)
                "agent_rccl_preload": sorted(preloads),
                # node install step outside the timed region (ops/rccl_slim.py)
                "rccl_slim": ({k: slim_meta.get(k) for k in ("prepare_s", "cached", "source_fatbin_bytes",
                                                              "loaded_code_object_bytes", "verified")}
                              if slim_meta else None),
                # node state the timed steps find, as a node does after its first GPU process: the
                # HIP code-object cache the warmup's RCCL init filled (a fresh box's first init
                # pays ~5.5 s instead of ~1.8 s, once)
                "comgr_cache": comgr,
            },
            "create_to_ready_s": ready,
            "agents_start_s_mean": round(sum(r["agents_start_s"] for r in results) / max(1, len(results)), 4),
            # the GPU agents' shutdown (ms_per_step - value), by stage: max over agents, mean over steps
            "gpu_agent_stop_ms": _stop_phases(results),
            "warm_create_to_ready_s": round(sum(warm) / len(warm), 4) if warm else None,
            "warm_create_to_ready_each_s": [round(w, 4) for w in warm],
            "warm_hbm_settle_s": [round(w["waited_s"], 3) for w in warm_settles],
            "warm_gpu_burnin_ms": [d.get("gpu_node_step_ms", {}).get("gpu_burnin") for d in warm_detail[1:]],
            "warm_rccl_init_ms": [(d.get("rccl") or {}).get("init_total") for d in warm_detail[1:]],
            # GPU nodes that joined with the health taint in any timed step (normally none)
            "gpu_unhealthy_nodes": sorted({h for r in results for h in r.get("gpu_unhealthy", [])}),
            # the gate communicator's device memory per GPU (MiB, max over agents, last timed step):
            # what the burn-in span's headroom must leave (node/agent_gate.py:span_headroom).
            # footprint_kind 1: the agent's own VRAM; 2: the device's used-memory delta, which
            # in a cold step also counts the burn-in child allocating its span meanwhile: then
            # footprint_kept is 0 and the node did not take it as a footprint
            "rccl_footprint_mib": next(({k: r["rccl"].get(k) for k in ("footprint_mib", "footprint_total_mib",
                                                                       "footprint_kind", "footprint_kept")}
                                        for r in reversed(results) if r.get("rccl")), None),
            # timed steps whose gate init ran out of HBM and was retried after the spans' release
            "gate_retry_steps": [r["step"] for r in results if r.get("gate_retry")],
            # what the GPU nodes keep for their next burn-in's headroom after the last timed step
            # (/etc/triton-kubernetes/gate-footprint.json, carried from step to step as on a node)
            "node_gate_footprints": results[-1].get("gate_footprints") if results else None,
            # ranks of the cluster RCCL gate per timed step (every GPU of the worker tier)
            "rccl_gate_ranks": [r.get("rccl_gate_ranks", 0) for r in results],
            # the GPU nodes' measured xGMI peer-read matrix (2+ GPUs per node), last timed step
            "xgmi_links": next((r["xgmi_links"] for r in reversed(results) if r.get("xgmi_links")), None),
            # the GPU node's burn-in step, per timed step (max over worker nodes), and its screens
            "gpu_burnin_ms": [r.get("gpu_node_step_ms", {}).get("gpu_burnin") for r in results],
            "burnin_phase_ms": [r.get("burnin_phase_ms") for r in results],
            # before each timed step, outside the timed region: the wait for the driver to clear
            # the previous step's released HBM (ops/hbm.py; --hbm-settle off for the A/B)
            "hbm_settle": args.hbm_settle,
            "hbm_settle_cards": my_cards,
            "hbm_settle_s": [s["waited_s"] for s in settles],
            "hbm_settle_released_gib": [s["released_gib"] for s in settles],
            "hbm_settle_reached_floor": [s.get("reached_floor") for s in settles],
            # the run's wall-clock guard (RunBudget): what it projected and what it shed to
            # stay inside --time-budget (never a timed step)
            "run_budget": budget.report(),
            "phase_ms_per_step": phase_ms,
        }
        print(json.dumps(line), flush=True)
        if args.report:
            with open(args.report, "w", encoding="utf-8") as fh:
                json.dump({"line": line, "steps": results, "warm_s": warm, "warm_steps": warm_detail, "warm_settles": warm_settles, "trace": trace}, fh, indent=1,
                          default=str)
    devnull.close()
    if fake is not None:
        fake.stop()
    shutil.rmtree(work, ignore_errors=True)  # the run's manager state, agent roots and node files
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
