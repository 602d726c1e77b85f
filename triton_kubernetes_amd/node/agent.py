"""Node agent: executes bootstrap plans on a host, in-process.

``tk-node-agent`` is the pull-side alternative to SSH delivery: it runs on a
host (a systemd unit on real nodes; a fresh process per simulated node and step in
``bench.py``; an in-process object in tests) and executes :class:`~.plan.BootstrapPlan`
steps natively.

Security model (``node/security.py``): the agent never executes shell text it
receives.  A plan's ``shell`` fields are only for the SSH renderer; the agent
dispatches on the step ``action`` and runs fixed, agent-side argv lists built from
*validated* parameters (hostname, image reference, registry, Rancher URL).  Off loopback it
serves only TLS, with a certificate for the node's address signed by its cluster
manager's CA; plain HTTP needs ``--insecure-local`` and binds loopback only.  Every
request must carry the node's own token (``X-TK-Agent-Token``, derived per node
from the manager secret; a random one when none is given).  A plan whose agent
step names an image (RKE1) or a Rancher server (RKE2) outside the node's allow-list
(:class:`AgentPolicy`, set by the manager at enrollment) is refused before any step
runs (HTTP 403).

Modes:

* ``exec`` — runtime steps run the fixed commands (RKE1: the container runtime must
  already be installed; installing it is the SSH path's job); the ``agent`` step runs
  ``docker run rancher/rancher-agent`` (RKE1) or the allowed server's
  ``system-agent-install.sh`` (RKE2);
* ``sim`` — runtime steps are recorded as no-ops (simulated hosts have no
  container runtime) and the ``agent`` step registers with Rancher through
  ``POST /v3/connect/register`` (``X-Cattle-Agent-Kind: system-agent`` for RKE2,
  after fetching the installer as a real node does) instead.

In both modes the MI355X steps call the native probes directly on the agent's
GPUs: topology labeller (N1), HBM/MFMA/memtest burn-in, RCCL env file and the
node-level RCCL sweep (N2).

HTTP API (JSON): ``GET /v1/info``, ``GET /v1/health`` (GPU RAS verdict, ``node/health.py``), ``GET /metrics``
(Prometheus text: GPU RAS / PCIe now, the last bring-up's steps and measurements; ``node/metrics.py``), ``POST /v1/plan``, ``POST /v1/rccl-uid``,
``POST /v1/rccl-prepare`` (without a ``uid``: host the rendezvous and return it; start this node's ranks of the cluster-wide RCCL
communicator, non-blocking), ``POST /v1/rccl-gate`` (run them: verified
all-reduce sweep), ``POST /v1/rccl-abort``, ``POST /v1/cleanup``, ``POST /v1/shutdown``
(the daemon stops and exits).

Layout, by concern:

==================  =====================================================================
``agent.py``        :class:`NodeAgent` (policy check, plan runner, warm start, stop), ``main``
``agent_steps.py``  what each plan action does on the host (validated fixed argv, GPU steps)
``agent_gate.py``   this node's ranks of cluster RCCL gates
``agent_http.py``   the HTTP(S) API and its authentication
==================  =====================================================================
"""

import concurrent.futures as cf
import json
import os
import secrets
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..utils import procstat
from ..utils.trace import span
from .agent_gate import AgentGateMixin
from .agent_http import AgentHTTPMixin
from .agent_steps import AgentStepsMixin, StepFailed, StepResult
from .plan import BootstrapPlan
from .security import AgentPolicy, is_loopback

MODES = ("sim", "exec")


@dataclass
class NodeAgent(AgentStepsMixin, AgentGateMixin, AgentHTTPMixin):
    HISTORY_KEEP = 32  # plan results kept (history[-1] feeds /metrics); a daemon runs many
    name: str = "node"
    mode: str = "sim"
    devices: List[int] = field(default_factory=list)
    root: str = "/"
    token: str = ""
    topology_override: Optional[Dict[str, Any]] = None
    burnin_override: Optional[Callable[[int, str], Dict[str, Any]]] = None
    # the Rancher agent images / servers this node may run (default: the pinned agent
    # image; Rancher servers on loopback only)
    policy: Optional[AgentPolicy] = None
    # cluster RCCL gate: "auto" = RCCL on real GPUs, a simulated gate on synthetic ones;
    # "rccl" = the RCCL ABI even on synthetic GPUs (a dry run with TK_RCCL_LIB naming the
    # ABI stub, ops/csrc/tk_rccl_stub.cpp)
    gate_backend: str = field(default_factory=lambda: os.environ.get("TK_GATE_BACKEND", "auto"))

    def __post_init__(self):
        if self.mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}")
        if not self.token:
            self.token = secrets.token_urlsafe(24)
        if self.policy is None:
            from ..versions import AGENT_IMAGE

            self.policy = AgentPolicy([AGENT_IMAGE], loopback_servers=True)
        self.lock = threading.Lock()
        self._gate_mu = threading.Lock()
        self._stopped = False  # stop(): refuse requests on connections still open
        # long-lived workers for topology prefetch and per-GPU burn-in: no thread is created
        # on the bring-up path (thread creation contends with RCCL/HIP work in the process)
        self._pool = cf.ThreadPoolExecutor(max_workers=len(self.devices) + 2,
                                           thread_name_prefix=f"tk-agent-{self.name}")
        # uid -> (gate, created, {"world", "rank_base", "sizes"})
        self._gates: Dict[bytes, Any] = {}
        # uid -> (SweepResult, finished): whole-node gates the rccl_local step already swept
        self._gate_results: Dict[bytes, Any] = {}
        # uid -> gate whose sweep is running (waiting for peers): /v1/rccl-abort cancels it
        self._sweeping: Dict[bytes, Any] = {}
        # uid -> when /v1/rccl-abort named it: a later prepare/gate for it fails at once
        self._aborted_uids: Dict[bytes, float] = {}
        # one RCCL unique id kept ready (new_uid): the gate's first request gets it without
        # an ncclGetUniqueId on the bring-up path; the pool makes the next one afterwards
        self._spare_uid: Optional[bytes] = None
        self._uid_mu = threading.Lock()
        self.last_labels: Dict[str, str] = {}
        # the health limits of the last gpu_health step (what /metrics judges by)
        self.health_limits: Tuple[int, int] = (0, -1)
        self.history: List[Dict[str, Any]] = []
        self._server: Optional[Any] = None  # the HTTP(S) server (agent_http.py)
        self.shutdown_requested = threading.Event()

    # --- files ---------------------------------------------------------------------------
    def path(self, p: str) -> str:
        return os.path.join(self.root, p.lstrip("/")) if self.root not in ("", "/") else p

    def write_file(self, p: str, data: str) -> str:
        full = self.path(p)
        os.makedirs(os.path.dirname(full), exist_ok=True)
        with open(full, "w", encoding="utf-8") as fh:
            fh.write(data)
        return full

    # --- plan execution ---------------------------------------------------------------------
    def refusals(self, plan: BootstrapPlan) -> List[str]:
        """Why this node refuses ``plan``: an agent step for a distribution the node was not
        enrolled for, or whose Rancher server (either distribution: RKE2 runs its installer,
        RKE1 hands it to a privileged ``rancher-agent``) or image (RKE1) is outside the
        node's allow-list; an ``rccl_env`` step with a setting the node's RCCL environment
        may not hold (one naming a library, plugin or path, or a value that is not plain
        tokens: ``parallel/rccl_env.py:env_problems``); a ``gpu_metrics`` step whose
        directory is not an absolute path free of ``..``."""
        from ..parallel.rccl_env import env_problems

        out = []
        for s in plan.steps:
            if s.action == "rccl_env":
                # the file this step writes is loaded as root by the agent's service
                out.extend(env_problems(s.params.get("env", {}) or {}))
                continue
            if s.action == "gpu_metrics":
                # the agent writes the textfile as root: an absolute directory, no "..",
                # as the config check requires (node/metrics.py:textfile_dir_of)
                from ..errors import ConfigError
                from .metrics import textfile_dir_of

                try:
                    if not textfile_dir_of({"gpu_metrics_textfile": s.params.get("dir")}):
                        out.append("gpu_metrics step without a directory")
                except ConfigError as exc:
                    out.append(str(exc))
                continue
            if s.action != "agent":
                continue
            dist = str(s.params.get("distribution", plan.distribution))
            if not self.policy.allows_distribution(dist):
                out.append(f"distribution {dist!r} is not the one this node was enrolled for "
                           f"({', '.join(self.policy.distributions)})")
                continue
            server = str(s.params.get("server") or plan.rancher_url)
            if not self.policy.allows_server(server) or server != plan.rancher_url:
                out.append(f"Rancher server {server!r} is not in this node's allow-list")
            if dist != "rke2" and not self.policy.allows(str(s.params.get("image", ""))):
                out.append(f"image {str(s.params.get('image', ''))!r} is not in this node's allow-list")
        return out

    def run_plan(self, plan: BootstrapPlan) -> Dict[str, Any]:
        bad = self.refusals(plan)
        if bad:
            raise PermissionError(bad[0])
        results: List[StepResult] = []
        ctx: Dict[str, Any] = {"labels": {}, "capacity": {}, "taints": []}
        t_plan = time.perf_counter()
        self._touch()
        error = None
        if any(s.action == "gpu_labels" for s in plan.steps):
            # topology discovery (host-side sysfs reads) overlaps the preflight
            # and burn-in kernels instead of running after them
            ctx["topology_future"] = self._pool.submit(self._topology)
        with self.lock:
            # the burn-in children keep the HBM they tested until this plan's link matrix is
            # measured too: the driver's clearing of their release would run beside it
            self._links_pending = any(s.action == "gpu_links" for s in plan.steps)
            try:
                for step in plan.steps:
                    t0 = time.perf_counter()
                    try:
                        with span(f"node.{step.action}", node=plan.hostname):
                            detail = self._run_step(plan, step, ctx)
                        results.append(StepResult(step.name, True, (time.perf_counter() - t0) * 1e3, detail))
                    except Exception as exc:  # noqa: BLE001 - reported to the executor
                        results.append(StepResult(step.name, False, (time.perf_counter() - t0) * 1e3, str(exc)))
                        error = f"{step.name}: {exc}"
                        break
                    finally:
                        if step.action == "gpu_links":
                            self._links_pending = False
            finally:
                self._links_pending = False
        doc = {"hostname": plan.hostname, "ok": error is None, "error": error,
               "ms": (time.perf_counter() - t_plan) * 1e3,
               "steps": [r.__dict__ for r in results], "labels": ctx["labels"], "capacity": ctx["capacity"],
               "taints": ctx["taints"]}
        self.history.append(doc)
        del self.history[:-self.HISTORY_KEEP]  # a daemon's record of its last plans, not all
        self._touch()
        return doc

    def health(self, max_uncorrectable: int = 0, max_bad_pages: int = -1) -> Dict[str, Any]:
        """This node's GPU health verdict now (``GET /v1/health``; node/health.py)."""
        from .health import evaluate

        verdict = evaluate(self._topology(), max_uncorrectable, max_bad_pages)
        verdict["node"] = self.name
        return verdict

    def metrics(self) -> str:
        """``GET /metrics``: Prometheus text of the node (node/metrics.py)."""
        from .metrics import bringup_metrics, gpu_metrics

        gpu_text, ok = "", None
        if self.devices or self.topology_override is not None:
            try:  # a failed GPU read costs the GPU families of this scrape, not the endpoint
                gpu_text, ok = gpu_metrics(self.health(*self.health_limits), self.name), True
            except Exception:  # noqa: BLE001
                ok = False
        return bringup_metrics(self.history[-1] if self.history else None, self.name, self.mode, ok,
                               self.last_labels) + gpu_text

    # --- native warm start ------------------------------------------------------------------------
    def warm_native(self) -> None:
        """Load the native libraries (and everything they pull in) once, up front.

        A dlopen issued while a gate's communicator init is running on another thread can
        deadlock against the HIP runtime (dlopen holds the loader lock; the init thread holds
        runtime locks and needs the loader lock) — observed under rocprofv3.  Loading them here,
        before any request is served, keeps dlopen off the bring-up path."""
        # one fd-table resize now instead of RCU-synchronized resizes on the bring-up path
        slots = int(os.environ.get("TK_FD_TABLE", "16384") or 0)
        if slots > 0:
            procstat.presize_fd_table(slots)
        t0 = time.perf_counter()
        self.startup_ms: Dict[str, float] = {}
        if self.topology_override is not None or not self.devices:
            return
        from ..ops import probe, rccl, topo

        # RCCL reads its settings once per process, the bootstrap interface at the first
        # unique id (made below): the node's RCCL environment goes in first
        self.rccl_env_applied = self.apply_node_rccl_env() if os.environ.get("TK_AGENT_RCCL_ENV", "1") != "0" else {}
        if getattr(self, "rccl_env_skipped", None):
            print(f"tk-node-agent: /etc/rccl/rccl.env settings not applied (they name a library, plugin or "
                  f"path, or hold more than plain tokens): {', '.join(self.rccl_env_skipped)}", file=sys.stderr)
        probe._lib()
        rccl._lib()
        self.startup_ms["dlopen"] = round((time.perf_counter() - t0) * 1e3, 1)
        # 1 (default): right after dlopen; after-uid: once the unique id is made; 0: off
        # (profiles/round5/rccl_preload_ab.jsonl: the gate's init 1.81 -> 1.73 s)
        preload = os.environ.get("TK_RCCL_PRELOAD", "1")
        if preload == "1":
            # RCCL's device code starts loading now, beside the rest of the start-up, not
            # after the cluster gate's first request (tkr_preload_device_code)
            self.startup_ms["rccl_preload_started"] = float(rccl.preload_device_code(self.devices))
            self.rccl_preload = rccl.preload_report()
        # the full burn-in's ~300 GB memtest memory is released off the bring-up path
        probe.set_async_free(True)
        # ... and the full memtest's ~300 GB is held and released by a gpu-burnin child, so no
        # hipFree of it blocks this process's other HIP calls (ops/probe.py:memtest_span_process)
        probe.set_span_process(os.environ.get("TK_SPAN_PROCESS", "1") != "0")
        # the whole burn-in of a GPU runs in a gpu-burnin child: beside this process's RCCL
        # communicator start, whose code-object loading held up the screens' launches here
        # (ops/probe.py:_burnin_child)
        burnin_child = os.environ.get("TK_BURNIN_PROCESS", "1") != "0"
        probe.set_burnin_process(burnin_child)
        # the gate's communicator over this node's GPUs allocates while the span is held
        # (the constant floor, or what this node's gates measured: node/agent_gate.py)
        probe.set_span_headroom(self.span_headroom(len(self.devices)))
        # ...and releases the HBM it tested only once this agent's RCCL communicator inits
        # are through: the driver's clearing of that release held their device-code load up
        if os.environ.get("TK_BURNIN_RELEASE_HOLD", "1") != "0":
            probe.set_release_hold(self._await_rccl_inits)
        # burn-in arena (in-process burn-ins only): resident for the agent's lifetime,
        # released after an idle period
        if os.environ.get("TK_PROBE_SCRATCH_CACHE", "0" if burnin_child else "1") != "0":
            level = os.environ.get("TK_PROBE_SCRATCH_LEVEL", "quick")
            t1 = time.perf_counter()
            list(self._pool.map(lambda d: probe.prealloc_scratch(d, level), self.devices))
            self.startup_ms["hip_init_arena"] = round((time.perf_counter() - t1) * 1e3, 1)
            idle_s = float(os.environ.get("TK_PROBE_SCRATCH_IDLE_S", "300") or 0)
            if idle_s > 0:
                self._start_janitor(idle_s)
        quiet = float(os.environ.get("TK_TEARDOWN_QUIET_MS", "0") or 0)
        if quiet > 0:
            rccl.set_teardown_quiet_ms(quiet)
        t2 = time.perf_counter()
        self._refill_uid()  # the first gate's unique id, ready before any request
        self.startup_ms["uid"] = round((time.perf_counter() - t2) * 1e3, 1)
        if preload == "after-uid":  # the same, once RCCL's bootstrap has made the unique id
            self.startup_ms["rccl_preload_started"] = float(rccl.preload_device_code(self.devices))
            self.rccl_preload = rccl.preload_report()
        try:
            topo.native_topology("sysfs", "/nonexistent")  # loads libtk_topo.so
        except Exception:  # noqa: BLE001 - topology falls back to other sources later
            pass

    # RCCL settings the gate's communicators need from the node's environment: RCCL reads
    # them once per process, so they must be in place before the agent's first RCCL call.
    # HSA_* (the ROCm runtime's, e.g. fine-grained PCIe memory for RDMA) are read once at
    # HIP's initialisation: they are applied at agent start only
    RCCL_ENV_PREFIXES = ("NCCL_", "RCCL_")
    STARTUP_ENV_PREFIXES = RCCL_ENV_PREFIXES + ("HSA_",)

    def apply_node_rccl_env(self) -> Dict[str, str]:
        """Put the node's RCCL settings into this process's environment, for the agent's own
        communicators (the cluster gate): ``/etc/rccl/rccl.env`` as the last bring-up wrote it
        (the systemd unit loads the same file, ``EnvironmentFile=``; this covers agents started
        another way).  Keys the process environment already sets win.  Without the file RCCL
        detects the node's RDMA ports itself, which is what the discovered settings would say
        (every active port; RoCE v2 GIDs) -- measured: with them set, a cold create->ready on
        MI355X was 0.07 and 0.25 s slower in two A/B pairs (``profiles/round4/rccl_env_ab.txt``).  Returns
        what was applied.  Called before the agent's first HIP or RCCL call (``warm_native``).
        A setting the file may not hold (``parallel/rccl_env.py:env_problems``: one naming a
        library, plugin or path; written by hand or by an older release) is skipped and listed
        in ``rccl_env_skipped``."""
        from ..parallel.rccl_env import env_problems, parse_env_file

        self.rccl_env_skipped = []
        try:
            with open(self.path("/etc/rccl/rccl.env"), "r", encoding="utf-8", errors="replace") as fh:
                env = parse_env_file(fh.read())
        except OSError:
            return {}
        applied = {}
        for k, v in env.items():
            if not k.startswith(self.STARTUP_ENV_PREFIXES) or k in os.environ:
                continue
            if env_problems({k: v}):
                self.rccl_env_skipped.append(k)
                continue
            os.environ[k] = v
            applied[k] = v
        return applied

    def _start_janitor(self, idle_s: float) -> None:
        """One long-lived thread frees the burn-in arena once no plan has run for ``idle_s``
        (the next burn-in re-allocates it)."""
        if getattr(self, "_janitor", None) is not None:
            return
        self._idle_cv = threading.Condition()
        self._last_active = time.monotonic()
        self._stopping = False

        def loop():
            from ..ops import probe

            held = True
            with self._idle_cv:
                while not self._stopping:
                    if not held:
                        self._idle_cv.wait()  # until a plan runs (its burn-in re-allocates) or stop
                        held = True
                        continue
                    left = self._last_active + idle_s - time.monotonic()
                    if left <= 0:
                        probe.release_scratch()
                        held = False
                    else:
                        self._idle_cv.wait(timeout=left)
            probe.release_scratch()
            probe.set_scratch_cache(False)

        self._janitor = threading.Thread(target=loop, name=f"tk-agent-{self.name}-janitor", daemon=True)
        self._janitor.start()

    def _touch(self) -> None:
        cv = getattr(self, "_idle_cv", None)
        if cv is not None:
            with cv:
                self._last_active = time.monotonic()
                cv.notify()

    def stop(self, drain_rccl: bool = True) -> None:
        """Shut the agent down.  ``drain_rccl`` False: the caller leaves the process at once
        (``main``'s quick exit), so the communicators' teardown is not waited for -- it only
        frees device memory the kernel reclaims from an exiting process anyway, and its
        frees queue behind the driver's wipe of a burn-in's release (~0.6 s per create)."""
        self._stopped = True
        t = time.perf_counter()
        ms: Dict[str, float] = {}

        def lap(name: str) -> None:
            nonlocal t
            now = time.perf_counter()
            ms[name] = round((now - t) * 1e3, 1)
            t = now

        cv = getattr(self, "_idle_cv", None)
        if cv is not None:
            with cv:
                self._stopping = True
                cv.notify()
            self._janitor.join(timeout=30)
            self._janitor = None
        lap("janitor")
        self._pool.shutdown(wait=True)
        lap("pool")
        if self._server is not None:
            self._server.shutdown()
            self._server.server_close()
            self._server = None
        lap("server")
        with self._gate_mu:
            pending = [e[0] for e in self._gates.values()]
            self._gates.clear()
            self._gate_results.clear()
        for g in pending:
            g.abort()
        if getattr(self, "_used_rccl", False) and drain_rccl:
            from ..ops import rccl

            rccl.drain()
        lap("rccl_drain")
        if self.devices and self.topology_override is None:
            from ..ops import rccl

            deadline = time.monotonic() + 60.0  # a device-code preload still running: let it end
            while rccl.preloads_running() > 0 and time.monotonic() < deadline:
                time.sleep(0.01)
        lap("preloads")
        if self.devices and self.topology_override is None and self.burnin_override is None:
            from ..ops import probe

            # this process's own releases; a burn-in child still releasing what it tested
            # finishes on its own (its stdin closes with this process: no hold outlives it)
            probe.wait_frees(children=False)
        lap("frees")
        self.stop_ms = ms  # where a shutdown's time went (logged by main)

def _listen_arg(text: str) -> str:
    """``HOST:PORT`` with a port of 0..65535 (0: any free port)."""
    import argparse

    host, sep, port = text.rpartition(":")
    if not sep or not port.isdigit() or not 0 <= int(port) <= 65535 or not host:
        raise argparse.ArgumentTypeError(f"HOST:PORT with a port of 0..65535, not {text!r}")
    return text


def _devices_arg(text: str) -> List[int]:
    """Comma-separated local GPU indices, each once ("" = none)."""
    import argparse

    parts = [d.strip() for d in text.split(",") if d.strip()]
    if not all(d.isdigit() for d in parts):
        raise argparse.ArgumentTypeError(f"comma-separated GPU indices (0, 1, ...), not {text!r}")
    devices = [int(d) for d in parts]
    if len(set(devices)) != len(devices):
        raise argparse.ArgumentTypeError(f"a GPU index given twice: {text!r}")
    return devices


def _count_arg(text: str) -> int:
    import argparse

    if not text.strip().isdigit():
        raise argparse.ArgumentTypeError(f"a whole number >= 0, not {text!r}")
    return int(text)


def main(argv: Optional[List[str]] = None) -> int:
    """``tk-node-agent``: serve the agent API on a host (127.0.0.1 by default).  A command
    line it cannot use (a bad listen address, GPU list, credential directory or token file)
    is an argparse error (exit 2), not a traceback from deep inside the start-up."""
    import argparse

    t_main = time.perf_counter()
    ap = argparse.ArgumentParser(prog="tk-node-agent")
    ap.add_argument("--listen", default="127.0.0.1:7946", type=_listen_arg)
    ap.add_argument("--mode", default="exec", choices=MODES)
    ap.add_argument("--devices", default=[], type=_devices_arg, help="comma-separated local GPU indices")
    ap.add_argument("--credentials", default="",
                    help="the node's credential directory (agent-token, agent.crt/.key, agent-policy.json; "
                         "`triton-kubernetes credentials node`): serve TLS with the node's token and allow-list")
    ap.add_argument("--insecure-local", action="store_true",
                    help="plain HTTP on a loopback address (development, single-box tests)")
    ap.add_argument("--token-file", default="", help="file holding the token (with --insecure-local)")
    ap.add_argument("--allow-server", action="append", default=[],
                    help="with --insecure-local: a Rancher server URL whose RKE2 installer the node may run "
                         "(besides loopback ones); repeatable")
    ap.add_argument("--root", default="/")
    ap.add_argument("--name", default="", help="agent name (defaults to the listen host)")
    ap.add_argument("--synthetic-gpus", type=_count_arg, default=0,
                    help="tests / CPU dry runs only: a synthetic MI355X topology with this many GPUs, "
                         "no burn-in kernels, no RCCL")
    args = ap.parse_args(argv)
    token = ""
    ssl_ctx = None
    policy = None
    host, _, port = args.listen.rpartition(":")
    if args.credentials:
        from .security import read_credentials

        try:
            creds = read_credentials(args.credentials)
        except (OSError, ValueError) as exc:  # ssl.SSLError is an OSError
            ap.error(f"--credentials {args.credentials}: {exc}")
        token, ssl_ctx, policy = creds["token"], creds["ssl_context"], creds["policy"]
    elif not args.insecure_local:
        ap.error("--credentials DIR is required (or --insecure-local for plain HTTP on loopback)")
    elif not is_loopback(host):
        ap.error(f"--insecure-local serves plain HTTP on loopback only, not {host}")
    else:
        from ..versions import AGENT_IMAGE

        policy = AgentPolicy([AGENT_IMAGE], servers=list(args.allow_server), loopback_servers=True)
    if args.token_file and not token:
        try:
            with open(args.token_file, "r", encoding="utf-8") as fh:
                token = fh.read().strip()
        except (OSError, UnicodeDecodeError) as exc:
            ap.error(f"--token-file {args.token_file}: {exc}")
    devices = args.devices
    agent = NodeAgent(name=args.name or host, mode=args.mode, devices=devices, root=args.root, token=token,
                      policy=policy)
    if args.synthetic_gpus > 0:
        from .labels import synthetic_topology

        agent.topology_override = synthetic_topology(args.synthetic_gpus)
        agent.burnin_override = lambda dev, level: {"ok": True, "simulated": True, "level": level}

    import signal
    import sys

    # SIGTERM / SIGINT / POST /v1/shutdown all take the same path: stop() (gates aborted,
    # communicator teardowns drained, arena released), then a prompt exit
    signal.signal(signal.SIGTERM, lambda *_: agent.shutdown_requested.set())
    signal.signal(signal.SIGINT, lambda *_: agent.shutdown_requested.set())
    url = agent.serve(host or "127.0.0.1", int(port), ssl_context=ssl_ctx)
    import gc

    gc.collect()
    gc.freeze()  # long-lived daemon: keep startup objects out of every later collection
    from ..ops import native

    print(json.dumps({"listening": url, "token_from_file": bool(token), "tls": ssl_ctx is not None,
                      "hip_runtime": native._runtime_dir or "not loaded",
                      # the kernel handle RCCL's device-code preload used, or "none" (a librccl
                      # exporting no device kernel: the gate's first init then loads it)
                      "rccl_preload": getattr(agent, "rccl_preload", {"symbol": "none", "how": "none"}),
                      "startup_ms": dict(getattr(agent, "startup_ms", {}),
                                         main_to_serve=round((time.perf_counter() - t_main) * 1e3, 1))}),
          flush=True)
    while not agent.shutdown_requested.wait(3600):
        pass
    t0 = time.perf_counter()
    quick_exit = bool(agent.devices) and not _profiled() and os.environ.get("TK_AGENT_EXIT", "quick") != "normal"
    agent.stop(drain_rccl=not quick_exit or os.environ.get("TK_AGENT_STOP_DRAIN") == "1")
    print(json.dumps({"stopped": True, "stop_ms": round((time.perf_counter() - t0) * 1e3, 1),
                      "stop_phases_ms": getattr(agent, "stop_ms", {})}), flush=True)
    sys.stdout.flush()
    sys.stderr.flush()
    if getattr(agent, "_used_rccl", False):
        from ..ops import rccl

        # every communicator was torn down by stop(); only an init still blocked on absent
        # peers would hang a normal exit (which also lets tools such as rocprofv3 finalize)
        if rccl.abandoned_inits():
            rccl.exit_now(0)
    if quick_exit:
        # what a normal exit would add is the HIP runtime's own teardown (and, undrained, the
        # communicators'), which the kernel does for an exiting process anyway (gpu-burnin's
        # took 2.6 s behind the driver's VRAM wipe)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    return 0


def _profiled() -> bool:
    """A profiler's preloaded tool finalises in the normal exit path: keep it then."""
    return "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ)


__all__ = ["NodeAgent", "StepFailed", "StepResult", "MODES", "main"]


if __name__ == "__main__":
    import sys

    sys.exit(main())

