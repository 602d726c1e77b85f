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
"""

import base64
import concurrent.futures as cf
import hashlib
import hmac
import http.server
import json
import socket
import os
import re
import secrets
import shutil
import ssl
import subprocess
import tempfile
import threading
import time
import urllib.parse
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..cloud.http import HTTPClient
from ..parallel.rccl_env import render_env_file, site_env_from_topology
from ..rancher.fake import tunnel_params
from ..utils import procstat
from ..utils.httpserver import Server as HTTPServer
from ..utils.trace import span
from .labels import burnin_labels, labels_from_topology, link_labels
from .plan import BootstrapPlan, Step
from .security import AgentPolicy, is_loopback, metrics_token

MODES = ("sim", "exec")
_HOSTNAME_RE = re.compile(r"^[a-z0-9]([-a-z0-9]{0,61}[a-z0-9])?(\.[a-z0-9]([-a-z0-9]{0,61}[a-z0-9])?)*$")
_IMAGE_RE = re.compile(r"^[A-Za-z0-9][A-Za-z0-9._/:@-]{0,254}$")
_TOKEN_RE = re.compile(r"^[A-Za-z0-9._:-]{1,512}$")
_URL_RE = re.compile(r"^https?://[A-Za-z0-9._:\[\]-]+(/[A-Za-z0-9._/-]*)?$")
_ROLES = ("worker", "etcd", "controlplane")


def _ca_args(plan: BootstrapPlan) -> List[str]:
    """``--ca-checksum`` for the agent; none when the server's certificate is publicly
    trusted (Rancher reports no CA and no checksum then)."""
    if not plan.ca_checksum:
        return []
    return ["--ca-checksum", _check(_TOKEN_RE, plan.ca_checksum, "ca checksum")]


_TAINT_RE = re.compile(r"^[A-Za-z0-9./-]{1,253}=[A-Za-z0-9._-]{0,63}:(NoSchedule|PreferNoSchedule|NoExecute)$")


def _taint_args(taints: Optional[List[Dict[str, str]]]) -> List[str]:
    """``--taints key=value:Effect`` per taint (both Rancher agents take the flag)."""
    out: List[str] = []
    for t in taints or []:
        out += ["--taints", _check(_TAINT_RE, f"{t['key']}={t.get('value', '')}:{t['effect']}", "taint")]
    return out


class StepFailed(RuntimeError):
    def __init__(self, step: str, message: str):
        super().__init__(f"step {step} failed: {message}")
        self.step = step


@dataclass
class StepResult:
    name: str
    ok: bool
    ms: float
    detail: Any = None


def _check(pattern: re.Pattern, value: str, what: str) -> str:
    if not isinstance(value, str) or not pattern.match(value):
        raise ValueError(f"invalid {what}: {value!r}")
    return value


class _SimGate:
    """Stand-in for ops.rccl.GateComm on agents with synthetic GPUs (no RCCL)."""

    def __init__(self, devices: List[int]):
        self.devices = list(devices)

    def sweep(self, sizes, iters=10, warmup=3, dtype="f32", timeout_s=600.0, async_teardown=True):
        from ..ops.rccl import SweepResult

        n = len(sizes)
        return SweepResult(len(self.devices), dtype, list(sizes), [0.0] * n, [0.0] * n, [0.0] * n, [0] * n, 0.0,
                           {"simulated": 1.0})

    def abort(self) -> None:
        pass

    def cancel(self) -> None:
        pass


@dataclass
class NodeAgent:
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
        # one RCCL unique id kept ready (new_uid): the gate's first request gets it without
        # an ncclGetUniqueId on the bring-up path; the pool makes the next one afterwards
        self._spare_uid: Optional[bytes] = None
        self._uid_mu = threading.Lock()
        self.last_labels: Dict[str, str] = {}
        # the health limits of the last gpu_health step (what /metrics judges by)
        self.health_limits: Tuple[int, int] = (0, -1)
        self.history: List[Dict[str, Any]] = []
        self._server: Optional[http.server.ThreadingHTTPServer] = None
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
        node's allow-list."""
        out = []
        for s in plan.steps:
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
        doc = {"hostname": plan.hostname, "ok": error is None, "error": error,
               "ms": (time.perf_counter() - t_plan) * 1e3,
               "steps": [r.__dict__ for r in results], "labels": ctx["labels"], "capacity": ctx["capacity"],
               "taints": ctx["taints"]}
        self.history.append(doc)
        self._touch()
        return doc

    @staticmethod
    def _run_argv(argv: List[str], stdin: Optional[str] = None, timeout: float = 1800) -> str:
        proc = subprocess.run(argv, input=stdin, capture_output=True, text=True, timeout=timeout, check=False)
        if proc.returncode != 0:
            raise RuntimeError(f"{argv[0]} exited {proc.returncode}: {(proc.stderr or proc.stdout)[-1000:]}")
        return proc.stdout

    def _exec_runtime(self, plan: BootstrapPlan, step: Step) -> Any:
        """Fixed command lists for the runtime actions (exec mode)."""
        a = step.action
        if a == "firewall":
            if shutil.which("firewalld"):
                self._run_argv(["systemctl", "disable", "--now", "firewalld.service"])
            return {"firewalld": bool(shutil.which("firewalld"))}
        if a == "runtime":
            if not shutil.which("docker"):
                raise RuntimeError("container runtime not installed (exec mode requires a pre-installed docker)")
            return {"docker": self._run_argv(["docker", "version", "--format", "{{.Server.Version}}"]).strip()}
        if a == "hostname":
            hostname = _check(_HOSTNAME_RE, plan.hostname, "hostname")
            return self._run_argv(["hostnamectl", "set-hostname", hostname])
        if a == "registry_login":
            reg = _check(_IMAGE_RE, step.params.get("registry", ""), "registry")
            user = step.params.get("username", "")
            password = step.params.get("password", "")
            return self._run_argv(["docker", "login", "-u", user, "--password-stdin", reg], stdin=password)
        raise StepFailed(step.name, f"unknown runtime action {a!r}")

    def _exec_agent(self, plan: BootstrapPlan, step: Step, labels: Dict[str, str],
                    taints: Optional[List[Dict[str, str]]] = None) -> Any:
        role = plan.role if plan.role in _ROLES else ""
        if not role:
            raise ValueError(f"invalid role {plan.role!r}")
        if step.params.get("distribution", plan.distribution) == "rke2":
            return self._exec_system_agent(plan, role, labels, taints)
        image = _check(_IMAGE_RE, step.params.get("image", ""), "agent image")
        argv = ["docker", "run", "-d", "--privileged", "--restart=unless-stopped", "--net=host",
                "-v", "/etc/kubernetes:/etc/kubernetes", "-v", "/var/run:/var/run", image,
                "--server", _check(_URL_RE, plan.rancher_url, "rancher url"),
                "--token", _check(_TOKEN_RE, plan.token, "registration token"), *_ca_args(plan), f"--{role}"]
        for k in sorted(labels):
            argv += ["--label", f"{k}={labels[k]}"]
        return self._run_argv(argv + _taint_args(taints))

    def _fetch_installer(self, plan: BootstrapPlan) -> bytes:
        """The allowed server's ``system-agent-install.sh``, over TLS verified against the
        server's CA -- itself checked against the cluster's ``--ca-checksum`` first (the
        sha256 of ``GET /cacerts``; an empty CA means a publicly trusted certificate)."""
        from ..versions import SYSTEM_AGENT_INSTALL_PATH

        url = _check(_URL_RE, plan.rancher_url, "rancher url")
        client = HTTPClient(base_url=url)
        if url.startswith("https://"):
            pem = HTTPClient(base_url=url, verify_tls=False).request("GET", "/cacerts").body
            if pem.strip():
                if not hmac.compare_digest(hashlib.sha256(pem).hexdigest(), plan.ca_checksum):
                    raise RuntimeError(f"the CA {url} serves does not match the cluster's CA checksum")
                client = HTTPClient(base_url=url, ssl_context=ssl.create_default_context(cadata=pem.decode()))
        body = client.request("GET", SYSTEM_AGENT_INSTALL_PATH).body
        if not body.startswith(b"#!"):
            raise RuntimeError(f"{url}{SYSTEM_AGENT_INSTALL_PATH} is not an installer script")
        return body

    def _exec_system_agent(self, plan: BootstrapPlan, role: str, labels: Dict[str, str],
                           taints: Optional[List[Dict[str, str]]] = None) -> Any:
        script = self._fetch_installer(plan)
        fd, path = tempfile.mkstemp(prefix="tk-system-agent-install-", suffix=".sh")
        try:
            with os.fdopen(fd, "wb") as fh:
                fh.write(script)
            argv = ["sh", path, "--server", _check(_URL_RE, plan.rancher_url, "rancher url"),
                    "--label", "cattle.io/os=linux",
                    "--token", _check(_TOKEN_RE, plan.token, "registration token"),
                    *_ca_args(plan),
                    "--node-name", _check(_HOSTNAME_RE, plan.hostname, "hostname"), f"--{role}"]
            for k in sorted(labels):
                argv += ["--label", f"{k}={labels[k]}"]
            return self._run_argv(argv + _taint_args(taints))
        finally:
            os.unlink(path)

    def _run_step(self, plan: BootstrapPlan, step: Step, ctx: Dict[str, Any]) -> Any:
        a = step.action
        if a in ("firewall", "runtime", "hostname", "registry_login"):
            if self.mode == "exec":
                return self._exec_runtime(plan, step)
            return {"simulated": True}
        if a == "gpu_preflight":
            out = self._gpu_preflight(int(step.params.get("count", len(self.devices))))
            if "compute_partition" in step.params:
                # the node must run the cluster's partition modes (node/partition.py): checked
                # against the topology the labeller reads (prefetched by run_plan)
                from .partition import check, normalize, topology_modes

                want = normalize(step.params.get("compute_partition"), step.params.get("memory_partition"))
                fut = ctx.get("topology_future")
                have = topology_modes(fut.result() if fut is not None else self._topology())
                problem = check(want, have)
                if problem:
                    raise StepFailed(step.name, problem)
                out["partition"] = {"compute": want[0], "memory": want[1]}
            tuning = step.params.get("host_tuning", "off")
            if tuning != "off":
                # NUMA auto-balancing and IOMMU mode (node/hosttune.py): labels, warnings
                from . import hosttune

                f = hosttune.facts(self.root)
                ctx["labels"].update(hosttune.labels(f))
                bad = hosttune.problems(f)
                if bad and tuning == "enforce":
                    raise StepFailed(step.name, "host tuning: " + "; ".join(bad))
                out["host"] = dict(f, warnings=bad)
            return out
        if a == "gpu_labels":
            fut = ctx.get("topology_future")
            topo = fut.result() if fut is not None else self._topology()
            labels = labels_from_topology(topo)
            ctx["topology"] = topo
            ctx["labels"].update(labels)
            self.last_labels = labels
            self.write_file("/etc/triton-kubernetes/gpu-topology.json", json.dumps(topo))
            self.write_file("/etc/triton-kubernetes/gpu-labels",
                            "".join(f"{k}={v}\n" for k, v in sorted(labels.items())))
            return labels
        if a == "gpu_burnin":
            level = step.params.get("level", "full")
            parts = (step.params.get("compute_partition", "spx"), step.params.get("memory_partition", "nps1"))
            self._quiesce_gpus()
            # every (logical) GPU of the node burns in concurrently (one host thread each;
            # the probes pin their device per thread); floors scaled to a partition's share
            if len(self.devices) > 1:
                results = dict(zip(self.devices, self._pool.map(lambda d: self._burnin(d, level, parts),
                                                                self.devices)))
            else:
                results = {d: self._burnin(d, level, parts) for d in self.devices}
            out = {}
            for dev in self.devices:
                res = results[dev]
                out[str(dev)] = res
                if not res.get("ok", False):
                    raise StepFailed(step.name, f"GPU {dev}: {res.get('failures')}")
            ctx["capacity"]["amd.com/gpu"] = len(self.devices)
            # what the burn-in covered travels with the node (level, HBM held by the memtest)
            ctx["labels"].update(burnin_labels(level, results))
            return out
        if a == "gpu_health":
            # RAS verdict per physical GPU (node/health.py) on the topology the labels came
            # from; an unhealthy node fails (policy fail) or joins tainted (policy taint)
            from .health import HEALTH_TAINT, evaluate, health_labels

            topo = ctx.get("topology")
            if topo is None:
                fut = ctx.get("topology_future")
                topo = fut.result() if fut is not None else self._topology()
            self.health_limits = (int(step.params.get("max_uncorrectable", 0)),
                                  int(step.params.get("max_bad_pages", -1)))
            verdict = evaluate(topo, *self.health_limits)
            self.write_file("/etc/triton-kubernetes/gpu-health.json", json.dumps(verdict))
            ctx["labels"].update(health_labels(verdict))
            if verdict["status"] != "healthy":
                if step.params.get("policy", "fail") != "taint":
                    raise StepFailed(step.name, "unhealthy GPUs (gpu_health = fail): " + "; ".join(verdict["reasons"]))
                ctx["taints"].append(dict(HEALTH_TAINT))
            return verdict
        if a == "gpu_metrics":
            # the textfile for node_exporter (an agent node also serves GET /metrics)
            from .health import evaluate
            from .metrics import TEXTFILE_NAME, gpu_metrics

            topo = ctx.get("topology") or self._topology()
            verdict = evaluate(topo, int(step.params.get("max_uncorrectable", 0)),
                               int(step.params.get("max_bad_pages", -1)))
            path = os.path.join(str(step.params["dir"]), TEXTFILE_NAME)
            return {"file": self.write_file(path, gpu_metrics(verdict, self.name)), "served": "/metrics"}
        if a == "gpu_links":
            # every ordered GPU pair's peer read (a kernel on the receiver), disjoint pairs at
            # a time: a link below the node's median fraction or the absolute floor fails the
            # node; a pair the runtime cannot measure is recorded, not fatal
            if len(self.devices) < 2:
                return {"skipped": "single GPU"}
            if self.topology_override is not None:  # synthetic GPUs (tests / dry runs)
                return {"simulated": True}
            from ..ops import probe

            verdict = link_labels(probe.link_matrix(self.devices, method=str(step.params.get("method", "kernel-read"))),
                                  float(step.params.get("min_frac", 0.5)),
                                  float(step.params.get("min_gbps", probe.DEFAULT_MIN_LINK_GBPS)))
            ctx["labels"].update(verdict["labels"])
            if verdict["status"] == "degraded":
                raise StepFailed(step.name, f"degraded xGMI links: {verdict['degraded']}")
            return verdict
        if a == "rccl_env":
            # discovered inter-node settings, then the configured values (which win)
            env = site_env_from_topology(ctx.get("topology") or {})
            discovered = sorted(env)
            env.update(step.params.get("env", {}))
            return {"file": self.write_file("/etc/rccl/rccl.env", render_env_file(env)), "discovered": discovered}
        if a == "rccl_slim":
            # an agent chose its runtime at start (its unit's ExecStartPre prepared the
            # single-target RCCL): report which one the gate runs on
            from ..ops import native

            rt = native._runtime_dir or native.select_runtime()
            return {"runtime": rt, "slim": os.path.exists(os.path.join(str(rt), "slim.json"))}
        if a == "rccl_local":
            if len(self.devices) < 2:
                return {"skipped": "single GPU"}
            taken = self._take_node_gate()
            if taken is None and self.topology_override is not None:  # synthetic GPUs (tests / dry runs)
                return {"simulated": True}
            from ..ops import rccl

            # every local GPU as one communicator (grouped init), the verified sweep, and the
            # ~0.5 s-per-communicator teardown off the plan (drained at stop).  On a one-node
            # cluster the gate's pending communicator is exactly that: sweep it (with the
            # gate's sizes too) instead of a second init, and keep the result for the gate.
            if self.topology_override is None:
                self._used_rccl = True
            sizes = list(rccl.DEFAULT_SIZES)
            if taken is not None:
                uid, gate, meta = taken
                sizes = sorted(set(sizes) | set(meta.get("sizes") or []))
            else:
                gate = rccl.GateComm(self._make_uid(), len(self.devices), 0, self.devices, blocking=True,
                                     prealloc_bytes=max(sizes))
            res = gate.sweep(sizes, iters=10, warmup=2, async_teardown=True)
            if taken is not None:
                with self._gate_mu:
                    self._gate_results[uid] = (res, time.time())
            floor = float(step.params.get("min_busbw", 0) or 0)
            if not res.ok:
                raise StepFailed(step.name, "RCCL verification failed")
            if floor and res.peak_busbw < floor:
                raise StepFailed(step.name, f"RCCL busbw {res.peak_busbw:.0f} GB/s below {floor:.0f}")
            out = res.to_json()
            if taken is not None:
                out["shared_with"] = "cluster_gate"
            return out
        if a == "agent":
            if plan.gpu is not None:
                ctx["capacity"].setdefault("amd.com/gpu", len(self.devices))
            if self.mode == "exec":
                return self._exec_agent(plan, step, ctx["labels"], ctx["taints"])
            return self._register(plan, ctx)
        raise StepFailed(step.name, f"unknown action {a!r}")

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

    def _gpu_preflight(self, expected: int) -> Dict[str, Any]:
        if self.topology_override is not None:
            n = len(self.topology_override.get("gpus", []))
        else:
            if not os.path.exists("/dev/kfd"):
                raise RuntimeError("/dev/kfd missing (amdgpu driver not loaded)")
            from ..ops import probe

            total = probe.device_count()
            n = min(total, len(self.devices)) if self.devices else total
        if n < expected:
            raise RuntimeError(f"expected {expected} GPUs, found {n}")
        return {"gpus": n}

    def _topology(self) -> Dict[str, Any]:
        if self.topology_override is not None:
            return self.topology_override
        from ..ops import topo

        doc = topo.discover()
        gpus = doc.get("gpus", [])
        if self.devices and gpus:
            keep = [g for g in gpus if g.get("hip_id", g.get("index")) in self.devices]
            if keep:
                # re-index; drop links to GPUs that belong to other (simulated) nodes
                idx = {g["index"]: i for i, g in enumerate(keep)}
                trimmed = []
                for g in keep:
                    g = dict(g, index=idx[g["index"]])
                    g["links"] = [dict(lk, peer=idx[lk["peer"]]) for lk in g.get("links", []) if lk["peer"] in idx]
                    trimmed.append(g)
                doc = dict(doc, gpus=trimmed)
        return doc

    def _quiesce_gpus(self) -> None:
        """Let GPU work left over from an earlier request finish before the throughput
        gates run: a previous full burn-in's background release of its ~300 GB memtest
        memory would otherwise overlap (and slow) the short burn-in kernels.  A previous
        gate's communicator teardown is NOT waited for (TK_QUIESCE_TEARDOWNS=1 restores
        that): its ~0.5 s is spent inside ncclCommDestroy, and burn-ins measured next to
        it read the same as after it (round 2 A/B, in the git history of profiles/round2); a one-off
        low reading is re-measured by the burn-in itself (ops/probe.py:REMEASURE)."""
        if self.burnin_override is not None or self.topology_override is not None or not self.devices:
            return
        from ..ops import probe

        probe.wait_frees()
        if getattr(self, "_used_rccl", False) and os.environ.get("TK_QUIESCE_TEARDOWNS") == "1":
            from ..ops import rccl

            rccl.drain()

    def _burnin(self, dev: int, level: str, parts=("spx", "nps1")) -> Dict[str, Any]:
        if self.burnin_override is not None:
            return self.burnin_override(dev, level)
        from ..ops import probe

        return probe.run_burnin(dev, level, probe.Thresholds.for_partition(*parts)).to_json()

    def _register(self, plan: BootstrapPlan, ctx: Dict[str, Any]) -> Dict[str, Any]:
        roles = {"etcd": plan.role == "etcd", "controlplane": plan.role == "controlplane",
                 "worker": plan.role == "worker"}
        http = HTTPClient(base_url=plan.rancher_url, verify_tls=False)
        hdrs = {"X-API-Tunnel-Token": plan.token,
                "X-API-Tunnel-Params": tunnel_params(plan.hostname, roles, ctx["labels"], ctx["capacity"],
                                                     ctx.get("taints"))}
        if plan.distribution == "rke2":
            self._fetch_installer(plan)  # what a real node runs first
            hdrs["X-Cattle-Agent-Kind"] = "system-agent"
        return http.request("POST", "/v3/connect/register", headers=hdrs, data=b"{}").json()

    # --- RCCL gate (this node's ranks) ---------------------------------------------------------
    # Gate communicators pending by uid: started by /v1/rccl-prepare, consumed by
    # /v1/rccl-gate, released by /v1/rccl-abort, stop(), or expiry.
    GATE_TTL_S = 900.0

    def _gate_devices(self, ndev: int) -> List[int]:
        devs = self.devices or [0]
        if ndev < 1 or ndev > len(devs):
            raise ValueError(f"gate wants {ndev} GPUs, agent has {len(devs)}")
        return devs[:ndev]

    def _expire_gates(self) -> None:
        now = time.time()
        with self._gate_mu:
            stale = [k for k, e in self._gates.items() if now - e[1] > self.GATE_TTL_S]
            gates = [self._gates.pop(k)[0] for k in stale]
            for k in [k for k, e in self._gate_results.items() if now - e[1] > self.GATE_TTL_S]:
                del self._gate_results[k]
        for g in gates:
            g.abort()

    @property
    def _sim_gate(self) -> bool:
        """Synthetic GPUs without the RCCL ABI: the gate is simulated (no library call)."""
        return self.topology_override is not None and self.gate_backend != "rccl"

    def _make_uid(self) -> bytes:
        if self._sim_gate:  # synthetic GPUs (tests / dry runs)
            return secrets.token_bytes(128)
        from ..ops import rccl

        self._used_rccl = True
        return rccl.unique_id()

    def _refill_uid(self) -> None:
        uid = self._make_uid()
        with self._uid_mu:
            if self._spare_uid is None:
                self._spare_uid = uid

    def new_uid(self) -> bytes:
        """A fresh RCCL unique id (a bootstrap rendezvous address, specific to no cluster):
        the spare if one is ready, otherwise made now; either way the next spare is made on
        the agent's pool, off this request."""
        with self._uid_mu:
            uid, self._spare_uid = self._spare_uid, None
        if uid is None:
            uid = self._make_uid()
        try:
            self._pool.submit(self._refill_uid)
        except RuntimeError:  # pool shut down: the agent is stopping
            pass
        return uid

    def rccl_prepare(self, uid: Optional[bytes], world: int, rank_base: int, ndev: int = 1,
                     max_bytes: int = 0, sizes: Optional[List[int]] = None) -> Dict[str, Any]:
        """Start this node's share of a cluster communicator (non-blocking init; with
        ``max_bytes`` the init thread also allocates the sweep buffers).  ``uid`` None: this
        node hosts the rendezvous — it takes a new unique id and returns it for the others.
        ``sizes``: the gate's message sizes, so a node that is the whole gate can sweep them
        in its ``rccl_local`` step (:meth:`_take_node_gate`)."""
        devs = self._gate_devices(ndev)
        self._expire_gates()
        if uid is None:
            uid = self.new_uid()
        with span("node.rccl_prepare", node=self.name, rank_base=rank_base, world=world):
            if self._sim_gate:  # synthetic GPUs (tests / dry runs)
                gate: Any = _SimGate(devs)
            else:
                from ..ops import rccl

                self._used_rccl = True
                gate = rccl.GateComm(uid, world, rank_base, devs, blocking=False, prealloc_bytes=max_bytes)
        with self._gate_mu:
            old = self._gates.pop(uid, None)
            self._gates[uid] = (gate, time.time(), {"world": world, "rank_base": rank_base,
                                                    "sizes": [int(x) for x in (sizes or [])]})
        if old is not None:
            old[0].abort()
        return {"ok": True, "ranks": list(range(rank_base, rank_base + len(devs))), "devices": devs,
                "uid": base64.b64encode(uid).decode()}

    def rccl_abort(self, uid: bytes) -> Dict[str, Any]:
        """Release this node's ranks of gate ``uid``: a pending communicator is aborted, and a
        sweep waiting for peers is canceled (it fails at once instead of at its timeout:
        another member of the gate failed)."""
        with self._gate_mu:
            entry = self._gates.pop(uid, None)
            done = self._gate_results.pop(uid, None)
            running = self._sweeping.get(uid)
        if entry is not None:
            entry[0].abort()
        if running is not None:
            running.cancel()
        return {"ok": True, "aborted": entry is not None or done is not None, "canceled": running is not None}

    def _take_node_gate(self) -> Optional[Tuple[bytes, Any, Dict[str, Any]]]:
        """A pending gate communicator that spans exactly this node's GPUs (a one-node
        cluster: world == ndev, every rank here), taken out of the pending set.

        Its all-reduce over the node's GPUs IS the node-level RCCL check, so ``rccl_local``
        sweeps it instead of initialising a second communicator over the same GPUs on the
        bring-up path, and the cluster gate later answers from that sweep."""
        devs = list(self.devices)
        with self._gate_mu:
            for uid, (gate, _, meta) in list(self._gates.items()):
                if (meta.get("world") == len(devs) and meta.get("rank_base") == 0
                        and list(getattr(gate, "devices", [])) == devs):
                    del self._gates[uid]
                    return uid, gate, meta
        return None

    def rccl_gate(self, rank: int, world: int, uid: bytes, sizes: List[int], iters: int = 10,
                  ndev: int = 1, timeout_s: float = 600.0) -> Dict[str, Any]:
        """Run this node's ranks ``rank .. rank+ndev-1`` of the cluster gate: the pending
        communicator from rccl_prepare when there is one, else a fresh init."""
        with self._gate_mu:
            entry = self._gates.pop(uid, None)
            done = self._gate_results.pop(uid, None)
        if done is not None:
            res = done[0]
            if set(sizes) <= set(res.sizes):  # the rccl_local step swept this communicator
                idx = [res.sizes.index(x) for x in sizes]
                pick = lambda xs: [xs[i] for i in idx]  # noqa: E731
                from ..ops.rccl import SweepResult

                sub = SweepResult(res.world, res.dtype, list(sizes), pick(res.time_us), pick(res.algbw_gbps),
                                  pick(res.busbw_gbps), pick(res.errors), res.init_ms, dict(res.phase_ms))
                with span("node.rccl_gate", node=self.name, rank=rank, world=world, pipelined=True,
                          shared_with="rccl_local"):
                    out = sub.to_json()
                out.update(pipelined=True, shared_with="rccl_local",
                           ranks=list(range(rank, rank + len(self._gate_devices(ndev)))))
                return out
            # sizes the local sweep did not cover: the node is the whole gate, so a fresh
            # communicator under a new id (every rank is here) measures them
            uid = self._make_uid()
        pipelined = entry is not None
        with span("node.rccl_gate", node=self.name, rank=rank, world=world, pipelined=pipelined):
            if entry is not None:
                gate = entry[0]
            elif self._sim_gate:
                gate = _SimGate(self._gate_devices(ndev))
            else:
                from ..ops import rccl

                self._used_rccl = True
                gate = rccl.GateComm(uid, world, rank, self._gate_devices(ndev), blocking=False)
            with self._gate_mu:
                self._sweeping[uid] = gate
            try:
                # the communicator teardown is not part of the readiness answer: it is
                # joined in stop() (or by the next process-exit drain), not here
                res = gate.sweep(sizes, iters=iters, warmup=2, async_teardown=True, timeout_s=timeout_s)
            finally:
                with self._gate_mu:
                    self._sweeping.pop(uid, None)
        out = res.to_json()
        out["pipelined"] = pipelined
        out["ranks"] = list(range(rank, rank + len(gate.devices)))
        return out

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

        probe._lib()
        rccl._lib()
        self.startup_ms["dlopen"] = round((time.perf_counter() - t0) * 1e3, 1)
        # the full burn-in's ~300 GB memtest memory is released off the bring-up path
        probe.set_async_free(True)
        # burn-in arena: resident for the agent's lifetime, released after an idle period
        if os.environ.get("TK_PROBE_SCRATCH_CACHE", "1") != "0":
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
        try:
            topo.native_topology("sysfs", "/nonexistent")  # loads libtk_topo.so
        except Exception:  # noqa: BLE001 - topology falls back to other sources later
            pass

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

    # --- HTTP server ----------------------------------------------------------------------------
    def serve(self, host: str = "127.0.0.1", port: int = 0, ssl_context: Any = None) -> str:
        """Serve the API; HTTPS with ``ssl_context`` (the node's certificate), plain HTTP
        only on a loopback address."""
        if ssl_context is None and not is_loopback(host):
            raise ValueError(f"refusing to serve plain HTTP on {host}: give the agent its TLS credentials "
                             "(node credentials) or use --insecure-local, which binds loopback only")
        agent = self
        self.warm_native()

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def setup(self):
                # TLS handshake here, on this connection's own thread with a deadline: a
                # client that connects and stalls cannot block the accept loop
                if ssl_context is not None:
                    self.request.settimeout(10.0)
                    self.request.do_handshake()
                    self.request.settimeout(None)
                super().setup()
                # one request/response per segment: no Nagle/delayed-ACK stalls on keep-alive
                self.request.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

            def log_message(self, *args):
                pass

            def _reply(self, code: int, obj: Any):
                body = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                if self.close_connection:  # the client must not reuse this connection
                    self.send_header("Connection", "close")
                self.end_headers()
                self.wfile.write(body)

            def _body(self):
                n = int(self.headers.get("Content-Length") or 0)
                return json.loads(self.rfile.read(n) or b"{}") if n else {}

            def _gone(self) -> bool:
                """The agent stopped: a keep-alive connection accepted before is not served."""
                if agent._stopped:
                    self.close_connection = True
                    self._reply(503, {"error": "agent stopped"})
                return agent._stopped

            def _auth(self, read_only: bool = False) -> bool:
                """The node's agent token; for the read-only endpoints (``read_only``) also its
                scrape token (``security.metrics_token``), which is all Prometheus holds."""
                given = self.headers.get("X-TK-Agent-Token", "")
                bearer = self.headers.get("Authorization", "")
                if not given and bearer.startswith("Bearer "):  # Prometheus' scrape authorization
                    given = bearer[len("Bearer "):]
                if hmac.compare_digest(given, agent.token):
                    return True
                return read_only and hmac.compare_digest(given, metrics_token(agent.token))

            def do_GET(self):
                if self._gone():
                    return None
                path = urllib.parse.urlsplit(self.path).path
                if not self._auth(read_only=path in ("/metrics", "/v1/health")):
                    return self._reply(401, {"error": "unauthorized"})
                if urllib.parse.urlsplit(self.path).path == "/v1/info":
                    with agent._gate_mu:
                        pending = len(agent._gates)
                    return self._reply(200, {"name": agent.name, "mode": agent.mode, "devices": agent.devices,
                                             "labels": agent.last_labels, "pending_gates": pending})
                if urllib.parse.urlsplit(self.path).path == "/metrics":
                    from .metrics import CONTENT_TYPE

                    try:
                        body = agent.metrics().encode()
                    except Exception as exc:  # noqa: BLE001
                        return self._reply(500, {"error": f"{type(exc).__name__}: {exc}"})
                    self.send_response(200)
                    self.send_header("Content-Type", CONTENT_TYPE)
                    self.send_header("Content-Length", str(len(body)))
                    self.end_headers()
                    self.wfile.write(body)
                    return None
                if urllib.parse.urlsplit(self.path).path == "/v1/health":
                    try:
                        q = urllib.parse.parse_qs(urllib.parse.urlsplit(self.path).query)
                        return self._reply(200, agent.health(int(q.get("max_uncorrectable", ["0"])[0]),
                                                             int(q.get("max_bad_pages", ["-1"])[0])))
                    except Exception as exc:  # noqa: BLE001
                        return self._reply(500, {"error": f"{type(exc).__name__}: {exc}"})
                return self._reply(404, {"error": "not found"})

            def do_POST(self):
                if self._gone():
                    return None
                if not self._auth():
                    # the request body is not read: this connection cannot carry another request
                    self.close_connection = True
                    return self._reply(401, {"error": "unauthorized"})
                path = urllib.parse.urlsplit(self.path).path
                try:
                    body = self._body()
                    if path == "/v1/plan":
                        plan = BootstrapPlan.from_json(body["plan"])
                        bad = agent.refusals(plan)
                        if bad:
                            return self._reply(403, {"error": bad[0]})
                        return self._reply(200, agent.run_plan(plan))
                    if path == "/v1/rccl-uid":
                        return self._reply(200, {"uid": base64.b64encode(agent.new_uid()).decode()})
                    if path == "/v1/rccl-prepare":
                        uid = base64.b64decode(body["uid"]) if body.get("uid") else None
                        return self._reply(200, agent.rccl_prepare(uid,
                                                                   int(body["world"]), int(body["rank_base"]),
                                                                   int(body.get("ndev", 1)),
                                                                   int(body.get("max_bytes", 0)),
                                                                   [int(x) for x in body.get("sizes") or []]))
                    if path == "/v1/rccl-gate":
                        uid = base64.b64decode(body["uid"])
                        return self._reply(200, agent.rccl_gate(int(body["rank"]), int(body["world"]), uid,
                                                                [int(s) for s in body.get("sizes", [1 << 20])],
                                                                int(body.get("iters", 10)),
                                                                int(body.get("ndev", 1)),
                                                                float(body.get("timeout_s", 600.0))))
                    if path == "/v1/rccl-abort":
                        return self._reply(200, agent.rccl_abort(base64.b64decode(body["uid"])))
                    if path == "/v1/cleanup":
                        agent.last_labels = {}
                        return self._reply(200, {"ok": True})
                    if path == "/v1/shutdown":
                        # the daemon's main loop (main()) stops the agent and exits; an
                        # embedded agent (no main loop) ignores it
                        agent.shutdown_requested.set()
                        return self._reply(200, {"ok": True})
                except Exception as exc:  # noqa: BLE001
                    return self._reply(500, {"error": f"{type(exc).__name__}: {exc}"})
                return self._reply(404, {"error": "not found"})

        self._server = HTTPServer((host, port), H)
        self._server.daemon_threads = True
        if ssl_context is not None:
            self._server.socket = ssl_context.wrap_socket(self._server.socket, server_side=True,
                                                          do_handshake_on_connect=False)
        # short poll: stop() (server.shutdown) returns within ~20 ms instead of the default 0.5 s
        threading.Thread(target=self._server.serve_forever, kwargs={"poll_interval": 0.02},
                         name=f"agent-{self.name}", daemon=True).start()
        h, p = self._server.server_address[:2]
        return f"{'https' if ssl_context is not None else 'http'}://{h}:{p}"

    def stop(self) -> None:
        self._stopped = True
        cv = getattr(self, "_idle_cv", None)
        if cv is not None:
            with cv:
                self._stopping = True
                cv.notify()
            self._janitor.join(timeout=30)
            self._janitor = None
        self._pool.shutdown(wait=True)
        if self._server is not None:
            self._server.shutdown()
            self._server.server_close()
            self._server = None
        with self._gate_mu:
            pending = [e[0] for e in self._gates.values()]
            self._gates.clear()
            self._gate_results.clear()
        for g in pending:
            g.abort()
        if getattr(self, "_used_rccl", False):
            from ..ops import rccl

            rccl.drain()
        if self.devices and self.topology_override is None and self.burnin_override is None:
            from ..ops import probe

            probe.wait_frees()


def main(argv: Optional[List[str]] = None) -> int:
    """``tk-node-agent``: serve the agent API on a host (127.0.0.1 by default)."""
    import argparse

    t_main = time.perf_counter()
    ap = argparse.ArgumentParser(prog="tk-node-agent")
    ap.add_argument("--listen", default="127.0.0.1:7946")
    ap.add_argument("--mode", default="exec", choices=MODES)
    ap.add_argument("--devices", default="", help="comma-separated local GPU indices")
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
    ap.add_argument("--synthetic-gpus", type=int, default=0,
                    help="tests / CPU dry runs only: a synthetic MI355X topology with this many GPUs, "
                         "no burn-in kernels, no RCCL")
    args = ap.parse_args(argv)
    token = ""
    ssl_ctx = None
    policy = None
    host, _, port = args.listen.rpartition(":")
    if args.credentials:
        from .security import read_credentials

        creds = read_credentials(args.credentials)
        token, ssl_ctx, policy = creds["token"], creds["ssl_context"], creds["policy"]
    elif not args.insecure_local:
        ap.error("--credentials DIR is required (or --insecure-local for plain HTTP on loopback)")
    elif not is_loopback(host):
        ap.error(f"--insecure-local serves plain HTTP on loopback only, not {host}")
    else:
        from ..versions import AGENT_IMAGE

        policy = AgentPolicy([AGENT_IMAGE], servers=list(args.allow_server), loopback_servers=True)
    if args.token_file and not token:
        with open(args.token_file, "r", encoding="utf-8") as fh:
            token = fh.read().strip()
    devices = [int(d) for d in args.devices.split(",") if d.strip()]
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
                      "startup_ms": dict(getattr(agent, "startup_ms", {}),
                                         main_to_serve=round((time.perf_counter() - t_main) * 1e3, 1))}),
          flush=True)
    while not agent.shutdown_requested.wait(3600):
        pass
    t0 = time.perf_counter()
    agent.stop()
    print(json.dumps({"stopped": True, "stop_ms": round((time.perf_counter() - t0) * 1e3, 1)}), flush=True)
    sys.stdout.flush()
    sys.stderr.flush()
    if getattr(agent, "_used_rccl", False):
        from ..ops import rccl

        # every communicator was torn down by stop(); only an init still blocked on absent
        # peers would hang a normal exit (which also lets tools such as rocprofv3 finalize)
        if rccl.abandoned_inits():
            rccl.exit_now(0)
    return 0


if __name__ == "__main__":
    import sys

    sys.exit(main())
