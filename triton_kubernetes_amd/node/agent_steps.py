"""The node agent's plan steps: what each :class:`~.plan.BootstrapPlan` action does on a host.

Security model (``node/security.py``): the agent never executes shell text it receives.
A plan's ``shell`` fields are only for the SSH renderer; here every step dispatches on
its ``action`` and runs fixed, agent-side argv lists built from *validated* parameters
(hostname, image reference, registry, Rancher URL, token, taints: the ``_check`` patterns
below).  Which agent image and Rancher server a plan may name is decided before any step
runs (:meth:`~.agent.NodeAgent.refusals`).

* runtime steps (``firewall``, ``runtime``, ``hostname``, ``registry_login``): fixed
  commands in ``exec`` mode, recorded no-ops in ``sim`` mode;
* MI355X steps, on the agent's own GPUs through the native probes: ``gpu_preflight``
  (device count, partition modes, host tuning), ``gpu_labels`` (topology labeller, N1),
  ``gpu_burnin`` (HBM/MFMA/GEMM/memtest, every GPU concurrently), ``gpu_health`` (RAS
  verdict, taint or fail), ``gpu_metrics``, ``gpu_links`` (xGMI peer-read matrix),
  ``rccl_env``, ``rccl_slim`` and ``rccl_local`` (the node-level RCCL sweep, N2);
* ``agent``: ``docker run rancher/rancher-agent`` (RKE1) or the allowed server's
  ``system-agent-install.sh`` (RKE2) in ``exec`` mode; in ``sim`` mode the node registers
  through ``POST /v3/connect/register`` (after fetching the installer, for RKE2).
"""

import hashlib
import hmac
import json
import os
import re
import shutil
import ssl
import subprocess
import tempfile
import time
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

from ..cloud.http import HTTPClient
from ..parallel.rccl_env import render_env_file, site_env_from_topology
from ..rancher.connect import tunnel_params
from .labels import best_link_verdict, burnin_labels, labels_from_topology
from .plan import BootstrapPlan, Step

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
    if not isinstance(value, str) or not pattern.fullmatch(value):  # no trailing newline either
        raise ValueError(f"invalid {what}: {value!r}")
    return value

class AgentStepsMixin:
    """Mixin of :class:`~.agent.NodeAgent`: plan step execution and the GPU helpers it uses."""

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
            # the probes pin their device per thread); floors scaled to a partition's share.
            # A simulated burn-in (burnin_override: sim agents, tests) returns at once and runs
            # inline: hundreds of sim agents in one process would otherwise each start a
            # thread per synthetic GPU, which under one interpreter lock took ~0.1 s apiece
            if len(self.devices) > 1 and self.burnin_override is None:
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
            from ..ops import native, probe

            method = str(step.params.get("method", "kernel-read"))

            def measure():
                if probe._BURNIN_PROCESS:  # beside this process's RCCL start, as the burn-in
                    try:
                        return probe.link_matrix_process(self.devices, method=method)
                    except native.NativeUnavailable:
                        pass  # no current gpu-burnin: measured here
                return probe.link_matrix(self.devices, method=method)

            # a matrix whose only fault is speed is measured again, best of 3 per pair
            # (node/labels.py:best_link_verdict); wrong data never is
            verdict = best_link_verdict(measure, float(step.params.get("min_frac", 0.5)),
                                        float(step.params.get("min_gbps", probe.DEFAULT_MIN_LINK_GBPS)))
            verdict.pop("matrix", None)
            ctx["labels"].update(verdict["labels"])
            if verdict["status"] == "degraded":
                raise StepFailed(step.name, f"degraded xGMI links: {verdict['degraded']}")
            return verdict
        if a == "rccl_env":
            # discovered inter-node settings, then the configured values (which win)
            env = site_env_from_topology(ctx.get("topology") or {})
            discovered = sorted(env)
            env.update(step.params.get("env", {}))
            out = {"file": self.write_file("/etc/rccl/rccl.env", render_env_file(env)), "discovered": discovered}
            if self.topology_override is None and self.devices:
                # this agent's own gate runs RCCL in this process, with the environment the
                # agent started with (it loads this file at start, and so does its unit).  The
                # environment is not changed under a running agent: RCCL's threads read it
                # (getenv) while a communicator initialises, and changing it then is a data
                # race.  Configured settings that differ take effect at the agent's next start
                configured = step.params.get("env", {}) or {}
                differs = sorted(k for k, v in configured.items()
                                 if k.startswith(self.RCCL_ENV_PREFIXES) and os.environ.get(k) != str(v))
                if differs:
                    out["agent_env_differs"] = differs
            return out
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

            used = [gate] if taken is not None else []

            def fresh():
                used.append(self._new_gate(self._make_uid(), len(self.devices), 0, self.devices, blocking=True,
                                           prealloc_bytes=max(sizes)))
                return used[-1]

            # an init that ran out of HBM beside the held burn-in spans: release them, retry
            # once (node/agent_gate.py:_sweep_oom_retry)
            res, retry = self._sweep_oom_retry(
                (lambda: gate) if taken is not None else fresh, fresh,
                lambda g: g.sweep(sizes, iters=10, warmup=2, async_teardown=True))
            self._note_gate_footprint(len(self.devices), res.phase_ms, getattr(used[-1], "window", None))
            if taken is not None:
                with self._gate_mu:
                    self._gate_results[uid] = (res, time.time(), retry)
            floor = float(step.params.get("min_busbw", 0) or 0)
            if not res.ok:
                raise StepFailed(step.name, "RCCL verification failed")
            if floor and res.peak_busbw < floor:
                raise StepFailed(step.name, f"RCCL busbw {res.peak_busbw:.0f} GB/s below {floor:.0f}")
            out = res.to_json()
            if taken is not None:
                out["shared_with"] = "cluster_gate"
            if retry:
                out.update(retry)
            return out
        if a == "agent":
            if plan.gpu is not None:
                ctx["capacity"].setdefault("amd.com/gpu", len(self.devices))
            from .cleanup import join_record, read_join_record, refusal, write_join_record

            record_here = self._host_is_sandbox() or self.mode == "exec"
            if record_here:  # a host still joined to another cluster is refused (node/cleanup.py)
                why = refusal(read_join_record(self.path), plan.rancher_url, plan.token)
                if why:
                    raise StepFailed(step.name, why)
            if self.mode == "exec":
                out = self._exec_agent(plan, step, ctx["labels"], ctx["taints"])
            else:
                out = self._register(plan, ctx)
            if record_here:
                rke1_image = step.params.get("image", "") if plan.distribution == "rke1" else ""
                write_join_record(self.path, join_record(plan.rancher_url, plan.token, plan.distribution,
                                                         plan.hostname, rke1_image))
            return out
        raise StepFailed(step.name, f"unknown action {a!r}")

    def _host_is_sandbox(self) -> bool:
        """A sim-mode agent models a host under its own root; with root ``/`` it models
        nothing (it never writes to the machine it runs on)."""
        return self.mode == "sim" and self.root not in ("", "/")

    def cleanup(self) -> Dict[str, Any]:
        """``POST /v1/cleanup``: take this host out of its cluster (node/cleanup.py) --
        the vendor uninstallers at fixed paths, the RKE1 containers, the state directories
        and the join record -- keeping this agent, the node tools and the runtime."""
        from .cleanup import cleanup_host

        self.last_labels = {}
        if self.mode == "exec":
            return cleanup_host(self.path, self._run_argv, docker=shutil.which("docker"))
        if not self._host_is_sandbox():
            return {"ok": True, "simulated": True, "actions": [], "ms": 0.0}
        # sim: the host model's uninstallers (rancher/fake/hostsim.py) under this root
        return dict(cleanup_host(self.path, self._run_argv, env=dict(os.environ, TK_HOST_ROOT=self.root)),
                    simulated=True)

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
        if self._host_is_sandbox():  # what the real installer meets on this host
            from ..rancher.fake import hostsim

            why = hostsim.conflict(self.root, plan.rancher_url, plan.token)
            if why:
                raise RuntimeError(f"system-agent-install: {why}" if plan.distribution == "rke2" else why)
        http = HTTPClient(base_url=plan.rancher_url, verify_tls=False)
        hdrs = {"X-API-Tunnel-Token": plan.token,
                "X-API-Tunnel-Params": tunnel_params(plan.hostname, roles, ctx["labels"], ctx["capacity"],
                                                     ctx.get("taints"))}
        if plan.distribution == "rke2":
            self._fetch_installer(plan)  # what a real node runs first
            hdrs["X-Cattle-Agent-Kind"] = "system-agent"
        out = http.request("POST", "/v3/connect/register", headers=hdrs, data=b"{}").json()
        if self._host_is_sandbox():
            from ..rancher.fake import hostsim

            hostsim.install(self.root, plan.rancher_url, plan.token, plan.distribution)
        return out

__all__ = ["AgentStepsMixin", "StepFailed", "StepResult"]
