#!/usr/bin/env python3
"""Headline benchmark: cluster create -> kubectl-ready wall-clock, bare-metal MI355X.

Metric (BASELINE.json): "cluster create->kubectl-ready wall-clock (s),
bare-metal at 1/2/4/8 workers" on config #5, "create cluster MI355X bare-metal
N-worker + ROCm device-plugin + xGMI topology labels".

One rank per GPU (``torchrun --nproc-per-node N``); every rank is one simulated
MI355X worker host running a :class:`NodeAgent` that owns its GPU.  A timed step
is one complete ``create cluster`` through the framework's real code path —
settings -> bare-metal provider -> ``main.tf.json`` -> DirectExecutor DAG ->
Rancher client -> parallel node bootstrap -> readiness waiter — with a fresh
cluster name per step, measured from the start of ``create cluster`` until the
waiter reports every phase done:

* cluster active, all nodes ``Ready``;
* every worker advertises ``amd.com/gpu`` (device-plugin add-on applied);
* per-GPU burn-in passed on each worker (HBM3E stream, bf16 + fp8 MFMA, memtest —
  hand-written gfx950 HIP kernels, run for real) and its topology labels
  (KFD sysfs via the in-process native labeller, plus RDMA NICs) attached at registration;
* a cluster-wide RCCL all-reduce gate across all N GPUs (native RCCL over xGMI).

What is simulated (and therefore excluded): the Rancher server is the
in-process v3 fake, whose RKE provisioning is instantaneous, and the host
runtime steps (docker install, hostname, agent container) are no-ops in the
agents' ``sim`` mode.  The reference publishes no number for this metric, so
``vs_baseline`` is null.

Rank 0 prints one JSON line (the driver's contract).
"""

import argparse
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "cluster create→kubectl-ready wall-clock (s), bare-metal at 1/2/4/8 workers"


def parse_args():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--burnin", default="quick", choices=["quick", "full", "off"])
    ap.add_argument("--no-rccl-gate", action="store_true")
    ap.add_argument("--rccl-mib", type=int, default=64, help="largest RCCL gate message (MiB)")
    ap.add_argument("--sim-gpu", action="store_true",
                    help="CPU dry run: synthetic topology, no burn-in kernels, no RCCL (never a valid measurement)")
    ap.add_argument("--no-gate-pipeline", action="store_true",
                    help="start the RCCL gate's communicator init after readiness instead of with the apply")
    ap.add_argument("--report", default="", help="write a per-step phase report (rank 0) to this file")
    return ap.parse_args()


def main() -> int:
    args = parse_args()
    import faulthandler

    watchdog = float(os.environ.get("TK_BENCH_WATCHDOG", "0") or 0)
    if watchdog > 0:  # debugging aid: dump every thread's Python stack periodically
        faulthandler.dump_traceback_later(watchdog, repeat=True, file=sys.stderr)
    step_watchdog = float(os.environ.get("TK_BENCH_STEP_WATCHDOG", "0") or 0)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    distributed = world > 1
    if distributed:
        # control-plane sync only (CPU); the GPU collectives are the native RCCL gate
        dist.init_process_group("gloo", init_method="env://")
    device = local_rank
    if args.sim_gpu:
        args.no_rccl_gate = True
    else:
        # one GPU per rank; a launcher that masks devices per rank leaves each rank only its own
        device = local_rank if torch.cuda.device_count() > local_rank else 0
        torch.cuda.set_device(device)

    from triton_kubernetes_amd import workflows as wf
    from triton_kubernetes_amd.backend import LocalBackend
    from triton_kubernetes_amd.config import Context, Settings
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.parallel.transport import AgentTransport
    from triton_kubernetes_amd.utils import procstat
    from triton_kubernetes_amd.utils.trace import TRACER

    token = os.environ.get("TK_BENCH_TOKEN", "bench-token-0123456789")
    work = tempfile.mkdtemp(prefix=f"tk-bench-r{rank}-")
    agent = NodeAgent(name=f"mi355x-{rank}", mode="sim", devices=[device], token=token,
                      root=os.path.join(work, "node"))
    if args.sim_gpu:
        from triton_kubernetes_amd.node.labels import synthetic_topology

        agent.topology_override = synthetic_topology(1)
        agent.burnin_override = lambda dev, level: {"ok": True, "simulated": True}
    my_url = agent.serve()
    urls = [my_url]
    if distributed:
        urls = [None] * world
        dist.all_gather_object(urls, my_url)

    fake = cp_agent = None
    backend = ctx_base = None
    devnull = open(os.devnull, "w", encoding="utf-8")  # workflow output (one handle for every step)
    if rank == 0:
        from triton_kubernetes_amd.rancher.fake import FakeRancher

        fake = FakeRancher.for_manager("bench", "bench-admin-pw-0123").start()
        cp_agent = NodeAgent(name="control-plane", mode="sim", token=token, root=os.path.join(work, "cp"))
        cp_url = cp_agent.serve()
        backend = LocalBackend(os.path.join(work, "state"))
        ctx_base = {"backend_provider": "local", "executor": "direct", "agent_token": token,
                    "non-interactive": True, "cluster_manager": "bench"}
        mgr = dict(ctx_base, manager_cloud_provider="baremetal", name="bench", rancher_admin_password="bench-admin-pw-0123",
                   host="rancher+" + fake.url, ssh_user="ubuntu", bastion_host="", key_path="~/.ssh/id_rsa")
        wf.new_manager(Context(settings=Settings(mgr, env={}), out=devnull), backend)

    sizes = [1 << 20, args.rccl_mib << 20]
    # long-lived startup objects (torch, the package, servers) leave the GC's working set,
    # so a full collection during a step does not walk them (a ~100 ms stall was measured)
    import gc

    gc.collect()
    gc.freeze()
    gc_events = []  # (generation, ms) of every collection during the run, for the report
    gc_t0 = {}

    def _gc_cb(phase, info):
        if phase == "start":
            gc_t0["t"] = time.perf_counter()
        elif "t" in gc_t0:
            gc_events.append((info.get("generation"), round((time.perf_counter() - gc_t0.pop("t")) * 1e3, 3)))

    gc.callbacks.append(_gc_cb)
    gc_mode = os.environ.get("TK_BENCH_GC", "")
    if gc_mode == "off":
        gc.disable()
    elif gc_mode.startswith("threshold:"):
        gc.set_threshold(*[int(x) for x in gc_mode.split(":", 1)[1].split(",")])

    def one_step(i: int) -> dict:
        name = f"bench-{i}"
        cfg = dict(ctx_base, cluster_cloud_provider="baremetal", name=name, k8s_version="v1.28.10-rancher1-1",
                   k8s_network_provider="flannel", gpu_addons=True, wait=True,
                   rccl_gate=not args.no_rccl_gate, rccl_pipeline=not args.no_gate_pipeline, wait_timeout=600,
                   nodes=[
                       {"rancher_host_label": "control", "node_count": 1, "hostname": f"{name}-cp",
                        "ssh_user": "ubuntu", "bastion_host": "", "key_path": "k", "hosts": ["agent+" + cp_url]},
                       {"rancher_host_label": "etcd", "node_count": 1, "hostname": f"{name}-etcd",
                        "ssh_user": "ubuntu", "bastion_host": "", "key_path": "k", "hosts": ["agent+" + cp_url]},
                       {"rancher_host_label": "worker", "node_count": world, "hostname": f"{name}-gpu",
                        "ssh_user": "ubuntu", "bastion_host": "", "key_path": "k",
                        "hosts": ["agent+" + u for u in urls], "gpu": "mi355x", "gpu_count": 1,
                        "gpu_burnin": args.burnin},
                   ])
        ctx = Context(settings=Settings(cfg, env={}), out=devnull)
        ctx.extras["agent_transport"] = AgentTransport(token=token)
        ps0 = procstat.snapshot()
        t0 = time.time()
        if step_watchdog > 0:  # diagnosis: every thread's Python stack if a step overruns
            faulthandler.dump_traceback_later(step_watchdog, file=sys.stderr)
        wf.new_cluster(ctx, backend)
        if step_watchdog > 0:
            faulthandler.cancel_dump_traceback_later()
        dt = time.time() - t0
        out = {"step": i, "seconds": dt, "proc": procstat.delta(ps0, procstat.snapshot())}
        rep = ctx.extras.get("last_readiness")
        ranks = ((rep.rccl or {}).get("ranks") or []) if rep is not None else []
        phases = [r.get("phase_ms") or {} for r in ranks]
        if phases:  # the gate's communicator init on every rank: where an N-GPU step goes
            out["rccl"] = {k: round(max(float(p.get(k, 0.0)) for p in phases), 3)
                           for k in ("init_total", "init_wait", "alloc", "sweep")}
        return out

    def sync():
        if not args.sim_gpu:
            torch.cuda.synchronize()

    def barrier():
        if distributed:
            dist.barrier()
        sync()

    results = []
    for w in range(args.warmup):
        barrier()
        if rank == 0:
            one_step(-1 - w)
        barrier()

    barrier()
    TRACER.reset()
    t_start = time.perf_counter()
    for i in range(args.steps):
        if rank == 0:
            results.append(one_step(i))
        if distributed:
            dist.barrier()
    sync()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank == 0:
        ms = elapsed / max(1, args.steps) * 1000.0
        phases = {}
        for sp in TRACER.report()["spans"]:
            if sp["name"].startswith(("ready.", "module.", "node.", "direct.apply", "apply")):
                phases.setdefault(sp["name"], []).append(sp["duration"])
        phase_ms = {k: round(sum(v) / max(1, args.steps) * 1000.0, 2) for k, v in sorted(phases.items())}
        # RCCL gate, max over ranks per step, mean over steps: communicator init wall time,
        # the part of it the readiness waiter still waited for, and the verified sweep
        gate = [r["rccl"] for r in results if "rccl" in r]
        for k in ("init_total", "init_wait", "sweep"):
            if gate:
                phase_ms[f"rccl.{k}_max_rank"] = round(sum(g[k] for g in gate) / len(gate), 2)
        line = {
            "metric": METRIC,
            "value": round(ms / 1000.0, 4),
            "unit": "s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": False,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": ("SIM-GPU DRY RUN (not a measurement); " if args.sim_gpu else "") + ("synthetic: in-process Rancher v3 fake (RKE provisioning not simulated) and sim-mode host "
                     "runtime steps; GPU steps real on MI355X (native KFD-sysfs topology + RDMA labels, HBM/MFMA/memtest "
                     f"burn-in level={args.burnin} through the agent's resident buffers, cluster-wide RCCL all-reduce "
                     f"gate {'off' if args.no_rccl_gate else 'on'}: a fresh communicator per create)"),
            "config": {
                "model": "create cluster MI355X bare-metal N-worker + ROCm device-plugin + xGMI topology labels",
                "workers": world, "gpus_per_worker": 1, "control_plane_nodes": 2,
                "global_batch": world, "seq_len": 0, "parallelism": f"{world} workers (1 GPU each)",
                "executor": "direct", "burnin": args.burnin, "rccl_gate": not args.no_rccl_gate,
                "rccl_gate_pipelined": not (args.no_rccl_gate or args.no_gate_pipeline),
            },
            "phase_ms_per_step": phase_ms,
        }
        print(json.dumps(line), flush=True)
        if args.report:
            with open(args.report, "w", encoding="utf-8") as fh:
                json.dump({"line": line, "steps": results, "trace": TRACER.report(), "gc": gc_events,
                           "cpu_quota": procstat.cpu_quota(), "cpu_affinity": len(os.sched_getaffinity(0)),
                           "cgroup_cpu_dir": procstat.cgroup_cpu_dir()},
                          fh, indent=1, default=str)
    devnull.close()
    agent.stop()
    if cp_agent is not None:
        cp_agent.stop()
    if fake is not None:
        fake.stop()
    import shutil

    shutil.rmtree(work, ignore_errors=True)  # the run's manager state, agent roots and node files
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
