#!/usr/bin/env python3
"""Control-plane scaling on CPU: ``create cluster --wait`` over W MI355X worker nodes.

The GPU bench (bench.py) measures one 8-GPU node on real hardware; this measures the
orchestration around it at fleet scale, where nothing is simulated away except the GPU
work and RKE itself:

* W node agents (sim mode, 8 synthetic MI355X GPUs each, every one with its own HTTP
  server) plus one control-plane agent, all in this process;
* the in-process Rancher v3 fake (instantaneous RKE, asynchronous registration tokens);
* the real workflow: settings -> bare-metal provider -> main.tf.json -> DirectExecutor
  DAG (node bootstrap fanned out over W agents) -> add-ons -> readiness waiter (cluster
  active, W+1 nodes Ready, 8W ``amd.com/gpu`` allocatable) -> the cluster RCCL gate with
  8W ranks (prepare fanned out with the apply, sweep after readiness; sim gates).

Prints one JSON line per W: create->ready wall-clock, per-phase times, and the thread
count at the peak.  ``--workers 8,32,128`` picks the sizes.
"""

import argparse
import io
import json
import os
import sys
import tempfile
import threading
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from triton_kubernetes_amd import versions  # noqa: E402
from triton_kubernetes_amd import workflows as wf  # noqa: E402
from triton_kubernetes_amd.backend import LocalBackend  # noqa: E402
from triton_kubernetes_amd.config import Context, Settings  # noqa: E402
from triton_kubernetes_amd.node.agent import NodeAgent  # noqa: E402
from triton_kubernetes_amd.node.labels import synthetic_topology  # noqa: E402
from triton_kubernetes_amd.parallel.transport import AgentTransport  # noqa: E402
from triton_kubernetes_amd.rancher.fake import FakeRancher  # noqa: E402
from triton_kubernetes_amd.utils.trace import TRACER  # noqa: E402

TOKEN = "control-plane-scale-token"


def run(workers: int, gpus: int, root: str, parallelism: int = 0) -> dict:
    fake = FakeRancher.for_manager("mgr", "tk-admin-pw-0123").start()
    t0 = time.perf_counter()
    agents = [NodeAgent(name=f"g{i}", mode="sim", devices=list(range(gpus)), token=TOKEN,
                        root=os.path.join(root, f"g{i}"), topology_override=synthetic_topology(gpus))
              for i in range(workers)]
    for a in agents:
        a.burnin_override = lambda dev, level: {"ok": True, "simulated": True, "level": level}
    cp = NodeAgent(name="cp", mode="sim", token=TOKEN, root=os.path.join(root, "cp"))
    urls = ["agent+" + a.serve() for a in agents]
    cp_url = "agent+" + cp.serve()
    t_agents = time.perf_counter() - t0
    backend = LocalBackend(os.path.join(root, "state"))
    base = {"backend_provider": "local", "executor": "direct", "agent_token": TOKEN, "non-interactive": True,
            "cluster_manager": "mgr"}
    out = io.StringIO()
    wf.new_manager(Context(settings=Settings(dict(base, manager_cloud_provider="baremetal", name="mgr",
                                                  rancher_admin_password="tk-admin-pw-0123",
                                                  rancher_bootstrap_password=fake.bootstrap_password, host="rancher+" + fake.url, ssh_user="u", bastion_host="",
                                                  key_path="k"), env={}), out=out), backend)
    cfg = dict(base, cluster_cloud_provider="baremetal", name=f"fleet-{workers}",
               k8s_version=versions.DEFAULT_K8S_VERSION, k8s_network_provider="flannel", gpu_addons=True, wait=True,
               rccl_gate=True, wait_timeout=600, **({"direct_parallelism": parallelism} if parallelism else {}),
               nodes=[{"rancher_host_label": "control", "node_count": 1, "hostname": "cp", "ssh_user": "u",
                       "bastion_host": "", "key_path": "k", "hosts": [cp_url]},
                      {"rancher_host_label": "etcd", "node_count": 1, "hostname": "etcd", "ssh_user": "u",
                       "bastion_host": "", "key_path": "k", "hosts": [cp_url]},
                      {"rancher_host_label": "worker", "node_count": workers, "hostname": "gpu", "ssh_user": "u",
                       "bastion_host": "", "key_path": "k", "hosts": urls, "gpu": "mi355x", "gpu_count": gpus,
                       "gpu_burnin": "quick"}])
    ctx = Context(settings=Settings(cfg, env={}), out=out)
    ctx.extras["agent_transport"] = AgentTransport(token=TOKEN)
    TRACER.reset()
    peak = [threading.active_count()]
    stop = threading.Event()

    def sample():
        while not stop.wait(0.05):
            peak[0] = max(peak[0], threading.active_count())

    sampler = threading.Thread(target=sample, daemon=True)
    sampler.start()
    t1 = time.perf_counter()
    wf.new_cluster(ctx, backend)
    create = time.perf_counter() - t1
    stop.set()
    rep = ctx.extras.get("last_readiness")
    phases = {}
    spans = TRACER.report()["spans"]
    agg = {}
    for sp in spans:
        n, tot, mx = agg.get(sp["name"], (0, 0.0, 0.0))
        agg[sp["name"]] = (n + 1, tot + sp["duration"], max(mx, sp["duration"]))
    top = {k: {"n": n, "sum_ms": round(t * 1e3, 1), "max_ms": round(m * 1e3, 1)}
           for k, (n, t, m) in sorted(agg.items(), key=lambda kv: -kv[1][2])[:12]}
    for sp in spans:
        if sp["name"] in ("direct.apply", "module.cluster", "module.host", "module.addon", "gate.prepare") or \
                sp["name"].startswith("ready."):
            phases[sp["name"]] = max(phases.get(sp["name"], 0.0), round(sp["duration"] * 1e3, 1))
    rccl = (rep.rccl or {}) if rep is not None else {}
    for a in agents + [cp]:
        a.stop()
    fake.stop()
    return {"workers": workers, "gpus": workers * gpus, "create_to_ready_s": round(create, 3),
            "agents_start_s": round(t_agents, 3), "phase_ms_max": phases, "peak_threads": peak[0],
            "slowest_spans": top,
            "gate": {"ok": rccl.get("ok"), "world": rccl.get("world"), "nodes": rccl.get("nodes"),
                     "pipelined": rccl.get("pipelined")}}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--workers", default="8,32,128")
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--parallelism", type=int, default=0, help="direct_parallelism (0: the default)")
    args = ap.parse_args()
    for w in [int(x) for x in args.workers.split(",")]:
        with tempfile.TemporaryDirectory(prefix=f"tk-scale-{w}-") as root:
            print(json.dumps(run(w, args.gpus, root, args.parallelism)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
