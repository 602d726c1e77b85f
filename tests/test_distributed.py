"""Multi-process paths on CPU: the bench harness under torchrun with the gloo control group.

``--sim-gpu`` swaps the GPU steps for synthetic topology / no-op burn-in and runs the
cluster RCCL gate over the libtk_rccl ABI stub (``ops/csrc/tk_rccl_stub.cpp``), so this
checks the distributed plumbing (agent URL all-gather, barriers, max-over-ranks timing,
rank-0 JSON line) and the gate's rank layout at the driver's 8-GPU shape — never a
measurement.
"""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("nproc,workers", [(2, 1), (4, 1), (4, 2)])
def test_bench_torchrun_gloo(nproc, workers):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for attempt in range(2):
        # a parallel test run can take the free port between this probe and torchrun's bind:
        # only that (EADDRINUSE) is retried, with a new port
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
               "--gpus", str(nproc), "--steps", "2", "--warmup", "1", "--warm-steps", "1", "--workers", str(workers),
               "--sim-gpu"]
        proc = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
        if proc.returncode == 0 or "address already in use" not in proc.stderr.lower() or attempt:
            break
    assert proc.returncode == 0, proc.stderr[-3000:]
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, proc.stdout  # rank 0 only
    doc = json.loads(lines[0])
    assert doc["n_gpus"] == nproc and doc["steps"] == 2 and doc["warmup"] == 1
    assert doc["higher_is_better"] is False and doc["scaling"] == "weak" and doc["vs_baseline"] is None
    # one worker node owns all N GPUs unless --workers splits them
    cfg = doc["config"]
    assert cfg["workers"] == workers and cfg["gpus_per_worker"] * workers == nproc
    assert cfg["simulated_phases"] == ["rke_provisioning", "runtime_install", "agent_container", "device_plugin_pod"]
    assert cfg["start"].startswith("cold")
    assert doc["data"].startswith("SIM-GPU DRY RUN")
    for phase in cfg["simulated_phases"]:
        assert phase in doc["data"]
    # value: mean create->ready of the cold steps; ms_per_step adds the agents' shutdown
    assert doc["value"] > 0 and doc["ms_per_step"] >= doc["value"] * 1000 - 1.0
    assert len(doc["create_to_ready_s"]) == 2 and doc["warm_create_to_ready_s"] > 0
    assert doc["phase_ms_per_step"]["module.host"] > 0
    assert doc["phase_ms_per_step"]["bench.agents_start"] > 0
    # the gate ran over the libtk_rccl ABI stub: every GPU of the worker tier is a rank
    assert doc["rccl_gate_ranks"] == [nproc, nproc] and "ABI stub" in doc["data"]
    assert doc["dtype"] == cfg["global_batch"] == cfg["seq_len"] == "n/a"


def test_bench_single_process_default():
    proc = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0",
                           "--sim-gpu"], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert proc.returncode == 0, proc.stderr[-2000:]
    doc = json.loads([ln for ln in proc.stdout.splitlines() if ln.startswith("{")][-1])
    assert doc["n_gpus"] == 1 and doc["unit"] == "s"
    assert doc["config"]["gpus_per_worker"] == doc["config"]["visible_gpus"] == 1


def test_bench_inproc_agents():
    """The graft smoke's shape: agents as objects in the bench process."""
    proc = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0",
                           "--agents", "inproc", "--warm-steps", "0", "--sim-gpu"],
                          capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert proc.returncode == 0, proc.stderr[-2000:]
    doc = json.loads([ln for ln in proc.stdout.splitlines() if ln.startswith("{")][-1])
    assert doc["warm_create_to_ready_s"] is None and "bench process" in doc["config"]["start"]


def test_bench_masked_launcher_one_agent_per_rank():
    """A launcher that masks devices per rank: every rank starts a 1-GPU agent, and the
    cluster has one worker per rank (the gate then spans the ranks' agents)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--warm-steps", "0", "--sim-gpu"]
    env = dict(os.environ, OMP_NUM_THREADS="1", TK_BENCH_ASSUME_MASKED="1")
    proc = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert proc.returncode == 0, proc.stderr[-3000:]
    doc = json.loads([ln for ln in proc.stdout.splitlines() if ln.startswith("{")][0])
    assert doc["config"]["workers"] == 2 and doc["config"]["gpus_per_worker"] == 1


@pytest.mark.slow
@pytest.mark.parametrize("masked", [False, True])
def test_bench_eight_ranks_gate_over_eight_gpus(masked):
    """The driver's N=8 SCALE shape on the CPU.  Unmasked: rank 0's one agent drives all 8
    ranks of the gate (ndev=8 grouped init); masked: 8 agents in 8 processes, one rank each,
    meet in the stub's cross-process rendezvous."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--steps", "1", "--warmup", "0", "--warm-steps", "0", "--sim-gpu"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    if masked:
        env["TK_BENCH_ASSUME_MASKED"] = "1"
    proc = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert proc.returncode == 0, proc.stderr[-3000:]
    doc = json.loads([ln for ln in proc.stdout.splitlines() if ln.startswith("{")][0])
    assert doc["n_gpus"] == 8 and doc["rccl_gate_ranks"] == [8]
    assert doc["config"]["workers"] == (8 if masked else 1)
    assert doc["config"]["gpus_per_worker"] == (1 if masked else 8)


def test_bench_failure_still_prints_a_diagnostic_line():
    """A run that fails (here: the second create) prints the line's shape with value null and
    the error, then fails: the first run on a new node shape leaves a diagnosis."""
    snippet = """
import sys
sys.path.insert(0, %r)
sys.argv = ["bench.py", "--sim-gpu", "--steps", "2", "--warmup", "1", "--warm-steps", "0", "--agents", "inproc"]
import triton_kubernetes_amd.workflows as wf
orig, n = wf.new_cluster, []
def boom(ctx, backend):
    n.append(1)
    if len(n) >= 2:
        raise RuntimeError("gate failed on purpose")
    return orig(ctx, backend)
wf.new_cluster = boom
import bench
bench.main()
""" % ROOT
    env = dict(os.environ, OMP_NUM_THREADS="1")
    res = subprocess.run([sys.executable, "-c", snippet], capture_output=True, text=True, timeout=300, env=env,
                         cwd=ROOT)
    assert res.returncode != 0
    line = json.loads(next(ln for ln in res.stdout.splitlines() if ln.startswith("{")))
    assert line["value"] is None and line["ms_per_step"] is None and line["completed_steps"] == 0
    assert "gate failed on purpose" in line["error"] and line["n_gpus"] == 1


def _line(stdout: str) -> dict:
    return json.loads([ln for ln in stdout.splitlines() if ln.startswith("{")][-1])


def test_bench_gpus_without_a_launcher_is_one_agent_over_n_gpus():
    """``python bench.py --gpus 8`` (no torchrun, WORLD_SIZE unset): one process, one node
    agent over devices 0..7, an 8-rank gate -- never a silent 1-GPU run."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    proc = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1",
                           "--warmup", "0", "--warm-steps", "0", "--sim-gpu"],
                          capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert proc.returncode == 0, proc.stderr[-3000:]
    assert "using WORLD_SIZE" not in proc.stderr
    doc = _line(proc.stdout)
    assert doc["n_gpus"] == 8 and doc["config"]["workers"] == 1 and doc["config"]["gpus_per_worker"] == 8
    assert doc["rccl_gate_ranks"] == [8]


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="counts on no visible GPU (the GPU box has its own test)")
def test_bench_fails_loudly_when_fewer_gpus_are_visible():
    """Without ``--sim-gpu`` this container sees no GPU: ``--gpus 2`` must not measure 0 or 1
    of them.  The line says what is wrong (value null) and the exit status is non-zero."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    proc = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                           "--warmup", "0"], capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert proc.returncode == 2
    doc = _line(proc.stdout)
    assert doc["value"] is None and doc["n_gpus"] == 2
    assert doc["error"] == "2 GPUs requested, 0 visible"


def test_bench_torchrun_world_must_match_gpus():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "4", "--steps", "1", "--warmup", "0", "--warm-steps", "0", "--sim-gpu"]
    proc = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT,
                          env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert proc.returncode != 0
    doc = _line(proc.stdout)
    assert doc["value"] is None and "WORLD_SIZE 2" in doc["error"]


def test_resolve_gpus_shapes():
    sys.path.insert(0, ROOT)
    import bench

    assert bench.resolve_gpus(8, 1, 8, sim=False) == {"n_gpus": 8, "visible": 8, "masked": False}
    assert bench.resolve_gpus(2, 1, 8, sim=False)["masked"] is False  # devices 0..1 of 8
    assert bench.resolve_gpus(8, 8, 8, sim=False)["masked"] is False  # torchrun, every rank sees all
    assert bench.resolve_gpus(8, 8, 1, sim=False)["masked"] is True   # torchrun, one GPU per rank
    assert bench.resolve_gpus(8, 1, 0, sim=True)["visible"] == 8
    for args, msg in (((8, 1, 1), "8 GPUs requested, 1 visible"), ((2, 1, 0), "2 GPUs requested, 0 visible"),
                      ((4, 2, 4), "WORLD_SIZE 2"), ((0, 1, 1), "at least 1"), ((8, 8, 0), "0 visible to rank")):
        with pytest.raises(bench.GpuCountError, match=msg):
            bench.resolve_gpus(*args, sim=False)


def test_bench_run_budget_end_to_end_under_torchrun():
    """The budget in the real loop, over 2 gloo ranks, with a slow (simulated) driver clear
    before each step: rank 0 decides, every rank follows -- the warm creates are shed, the
    later settles capped, and every timed step still runs."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--warm-steps", "2", "--sim-gpu", "--time-budget", "20"]
    env = dict(os.environ, OMP_NUM_THREADS="1", TK_BENCH_SIM_SETTLE_S="6")
    proc = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert proc.returncode == 0, proc.stderr[-3000:]
    doc = _line(proc.stdout)
    rb = doc["run_budget"]
    assert rb["shed"] == ["warm_creates", "hbm_settle_capped"] and rb["settle_cap_s"] < 6, rb
    assert rb["capped_settles"] >= 1
    assert doc["steps"] == 3 and len(doc["create_to_ready_s"]) == 3 and doc["warm_create_to_ready_s"] is None
    assert max(doc["hbm_settle_s"][1:]) < 6.0
    assert "the run budget capped" in doc["data"] and "warm creates were shed" in doc["data"]


def test_bench_carries_the_node_gate_footprint_from_step_to_step():
    """A node keeps /etc/triton-kubernetes/gate-footprint.json across agent restarts; the
    bench's cold steps start fresh agents in fresh roots but carry that file, as a node
    would.  Over the ABI stub a gate reports a 900 MiB per-process footprint."""
    env = dict(os.environ, OMP_NUM_THREADS="1", TK_RCCL_STUB_FOOTPRINT_MIB="900")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    proc = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                           "--warmup", "1", "--warm-steps", "0", "--sim-gpu"], capture_output=True, text=True,
                          timeout=240, cwd=ROOT, env=env)
    assert proc.returncode == 0, proc.stderr[-3000:]
    doc = _line(proc.stdout)
    assert doc["node_gate_footprints"] == {"mi355x-0": {"2": 900.0}}, doc["node_gate_footprints"]
    assert doc["rccl_footprint_mib"]["footprint_total_mib"] == 900.0
