"""MI355X native probe tests (real GPU).  Run with ``pytest -m gpu``."""

import json
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def probe():
    from triton_kubernetes_amd.ops import probe as p

    assert p.device_count() >= 1
    return p


def test_device_is_mi355x(probe):
    info = probe.device_info(0)
    assert info.is_gfx950, info
    assert info.wavefront_size == 64
    assert info.compute_units == 256
    assert info.total_mem_gib > 250


def test_hbm_bandwidth(probe):
    bw = probe.hbm_bandwidth(0, 2 << 30, iters=5)
    print(json.dumps(bw))
    # achievable is ~6.3 TB/s; a healthy GPU streams well above half of it
    assert bw["read_gbps"] > 3500
    assert bw["copy_gbps"] > 3500
    assert bw["write_gbps"] > 3000


@pytest.mark.parametrize("dtype,floor", [("bf16", 1300.0), ("fp8", 2600.0), ("f32", 80.0)])
def test_mfma_peak(probe, dtype, floor):
    r = probe.mfma_peak(0, dtype, iters=20000 if dtype != "f32" else 4000)
    print(dtype, json.dumps(r))
    assert r["tflops"] > floor


@pytest.mark.parametrize("dtype", ["bf16", "fp8", "f32"])
def test_mfma_issue_rate_at_held_clock(probe, dtype):
    """The MFMA loop issues at the per-clock peak; what it lacks in TFLOP/s vs the dense
    figures is the clock the chip holds under load (DVFS), measured in-kernel."""
    r = probe.mfma_clock(0, dtype, iters=20000 if dtype != "f32" else 4000, warm_ms=1000)
    print(dtype, json.dumps(r))
    assert 800 < r["mhz"] < 2500
    assert r["issue_efficiency"] > 0.85


def test_memtest_clean_and_detects_corruption(probe):
    r = probe.memtest(0, 1 << 30, passes=1)
    assert r["errors"] == 0
    assert probe.memtest_selfcheck(0, 64 << 20, 5) == 5
    assert probe.memtest_selfcheck(0, 64 << 20, 0) == 0


def test_memtest_passes_are_complementary_pairs(probe):
    """Pass 2k+1 writes the complement of pass 2k's pattern, so every bit is tested at 0 and
    at 1.  A stuck-at-0 bit (fail point: bit 0 of N words cleared after each fill) then
    mismatches in exactly one pass of the pair: two passes count exactly N, whatever the
    pattern's value there (independent random patterns would count about N/2 per pass)."""
    stuck = 4096
    probe.set_fail_point(f"memtest.stuck0={stuck}")
    try:
        one = probe.memtest(0, 256 << 20, passes=1)
        two = probe.memtest(0, 256 << 20, passes=2)
        four = probe.memtest(0, 256 << 20, passes=4)
    finally:
        probe.set_fail_point("")
    assert two["errors"] == stuck and four["errors"] == 2 * stuck, (one, two, four)
    assert 0 < one["errors"] < stuck  # one pass alone sees only the words whose bit was 1
    assert probe.memtest(0, 256 << 20, passes=2)["errors"] == 0


def test_burnin_quick(probe):
    res = probe.run_burnin(0, "quick")
    print(json.dumps(res.to_json(), default=str))
    assert res.ok, res.failures


def test_memtest_span_covers_most_of_hbm(probe):
    """The full burn-in's memtest: every free byte but the headroom, distinct chunks held
    at once (~270 GiB of the 288 GiB card), clean."""
    res = probe.memtest_span(0, 0, chunk=32 << 30, headroom=8 << 30, passes=1)
    print(json.dumps(res))
    assert res["errors"] == 0
    assert res["hbm_bytes"] > 250 << 30 and res["bytes"] > 0.85 * res["hbm_bytes"]


def test_burnin_labels_record_coverage(probe):
    from triton_kubernetes_amd.node.labels import burnin_labels

    res = probe.run_burnin(0, "quick").to_json()
    labels = burnin_labels("quick", {0: res})
    assert labels["amd.com/gpu.burnin"] == "passed" and labels["amd.com/gpu.burnin-level"] == "quick"
    assert labels["amd.com/gpu.burnin-hbm-tested-gib"] == "1" and float(labels["amd.com/gpu.burnin-hbm-tested-pct"]) < 1


def test_burnin_arena_resident_across_runs(probe):
    probe.release_scratch()  # the arena is process-wide: start from an empty one
    held = probe.prealloc_scratch(0, "quick")
    assert held == 2 << 30  # two 1 GiB stream buffers; the memtest runs in the first
    try:
        for _ in range(2):  # both runs stream/memtest through the resident buffers
            res = probe.run_burnin(0, "quick")
            assert res.ok, res.failures
    finally:
        freed = probe.release_scratch()
        probe.set_scratch_cache(False)
    assert freed == held
    assert probe.release_scratch() == 0


def test_rccl_single_rank_and_local():
    from triton_kubernetes_amd.ops import rccl

    assert rccl.version() > 0
    uid = rccl.unique_id()
    r = rccl.sweep_rank(0, 1, uid, 0, sizes=[1 << 20, 64 << 20], iters=5, warmup=2)
    assert r.ok and len(r.busbw_gbps) == 2
    r2 = rccl.sweep_local(1, sizes=[1 << 20], iters=5, warmup=1, dtype="bf16")
    assert r2.ok


def test_rccl_ready_executable():
    from triton_kubernetes_amd.ops.native import executable

    proc = subprocess.run([executable("rccl-ready"), "--ngpus", "1", "--iters", "3"], capture_output=True,
                          text=True, timeout=300)
    assert proc.returncode == 0, proc.stderr
    doc = json.loads([ln for ln in proc.stdout.splitlines() if ln.startswith("{")][-1])
    assert doc["ok"] and doc["ngpus"] == 1


def test_rccl_ready_cluster_mode_through_process_gate(tmp_path):
    """The SSH/Terraform nodes' cluster gate with the real tool: rank-0 node prints the
    unique id, joins, runs the verified sweep (1 node x 1 GPU here; the protocol is the
    same for N nodes)."""
    import os

    from triton_kubernetes_amd.ops.native import LIB_DIR
    from triton_kubernetes_amd.parallel.transport import HostRef, LocalTransport
    from triton_kubernetes_amd.readiness.process_gate import ProcessGate

    env_file = tmp_path / "rccl.env"
    env_file.write_text('NCCL_DEBUG="WARN"\n')
    gate = ProcessGate(LocalTransport(), [HostRef("local")], [1], [1 << 20, 16 << 20], iters=3, timeout=240,
                       tools_dir=LIB_DIR, env_file=str(env_file))
    res = gate.run()
    assert res["ok"] and res["world"] == 1 and res["mode"] == "process", res
    rank = res["ranks"][0]
    assert rank["rc"] == 0 and [r["bytes"] for r in rank["results"]] == [1 << 20, 16 << 20]
    assert all(r["errors"] == 0 for r in rank["results"]) and rank["init_ms"] > 0
    assert os.path.exists(os.path.join(LIB_DIR, "rccl-ready"))


def test_process_gate_two_nodes_rendezvous_and_fail_fast(tmp_path):
    """Two rccl-ready --cluster processes (world 2) on the box's one GPU: the unique id
    travels from the first process to the second and the bootstrap rendezvous completes --
    then RCCL refuses two ranks on one device ("invalid usage", its duplicate-GPU check runs
    on the exchanged peer info), and the gate fails fast instead of hanging."""
    import time

    from triton_kubernetes_amd.errors import TKError
    from triton_kubernetes_amd.ops.native import LIB_DIR
    from triton_kubernetes_amd.parallel.transport import HostRef, LocalTransport
    from triton_kubernetes_amd.readiness.process_gate import ProcessGate

    gate = ProcessGate(LocalTransport(), [HostRef("local"), HostRef("local")], [1, 1], [1 << 20], iters=2,
                       timeout=90, tools_dir=LIB_DIR, env_file=str(tmp_path / "none"))
    t0 = time.monotonic()
    try:
        res = gate.run()
        assert not res["ok"]
        assert all("invalid usage" in r.get("stderr", "") for r in res["ranks"]), res
    except TKError as exc:
        assert "invalid usage" in str(exc), exc
    assert time.monotonic() - t0 < 60


def test_link_matrix_child_matches_in_process():
    """The agent's links step runs ``gpu-burnin --p2p-child``: the same matrix form as the
    in-process measurement, for every GPU of the box.  A one-GPU box lists GPU 0 three times
    (pairs of a device with itself): the child's round-robin rounds, bye slot, peer reads and
    data checks then run as on a multi-GPU node."""
    from triton_kubernetes_amd.ops import probe

    devs = list(range(probe.device_count())) if probe.device_count() >= 2 else [0, 0, 0]
    child = probe.link_matrix_process(devs)
    here = probe.link_matrix(devs)
    assert set(child) == set(here) and child["method"] == here["method"] == "kernel-read"
    assert set(child["pairs"]) == set(here["pairs"]) and not child["errors"] and not child["data_errors"]
    for k, v in child["pairs"].items():  # 64 MiB peer reads: within a factor of two of each other
        assert 0.5 * here["pairs"][k] <= v <= 2.0 * here["pairs"][k], (k, v, here["pairs"][k])


def test_link_check_on_this_box(tmp_path):
    """The per-link xGMI check: on a one-GPU box it reports "single GPU" (exit 0, empty
    labels); the copy primitive it times still runs (device to itself)."""
    from triton_kubernetes_amd.ops import probe
    from triton_kubernetes_amd.ops.native import executable

    labels = tmp_path / "links"
    proc = subprocess.run([executable("gpu-burnin"), "--p2p", "--labels", str(labels)], capture_output=True,
                          text=True, timeout=120)
    assert proc.returncode == 0, proc.stderr
    doc = json.loads(proc.stdout.strip().splitlines()[-1])
    if probe.device_count() < 2:
        assert doc == {"skipped": "single GPU"} and labels.read_text() == ""
    else:
        assert doc["status"] == "passed" and "amd.com/xgmi.link-check=passed" in labels.read_text()
    r = probe.p2p_bandwidth(0, 0, 64 << 20, 3)
    assert r["gbps"] > 100  # a device-local copy through the same path
    cli = subprocess.run([sys.executable, "-m", "triton_kubernetes_amd", "gpu", "links"], capture_output=True,
                         text=True, timeout=120)
    assert cli.returncode == 0, cli.stderr
    if probe.device_count() < 2:
        assert json.loads(cli.stdout) == {"skipped": "single GPU"}


def test_link_matrix_rounds_cover_every_ordered_pair():
    """tkp_link_matrix's round-robin schedule (odd n: a bye each round) over three
    "devices" that are all GPU 0: every ordered pair is timed once, concurrently with the
    other pairs of its round, and nothing is left allocated or mapped."""
    import ctypes

    from triton_kubernetes_amd.ops import probe

    lib = probe._lib()
    for n in (2, 3, 4):
        gbps = (ctypes.c_double * (n * n))()
        acc = (ctypes.c_int * (n * n))()
        t0 = time.monotonic()
        rc = lib.tkp_link_matrix((ctypes.c_int * n)(*([0] * n)), n, 32 << 20, 2, gbps, acc)
        assert rc == 0, lib.tkp_last_error()
        vals = [gbps[i * n + j] for i in range(n) for j in range(n) if i != j]
        assert len(vals) == n * (n - 1) and all(v > 50 for v in vals), (n, vals)
        assert all(gbps[i * n + i] == 0.0 for i in range(n))
        assert time.monotonic() - t0 < 10


def test_kernel_peer_read_matrix_and_floor():
    """The primary link number is a kernel on the receiver reading the sender's memory
    (k_peer_read).  On one GPU the "peers" are GPU 0 itself, so both methods time a
    device-local transfer through the same schedule; every pair clears the absolute floor
    and the verdict records the method."""
    from triton_kubernetes_amd.node.labels import link_labels
    from triton_kubernetes_amd.ops import probe

    devs = [0, 0, 0, 0] if probe.device_count() < 2 else list(range(probe.device_count()))
    kread = probe.link_matrix(devs, 64 << 20, 3, method="kernel-read")
    sdma = probe.link_matrix(devs, 64 << 20, 3, method="sdma-copy")
    print(json.dumps({"kernel-read": kread["pairs"], "sdma-copy": sdma["pairs"]}))
    n = len(devs)
    assert kread["method"] == "kernel-read" and not kread["errors"] and len(kread["pairs"]) == len(set(
        f"{i}-{j}" for a, i in enumerate(devs) for b, j in enumerate(devs) if a != b))
    assert all(v > probe.DEFAULT_MIN_LINK_GBPS for v in kread["pairs"].values()), kread
    verdict = link_labels(kread)
    assert verdict["status"] == "passed" and verdict["labels"]["amd.com/xgmi.p2p-method"] == "kernel-read"
    assert n >= 2 and all(v > 0 for v in sdma["pairs"].values())


def test_topology_amdsmi():
    from triton_kubernetes_amd.ops import topo

    doc = topo.discover()
    print(json.dumps(doc)[:2000])
    assert doc["gpus"], doc
    g = doc["gpus"][0]
    assert "MI355" in g.get("market_name", "") or g.get("target_graphics_version", "").startswith("gfx950")


def test_labeller_executable():
    from triton_kubernetes_amd.ops.native import executable

    proc = subprocess.run([executable("amdgpu-topo-labeller")], capture_output=True, text=True, timeout=120)
    assert proc.returncode == 0, proc.stdout + proc.stderr
    assert json.loads(proc.stdout)["gpus"]


def test_native_labels_match_python_spec():
    """amd_smi and sysfs collectors (C++) agree, and both equal labels_from_topology (Python)."""
    import time

    from triton_kubernetes_amd.node.labels import labels_from_topology
    from triton_kubernetes_amd.ops import topo

    t0 = time.perf_counter()
    via_amdsmi = topo.amdsmi_labels(source="amdsmi")
    t1 = time.perf_counter()
    via_sysfs = topo.native_labels("sysfs")
    t2 = time.perf_counter()
    print(json.dumps({"amdsmi_ms": (t1 - t0) * 1e3, "sysfs_inprocess_ms": (t2 - t1) * 1e3}))
    print(json.dumps(via_sysfs, sort_keys=True))
    assert via_sysfs == via_amdsmi
    assert via_amdsmi == labels_from_topology(topo.amdsmi_topology())
    assert via_sysfs == labels_from_topology(topo.native_topology("sysfs"))
    assert via_sysfs["amd.com/gpu.product-name"] == "MI355X"
    assert via_sysfs["amd.com/gpu.target"] == "gfx950"
    assert via_sysfs["amd.com/gpu.vram"] == "288G"
    # the document fields both collectors read agree too (PCIe link, driver version)
    smi, sysfs = topo.amdsmi_topology(), topo.native_topology("sysfs")
    assert smi["driver"]["version"] == sysfs["driver"]["version"]
    for a, b in zip(smi["gpus"], sysfs["gpus"]):
        for k in ("pcie_width", "pcie_max_width", "pcie_max_speed_gts"):
            assert a.get(k) == b.get(k), k


def test_gate_comm_nonblocking_then_sweep():
    from triton_kubernetes_amd.ops import rccl

    g = rccl.GateComm(rccl.unique_id(), 1, 0, [0], blocking=False)
    r = g.sweep([1 << 20, 16 << 20], iters=3, warmup=1)
    print(json.dumps(r.phase_ms))
    assert r.ok and r.phase_ms["init_total"] > 0 and len(r.busbw_gbps) == 2
    g2 = rccl.GateComm(rccl.unique_id(), 1, 0, [0], blocking=False)
    g2.abort()
    assert rccl.pending_gates() == 0
    rccl.drain()


def test_gate_abort_mid_init_with_missing_peer():
    """world=2 with only rank 0 present: init cannot finish; abort must return at once (own process, bounded)."""
    code = ("import time; from triton_kubernetes_amd.ops import rccl; "
            "g = rccl.GateComm(rccl.unique_id(), 2, 0, [0], blocking=False); time.sleep(0.3); "
            "assert not g.ready(); t = time.time(); g.abort(); dt = time.time() - t; "
            "assert dt < 1.0, dt; assert rccl.pending_gates() == 0 and rccl.abandoned_inits() == 1; "
            "print('aborted-ok', round(dt * 1e3, 3)); rccl.exit_now(0)")
    proc = subprocess.run(["timeout", "-k", "5", "60", sys.executable, "-c", code], capture_output=True, text=True,
                          cwd=ROOT)
    assert proc.returncode == 0 and "aborted-ok" in proc.stdout, proc.stdout[-2000:] + proc.stderr[-2000:]


def test_agent_pipelined_gate_over_http():
    import base64

    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.parallel.transport import AgentTransport, HostRef

    agent = NodeAgent("gate-test", "sim", devices=[0], token="t0k")
    url = agent.serve()
    try:
        tr = AgentTransport(token="t0k")
        host = HostRef("agent+" + url)
        uid = tr.post(host, "/v1/rccl-uid", {})["uid"]
        assert len(base64.b64decode(uid)) == 128
        prep = tr.post(host, "/v1/rccl-prepare", {"uid": uid, "world": 1, "rank_base": 0, "ndev": 1})
        assert prep["ok"] and prep["ranks"] == [0]
        res = tr.post(host, "/v1/rccl-gate", {"uid": uid, "rank": 0, "world": 1, "ndev": 1, "sizes": [1 << 20],
                                             "iters": 3})
        assert res["ok"] and res["pipelined"] and res["ranks"] == [0]
        # prepare then abort leaves nothing pending
        uid2 = tr.post(host, "/v1/rccl-uid", {})["uid"]
        tr.post(host, "/v1/rccl-prepare", {"uid": uid2, "world": 1, "rank_base": 0, "ndev": 1})
        assert tr.post(host, "/v1/rccl-abort", {"uid": uid2})["aborted"] is True
    finally:
        agent.stop()


def test_default_runtime_maps_system_rccl_and_slim_is_verified_opt_in(tmp_path):
    """by default a fresh process (no torch) runs on /opt/rocm's librccl.  The
    single-target copy is opt-in: prepare() verifies it on the GPU (one-rank all-reduce in a
    child that must map it) before TK_HIP_RUNTIME=slim may select it."""
    from triton_kubernetes_amd.ops import native, rccl_slim

    code = ("import json, time; from triton_kubernetes_amd.ops import native, rccl\n"
            "t = time.perf_counter(); g = rccl.GateComm(rccl.unique_id(), 1, 0, [0], blocking=True)\n"
            "init_ms = (time.perf_counter() - t) * 1e3\n"
            "r = g.sweep([1 << 20, 8 << 20], iters=3, warmup=1, async_teardown=False)\n"
            "maps = [ln.split()[-1] for ln in open('/proc/self/maps') if 'librccl' in ln]\n"
            "print(json.dumps({'ok': r.ok, 'init_ms': init_ms, 'runtime': native.runtime_dir(),\n"
            "                  'rccl': sorted({os.path.realpath(m) for m in maps})}))\n")
    code = "import os\n" + code

    def run(**env):
        e = dict(os.environ, TK_RCCL_SLIM_DIR=str(tmp_path / "slim"))
        e.pop("TK_HIP_RUNTIME", None)
        e.update(env)
        proc = subprocess.run(["timeout", "-k", "5", "120", sys.executable, "-c", code], capture_output=True,
                              text=True, cwd=ROOT, env=e)
        assert proc.returncode == 0, proc.stdout[-2000:] + proc.stderr[-2000:]
        return json.loads([ln for ln in proc.stdout.splitlines() if ln.startswith("{")][-1])

    default = run()
    system_rccl = os.path.realpath(os.path.join(native.SYSTEM_LIB_DIR, "librccl.so"))
    assert default["ok"] and default["runtime"] == "system" and default["rccl"] == [system_rccl], default
    meta = rccl_slim.prepare(native.SYSTEM_LIB_DIR, root=str(tmp_path / "slim"))
    assert meta["verified"] and meta["loaded_code_object_bytes"] < meta["code_object_bytes"]
    slim = run(TK_HIP_RUNTIME="slim")
    print(json.dumps({"default": default, "slim": slim, "prepare": meta}))
    assert slim["ok"] and slim["runtime"] == meta["dir"]
    assert slim["rccl"] == [os.path.realpath(os.path.join(str(meta["dir"]), "librccl.so"))]


@pytest.mark.parametrize("point", ["memtest_span.after_alloc", "memtest_span.after_launch"])
def test_memtest_span_releases_everything_on_error(point):
    """an error inside the span memtest must not leave its chunks (up to ~300 GB
    in a full burn-in), the stream or the events allocated in a long-lived agent."""
    from triton_kubernetes_amd.ops import probe

    probe.wait_frees()
    before = probe.free_bytes(0)
    probe.set_fail_point(point)
    try:
        with pytest.raises(probe.ProbeError, match="injected failure"):
            probe.memtest_span(0, 48 << 30, chunk=16 << 30)
    finally:
        probe.set_fail_point("")
    after = probe.free_bytes(0)
    assert after >= before - (1 << 30), (before, after)
    # the next span memtest on the same GPU runs normally
    ok = probe.memtest_span(0, 4 << 30, chunk=2 << 30)
    assert ok["errors"] == 0 and ok["bytes"] == 4 << 30


def test_memtest_span_with_nothing_allocatable_reports_zero():
    from triton_kubernetes_amd.ops import probe

    res = probe.memtest_span(0, 4 << 40, chunk=2 << 40)  # a 2 TiB chunk never fits
    assert res["bytes"] == 0 and res["errors"] == 0


def test_memtest_span_tests_what_it_can_hold_when_hbm_shrinks():
    """the span is sized from hipMemGetInfo when it runs; HBM another
    process takes between that read and the allocations (simulated: chunk allocations after
    the third fail) shrinks the span instead of failing it, and everything is released."""
    from triton_kubernetes_amd.ops import probe

    probe.wait_frees()
    before = probe.free_bytes(0)
    probe.set_fail_point("memtest_span.alloc_limit=3")
    try:
        res = probe.memtest_span(0, 8 << 30, chunk=1 << 30)
    finally:
        probe.set_fail_point("")
    assert res["errors"] == 0 and res["bytes"] == 3 << 30
    probe.wait_frees()
    assert probe.free_bytes(0) >= before - (1 << 30)


def test_full_span_leaves_other_processes_memory_alone(tmp_path):
    """The driver's multi-rank SCALE shape: other processes hold contexts (and memory) on the
    GPU while the agent's full memtest runs.  The span covers what is free then, minus the
    headroom, and the other process's data is intact and it can still allocate."""
    from triton_kubernetes_amd.ops import probe

    holder = tmp_path / "holder.py"
    holder.write_text(
        "import sys, torch\n"
        "def chunk(k):  # 1 GiB of distinct int32 values (one arange kernel per GiB)\n"
        "    return torch.arange(k << 28, (k + 1) << 28, dtype=torch.int32, device='cuda')\n"
        "x = [chunk(k) for k in range(16)]  # 16 GiB\n"
        "torch.cuda.synchronize(); print('held', flush=True)\n"
        "sys.stdin.readline()\n"
        "ok = all(bool((x[k] == chunk(k)).all()) for k in range(16))\n"
        "y = torch.empty(1 << 30, dtype=torch.uint8, device='cuda')\n"
        "print('intact' if ok else 'corrupt', flush=True)\n")
    proc = subprocess.Popen([sys.executable, str(holder)], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        assert proc.stdout.readline().strip() == "held"
        probe.wait_frees()
        free_now = probe.free_bytes(0)
        res = probe.memtest_span(0, 0, headroom=4 << 30, passes=1)
        print(json.dumps(dict(res, free_before=free_now)))
        assert res["errors"] == 0
        assert free_now - (5 << 30) <= res["bytes"] <= free_now - (4 << 30)
        probe.wait_frees()
        out, _ = proc.communicate("go\n", timeout=120)
        assert proc.returncode == 0 and out.strip().endswith("intact"), out
    finally:
        if proc.poll() is None:
            proc.kill()


def test_full_span_memtests_the_burnin_arena_too(probe):
    """A full burn-in's bandwidth step grows the agent's arena to 2 x 16 GiB; the span
    memtest takes those buffers over and tests them in place (no free of 32 GiB, and no
    driver clearing of it, just before the span's own allocations), so that HBM is tested
    rather than left beside the span."""
    probe.set_scratch_cache(True)
    try:
        probe.prealloc_scratch(0, "full")
        probe.wait_frees()
        held_free = probe.free_bytes(0)
        res = probe.memtest_span(0, 0, headroom=4 << 30, passes=1)
        assert res["errors"] == 0
        assert res["bytes"] > held_free  # the 32 GiB the arena held were part of the span
        assert probe.release_scratch() == 0  # nothing was left cached
    finally:
        probe.release_scratch()
        probe.set_scratch_cache(False)
        probe.wait_frees()


def test_full_span_in_a_child_process(probe):
    """The agent's full memtest runs in ``gpu-burnin --memtest-span``: the verdict comes back
    while the child still holds the span; once it has exited the HBM is free again, and
    this process's HIP calls were never queued behind its frees."""
    probe.wait_frees()
    before = probe.free_bytes(0)
    t0 = time.perf_counter()
    res = probe.memtest_span_process(0, 0, headroom=4 << 30, passes=1, release_arena=False)
    verdict_s = time.perf_counter() - t0
    t1 = time.perf_counter()
    probe.memtest(0, 256 << 20, 1)  # this process's GPU work right after the verdict
    own_s = time.perf_counter() - t1
    probe.wait_frees()
    after = probe.free_bytes(0)
    print(json.dumps(dict(res, verdict_s=round(verdict_s, 3), own_memtest_s=round(own_s, 3),
                          free_before_gib=before / 2 ** 30, free_after_gib=after / 2 ** 30)))
    assert res["errors"] == 0
    assert before - (5 << 30) <= res["bytes"] <= before - (3 << 30)
    assert after >= before - (1 << 30)


def test_link_matrix_checks_the_data_it_moved():
    """Each pair's received data is checked against the sender's pattern after its last
    transfer: clean on a healthy device, and one flipped word (fail point) is reported on
    exactly one pair, which the verdict marks corrupt."""
    from triton_kubernetes_amd.node.labels import link_labels
    from triton_kubernetes_amd.ops import probe

    devs = [0, 0, 0] if probe.device_count() < 2 else list(range(min(4, probe.device_count())))
    for method in ("kernel-read", "sdma-copy"):
        clean = probe.link_matrix(devs, 32 << 20, 2, method=method)
        assert not clean["errors"] and clean["data_errors"] == {}, clean
    probe.set_fail_point("link_matrix.corrupt")
    try:
        hit = probe.link_matrix(devs, 32 << 20, 2, method="kernel-read")
    finally:
        probe.set_fail_point("")
    assert list(hit["data_errors"].values()) == [1], hit
    verdict = link_labels(hit, min_gbps=0.0)
    assert verdict["status"] == "degraded" and verdict["corrupt"] == list(hit["data_errors"])


def test_eight_concurrent_burnins_in_one_process(probe):
    """The agent burns in every GPU of a node at once, one thread each (node/agent_steps.py).
    On a one-GPU box the eight threads share GPU 0: throughput is split eight ways (the
    floors are off here), but the host code -- arena slots, streams, events, per-thread
    errors, the GEMM screen's one-time setup -- runs eight-way concurrent for real, and every
    correctness check must still hold."""
    import concurrent.futures as cf

    th = probe.Thresholds(min_read_frac=0.0, min_bf16_frac=0.0, min_fp8_frac=0.0, min_gemm_frac=0.0,
                          min_gemm_fp8_frac=0.0)
    probe.set_scratch_cache(True)
    try:
        with cf.ThreadPoolExecutor(max_workers=8) as pool:
            results = list(pool.map(lambda _: probe.run_burnin(0, "quick", th), range(8)))
    finally:
        probe.release_scratch()
    for r in results:
        assert r.ok, r.failures
        assert r.memtest["errors"] == 0 and r.gemm["ok"] and r.gemm_fp8["ok"], r.to_json()
        assert r.hbm["read_gbps"] > 0 and r.mfma["bf16"]["tflops"] > 0
    print(json.dumps({"read_gbps": [round(r.hbm["read_gbps"]) for r in results],
                      "bf16_tflops": [round(r.mfma["bf16"]["tflops"]) for r in results]}))


def test_rccl_preload_finds_a_kernel_handle_on_the_installed_librccl():
    """``tkr_preload_device_code`` must start on the librccl this box runs --
    /opt/rocm's (an agent's default runtime, no torch in the process) and torch's (a process
    that imported torch first).  A ROCm update that renames RCCL's kernels past what the
    scan recognises fails here, not as ~60 ms more on every create."""
    code = ("import json, time; from triton_kubernetes_amd.ops import native, rccl\n"
            "rccl.version()\n"
            "ok = rccl.preload_device_code([0])\n"
            "while rccl.preloads_running():\n"
            "    time.sleep(0.01)\n"
            "print(json.dumps(dict(rccl.preload_report(), started=ok, runtime=native.runtime_dir())), flush=True)\n"
            "rccl.exit_now(0)\n")
    env = dict(os.environ)
    env.pop("TK_HIP_RUNTIME", None)
    proc = subprocess.run(["timeout", "-k", "5", "120", sys.executable, "-c", code], capture_output=True, text=True,
                          cwd=ROOT, env=env)
    assert proc.returncode == 0, proc.stdout[-2000:] + proc.stderr[-2000:]
    system = json.loads([ln for ln in proc.stdout.splitlines() if ln.startswith("{")][-1])
    print(json.dumps({"system": system}))
    assert system["runtime"] == "system" and system["started"] is True
    assert system["how"] == "known" and "ncclDevKernel_Generic" in system["symbol"], system

    import torch  # noqa: F401  (this process: torch's librccl, loaded first)
    from triton_kubernetes_amd.ops import rccl

    assert rccl.preload_device_code([0]) is True
    while rccl.preloads_running():
        time.sleep(0.01)
    rep = rccl.preload_report()
    print(json.dumps({"in_process": rep}))
    assert rep["how"] in ("known", "scan") and "ncclDevKernelArgsStorage" in rep["symbol"], rep


def test_bench_refuses_more_gpus_than_visible():
    """``bench.py --gpus N`` (no launcher) with fewer than N GPUs visible (on
    this one-GPU box: ``--gpus 2``) must fail with the reason in its line, never measure one
    GPU as two."""
    import torch

    have = torch.cuda.device_count()
    want = have + 1
    proc = subprocess.run(["timeout", "-k", "5", "120", sys.executable, os.path.join(ROOT, "bench.py"), "--gpus",
                           str(want), "--steps", "1", "--warmup", "0"], capture_output=True, text=True, cwd=ROOT,
                          env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert proc.returncode == 2, proc.stdout[-2000:] + proc.stderr[-2000:]
    line = json.loads([ln for ln in proc.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["value"] is None and line["n_gpus"] == want
    assert line["error"] == f"{want} GPUs requested, {have} visible", line


def test_gate_communicator_footprint_is_measured():
    """the gate communicator's device footprint -- this process's own VRAM
    (KFD accounting, ``footprint_kind`` 1) where reachable, else the device's used-memory
    delta (kind 2: inside a PID namespace, as on this box; the agent keeps that only from a
    window without burn-in activity).  It sizes the burn-in span's headroom
    (node/agent_gate.py:span_headroom)."""
    code = ("import json; from triton_kubernetes_amd.ops import rccl\n"
            "g = rccl.GateComm(rccl.unique_id(), 1, 0, [0], blocking=False, prealloc_bytes=64 << 20)\n"
            "r = g.sweep([1 << 20, 64 << 20], iters=3, warmup=1, async_teardown=False)\n"
            "print(json.dumps({'ok': r.ok, 'footprint_mib': r.phase_ms['footprint_mib'],\n"
            "                  'footprint_total_mib': r.phase_ms['footprint_total_mib'],\n"
            "                  'footprint_kind': r.phase_ms['footprint_kind']}), flush=True)\n"
            "rccl.exit_now(0)\n")
    env = dict(os.environ)
    env.pop("TK_HIP_RUNTIME", None)
    proc = subprocess.run(["timeout", "-k", "5", "120", sys.executable, "-c", code], capture_output=True, text=True,
                          cwd=ROOT, env=env)
    assert proc.returncode == 0, proc.stdout[-2000:] + proc.stderr[-2000:]
    got = json.loads([ln for ln in proc.stdout.splitlines() if ln.startswith("{")][-1])
    print(json.dumps({"gate_footprint": got}))
    assert got["ok"] and got["footprint_kind"] in (1.0, 2.0)
    # RCCL's device code plus one rank's buffers; the 2 x 64 MiB sweep buffers on top
    assert 64 <= got["footprint_mib"] <= 8192, got
    assert got["footprint_total_mib"] >= got["footprint_mib"] + 128, got
