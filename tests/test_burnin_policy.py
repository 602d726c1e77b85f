"""Burn-in gate policy (``ops/probe.py:run_burnin``) with scripted measurements: a
throughput gate that reads low once is measured again, a GPU that reads low every time
fails, and a GEMM checksum mismatch in any run fails the GPU even if a later run is clean."""

import pytest

from triton_kubernetes_amd.ops import gemm, probe


def _info():
    return probe.DeviceInfo(0, "AMD Instinct MI355X", "gfx950:sramecc+:xnack-", 256, 64, 2400.0, 288.0, 287.0,
                            4 << 20, "0000:05:00.0")


def _screen(tflops, bad=0, dtype="bf16"):
    return gemm.ScreenResult(4096, 4096, 4096, tflops, 0.1, bad, bad, 0 if bad else -1, 0 if bad else -1, 0.01,
                             dtype)


@pytest.fixture
def scripted(monkeypatch):
    """Queues of results per measurement; the last value repeats."""
    script = {"hbm": [6800.0], "bf16": [1850.0], "fp8": [4000.0], "gemm_bf16": [_screen(1400.0)],
              "gemm_fp8": [_screen(2500.0, dtype="fp8")]}
    calls = {k: 0 for k in script}

    def take(key):
        i = calls[key]
        calls[key] += 1
        q = script[key]
        return q[min(i, len(q) - 1)]

    monkeypatch.setattr(probe, "device_info", lambda dev: _info())
    monkeypatch.setattr(probe, "hbm_bandwidth", lambda *a, **k: {"read_gbps": take("hbm"), "write_gbps": 6000.0,
                                                                  "copy_gbps": 5500.0})
    monkeypatch.setattr(probe, "mfma_peak", lambda dev, dtype, iters, *a, **k: {"tflops": take(dtype)})
    monkeypatch.setattr(gemm, "screen", lambda dev, m, n, k, reps, dtype="bf16": take(f"gemm_{dtype}"))
    monkeypatch.setattr(probe, "memtest", lambda dev, nbytes, passes: {"errors": 0, "verify_gbps": 5000.0})
    return script, calls


def test_healthy_gpu_measured_once(scripted):
    script, calls = scripted
    res = probe.run_burnin(0, "quick")
    assert res.ok and res.remeasured == [] and set(calls.values()) == {1}


def test_one_low_reading_is_measured_again(scripted):
    script, calls = scripted
    script["gemm_fp8"] = [_screen(1334.0, dtype="fp8"), _screen(2450.0, dtype="fp8")]  # one overlapped run
    script["hbm"] = [3000.0, 6900.0]
    res = probe.run_burnin(0, "quick")
    assert res.ok, res.failures
    assert res.remeasured == ["hbm", "gemm_fp8"]
    assert res.gemm_fp8["tflops"] == 2450.0 and res.hbm["read_gbps"] == 6900.0


def test_slow_every_time_fails_after_three_runs(scripted):
    script, calls = scripted
    script["bf16"] = [900.0]
    res = probe.run_burnin(0, "quick")
    assert not res.ok and any("bf16 MFMA 900 TF" in f for f in res.failures)
    assert calls["bf16"] == 1 + probe.REMEASURE


def test_checksum_mismatch_is_never_retried_away(scripted):
    script, calls = scripted
    # a corrupted AND slow first run, then a clean fast one: the GPU still fails
    script["gemm_bf16"] = [_screen(600.0, bad=3), _screen(1400.0)]
    res = probe.run_burnin(0, "quick")
    assert not res.ok and any("checksum mismatch" in f for f in res.failures)
    # a corrupted run at full speed is not re-measured at all, and fails too
    script["gemm_bf16"] = [_screen(1400.0, bad=1)]
    calls["gemm_bf16"] = 0
    res = probe.run_burnin(0, "quick")
    assert not res.ok and calls["gemm_bf16"] == 1


def test_default_burnin_level_is_full():
    """a node joining a cluster memtests its whole HBM by default; quick
    stays an explicit choice.  Pinned at every place a default lives."""
    import os
    import re

    from triton_kubernetes_amd.models import baremetal
    from triton_kubernetes_amd.node.plan import build_host_plan
    from triton_kubernetes_amd.state import State
    from triton_kubernetes_amd.terraform.catalog import MODULES_DIR

    from helpers import make_ctx

    st = State("mgr")
    name = baremetal.new_cluster(make_ctx({"name": "dev", "k8s_version": "v1.28.10-rancher1-1",
                                           "k8s_network_provider": "flannel"}), None, st)
    key = st.clusters()[name]
    node = {"rancher_host_label": "worker", "node_count": 1, "hostname": "g", "ssh_user": "u", "bastion_host": "",
            "key_path": "k", "hosts": ["10.0.0.20"], "gpu": "mi355x"}
    baremetal.new_node(make_ctx(node), "mgr", key, None, st)
    assert st.module("node_baremetal_dev_g-1")["gpu_burnin"] == "full"
    baremetal.new_node(make_ctx(dict(node, hosts=["10.0.0.21"], gpu_burnin="quick")), "mgr", key, None, st)
    assert st.module("node_baremetal_dev_g-2")["gpu_burnin"] == "quick"  # explicit choice kept
    # the Terraform host module's own default
    text = open(os.path.join(MODULES_DIR, "bare-metal-mi355x-rancher-k8s-host", "variables.tf")).read()
    block = re.search(r'variable "gpu_burnin" \{(.*?)\n\}', text, re.S).group(1)
    assert re.search(r'default\s*=\s*"full"', block)
    # a plan built from a block without the key, and the on-node executable's default
    cfg = dict(st.module("node_baremetal_dev_g-1"))
    cfg.pop("gpu_burnin")
    plan = build_host_plan(cfg, "https://r", "t", "c", mi355x=True)
    step = next(s for s in plan.steps if s.action == "gpu_burnin")
    assert step.params["level"] == "full"
    src = open(os.path.join(os.path.dirname(probe.__file__), "csrc", "tk_gpu_probe.hip")).read()
    assert 'const char* level = "full";' in src


def test_partitioned_full_memtest_frees_the_arena_before_sizing(scripted, monkeypatch):
    order = []
    monkeypatch.setattr(probe, "release_scratch", lambda dev=None: order.append(("release", dev)) or 0)
    monkeypatch.setattr(probe, "free_bytes", lambda dev: order.append(("free", dev)) or (280 << 30))
    monkeypatch.setattr(probe, "memtest_span", lambda dev, nbytes, passes=1: order.append(("span", nbytes)) or {
        "errors": 0, "verify_gbps": 5000.0, "bytes": nbytes, "hbm_bytes": 288 << 30})
    res = probe.run_burnin(0, "full", probe.Thresholds.for_partition("cpx", "nps2"))
    assert res.ok, res.failures
    assert [o[0] for o in order] == ["release", "free", "span"]


@pytest.fixture
def span_child(tmp_path, monkeypatch):
    """A stand-in gpu-burnin: prints the verdict line its argv asks for, then 'releases' for
    ``FAKE_RELEASE_S`` before it exits (what the real one's hipFree + driver clearing take)."""
    import stat
    import sys

    exe = tmp_path / "gpu-burnin"
    exe.write_text(f"""#!{sys.executable}
import json, os, sys, time
a = sys.argv
open(os.environ["FAKE_SPAN_ARGV"], "a").write(" ".join(a[1:]) + "\\n")
mode = os.environ.get("FAKE_SPAN_MODE", "ok")
if mode == "silent":
    sys.exit(3)
if mode == "error":
    print(json.dumps({{"ok": False, "error": "hipMalloc: out of memory"}}), flush=True)
    sys.exit(2)
if mode == "stale":  # a gpu-burnin that predates --memtest-span: a whole burn-in's report
    print(json.dumps({{"level": "full", "gpus": [{{"device": 0, "ok": True}}], "ok": True}}), flush=True)
    sys.exit(0)
n = int(a[a.index("--span-bytes") + 1]) or (300 << 30)
print("a library's banner on stdout", flush=True)
print(json.dumps({{"ok": True, "errors": 0, "verify_gbps": 6100.0, "bytes": n, "hbm_bytes": 309 << 30,
                  "alloc_ms": 412.0, "test_ms": 300.0}}), flush=True)
time.sleep(float(os.environ.get("FAKE_RELEASE_S", "0")))
""")
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)
    argv_log = tmp_path / "argv.log"
    monkeypatch.setenv("FAKE_SPAN_ARGV", str(argv_log))
    monkeypatch.setattr(probe, "_burnin_exe", lambda: str(exe))
    released = []
    monkeypatch.setattr(probe, "release_scratch", lambda dev=None: released.append(dev) or 0)

    class _Lib:
        def tkp_wait_frees(self):
            return 0

    monkeypatch.setattr(probe, "_lib", lambda: _Lib())
    return argv_log, released


def test_span_child_reports_before_it_releases(span_child, monkeypatch):
    """The agent's full memtest runs in a gpu-burnin child: the verdict comes back as soon as
    the child prints it; the release happens in the child, and wait_frees (and the same
    device's next span) wait for it to exit."""
    import time

    argv_log, released = span_child
    monkeypatch.setenv("FAKE_RELEASE_S", "3.0")
    t0 = time.monotonic()
    res = probe.memtest_span_process(3, 0, headroom=4 << 30, passes=3)
    assert time.monotonic() - t0 < 2.5  # did not wait for the release (margin for a loaded CPU)
    assert res["errors"] == 0 and res["bytes"] == 300 << 30 and res["free_ms"] == 0.0
    assert released == [3]  # this process's arena is part of the span
    assert argv_log.read_text().split() == ["--memtest-span", "--device", "3", "--span-bytes", "0",
                                            "--span-headroom", str(4 << 30), "--span-passes", "3",
                                            "--span-chunk", str(probe.SPAN_CHILD_CHUNK)]
    assert [d for d, _ in probe._span_children] == [3]
    probe.wait_frees()
    assert time.monotonic() - t0 >= 2.9 and probe._span_children == []


def test_span_child_waits_only_for_its_own_device(span_child, monkeypatch):
    """Concurrent spans on other devices (every GPU of a node burns in at once) do not wait
    for each other; a device's next span waits for its previous one's release."""
    import time

    monkeypatch.setenv("FAKE_RELEASE_S", "2.5")
    t0 = time.monotonic()
    probe.memtest_span_process(0, 1 << 30)
    probe.memtest_span_process(1, 1 << 30)
    assert time.monotonic() - t0 < 2.2  # (margin for a loaded CPU)
    probe.memtest_span_process(0, 1 << 30)  # waits for device 0's first child
    assert time.monotonic() - t0 >= 2.5
    probe.wait_frees()


def test_span_child_failures_are_errors(span_child, monkeypatch):
    monkeypatch.setenv("FAKE_SPAN_MODE", "error")
    with pytest.raises(probe.ProbeError, match="out of memory"):
        probe.memtest_span_process(0)
    monkeypatch.setenv("FAKE_SPAN_MODE", "silent")
    with pytest.raises(probe.ProbeError, match="exited 3 without a verdict"):
        probe.memtest_span_process(0)
    probe.wait_frees()


def test_span_child_stale_binary_is_an_error_not_a_keyerror(span_child, monkeypatch):
    """a stale gpu-burnin that ignores --memtest-span prints a whole burn-in's
    report (no ``errors``); that is a ProbeError naming the binary, not a KeyError."""
    monkeypatch.setenv("FAKE_SPAN_MODE", "stale")
    with pytest.raises(probe.ProbeError, match="no memtest-span verdict"):
        probe.memtest_span_process(0)
    probe.wait_frees()


@pytest.mark.parametrize("how", ["missing", "unstartable"])
def test_span_child_unusable_binary_falls_back_in_process(span_child, monkeypatch, tmp_path, how):
    """A missing or stale gpu-burnin (NativeUnavailable from native.executable) or one that
    cannot be started runs the same span memtest in this process, and says so."""
    from triton_kubernetes_amd.ops import native

    if how == "missing":
        def nope():
            raise native.NativeUnavailable("gpu-burnin is not built and building it failed: no hipcc")
        monkeypatch.setattr(probe, "_burnin_exe", nope)
    else:
        monkeypatch.setattr(probe, "_burnin_exe", lambda: str(tmp_path / "no-such-gpu-burnin"))
    calls = []
    monkeypatch.setattr(probe, "memtest_span", lambda dev, nbytes, headroom, passes: calls.append(dev) or {
        "errors": 0, "verify_gbps": 1.0, "bytes": 8, "hbm_bytes": 16, "alloc_ms": 0.0, "test_ms": 0.0,
        "free_ms": 0.0})
    res = probe.memtest_span_process(2, 0)
    assert calls == [2] and res["errors"] == 0
    assert ("no hipcc" if how == "missing" else "cannot start") in res["span_fallback"]


def test_executable_refuses_a_stale_tool_it_cannot_rebuild(monkeypatch):
    from triton_kubernetes_amd.ops import build, native

    monkeypatch.setattr(build, "current", lambda name: False)

    def fail(**kw):
        raise RuntimeError("hipcc: not found")
    monkeypatch.setattr(build, "build", fail)
    with pytest.raises(native.NativeUnavailable, match="hipcc: not found"):
        native.executable("gpu-burnin")


def test_full_burnin_uses_the_span_child_when_enabled(scripted, span_child, monkeypatch):
    monkeypatch.setattr(probe, "memtest_span", lambda *a, **k: pytest.fail("in-process span used"))
    probe.set_span_process(True)
    try:
        res = probe.run_burnin(0, "full")
    finally:
        probe.set_span_process(False)
        probe.wait_frees()
    assert res.ok and res.memtest["bytes"] == 300 << 30 and "process_ms" in res.memtest


def test_a_stuck_span_child_is_killed(span_child, monkeypatch):
    monkeypatch.setenv("FAKE_RELEASE_S", "60")
    monkeypatch.setattr(probe, "SPAN_RELEASE_TIMEOUT_S", 0.5)
    probe.memtest_span_process(0, 1 << 30)
    (_, proc), = probe._span_children
    probe.wait_frees()
    assert proc.returncode is not None and proc.returncode < 0 and probe._span_children == []


# --- the whole burn-in in a gpu-burnin child (node agents) -------------------------------------

CHILD_OK = {
    "ok": True, "device": 0,
    "info": {"name": "AMD Instinct MI355X", "arch": "gfx950:sramecc+:xnack-", "compute_units": 256,
             "wavefront_size": 64, "clock_khz": 2400000, "total_mem": 309 << 30, "free_mem": 300 << 30,
             "l2_bytes": 4 << 20, "pci_domain": 0, "pci_bus": 117, "pci_device": 0},
    "hbm": {"read_gbps": 6500.0, "write_gbps": 6200.0, "copy_gbps": 5800.0},
    "bf16": {"tflops": 1950.0, "ms": 1.0}, "fp8": {"tflops": 4300.0, "ms": 1.0},
    "gemm": {"tflops": 1400.0, "ms": 0.8, "bad_columns": 0, "bad_rows": 0, "first_bad_column": -1,
             "first_bad_row": -1, "max_norm_error": 0.01},
    "gemm_fp8": {"tflops": 2900.0, "ms": 0.4, "bad_columns": 0, "bad_rows": 0, "first_bad_column": -1,
                 "first_bad_row": -1, "max_norm_error": 0.01},
    "gemm_first_bad": None, "gemm_fp8_first_bad": None,
    "memtest": {"errors": 0, "verify_gbps": 6100.0, "bytes": 300 << 30, "hbm_bytes": 309 << 30,
                "alloc_ms": 900.0, "test_ms": 337.0},
    "remeasured": [], "phase_ms": {"hbm": 180.0, "memtest": 1300.0},
}


@pytest.fixture
def burnin_child(tmp_path, monkeypatch):
    """A stand-in ``gpu-burnin --burnin-child``: prints the verdict in $FAKE_CHILD_DOC."""
    import stat
    import sys

    exe = tmp_path / "gpu-burnin"
    exe.write_text(f"""#!{sys.executable}
import os, sys
open(os.environ["FAKE_CHILD_ARGV"], "w").write(" ".join(sys.argv[1:]))
print("a banner", flush=True)
print(os.environ["FAKE_CHILD_DOC"], flush=True)
""")
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)
    monkeypatch.setattr(probe, "_burnin_exe", lambda: str(exe))
    monkeypatch.setenv("FAKE_CHILD_ARGV", str(tmp_path / "argv"))

    class _Lib:
        def tkp_wait_frees(self):
            return 0

    monkeypatch.setattr(probe, "_lib", lambda: _Lib())
    monkeypatch.setattr(probe, "device_info", lambda dev: pytest.fail("in-process burn-in used"))
    probe.set_burnin_process(True)
    yield tmp_path / "argv"
    probe.set_burnin_process(False)
    probe.wait_frees()


def test_burnin_child_passes_levels_and_floors_and_is_judged_here(burnin_child, monkeypatch):
    import json

    monkeypatch.setenv("FAKE_CHILD_DOC", json.dumps(CHILD_OK))
    res = probe.run_burnin(0, "full")
    assert res.ok, res.failures
    assert res.device.is_gfx950 and res.memtest["bytes"] == 300 << 30 and "process" in res.phase_ms
    argv = burnin_child.read_text().split()
    assert argv[:3] == ["--burnin-child", "--device", "0"]
    hbm_bytes, hbm_iters, mfma_iters, mt_bytes, passes = probe.LEVELS["full"]
    opts = dict(zip(argv[3::2], argv[4::2]))
    assert opts["--hbm-bytes"] == str(hbm_bytes) and opts["--memtest-bytes"] == "0" and opts["--memtest-passes"] == "3"
    assert opts["--gemm"] == "8192,8192,8192,5" and opts["--span-chunk"] == str(probe.SPAN_CHILD_CHUNK)
    assert opts["--span-headroom"] == str(4 << 30)
    probe.set_span_headroom((4 << 30) + 7 * (512 << 20))  # an 8-GPU node's agent
    try:
        probe.run_burnin(0, "full")
        opts = dict(zip(burnin_child.read_text().split()[3::2], burnin_child.read_text().split()[4::2]))
        assert opts["--span-headroom"] == str((4 << 30) + 7 * (512 << 20))
    finally:
        probe.set_span_headroom(4 << 30)
    assert float(opts["--min-read-gbps"]) == pytest.approx(probe._floors(probe.Thresholds())["read"], rel=1e-3)
    labels = __import__("triton_kubernetes_amd.node.labels", fromlist=["burnin_labels"]).burnin_labels(
        "full", {0: res.to_json()})
    assert labels["amd.com/gpu.burnin"] == "passed"


def test_burnin_child_failures_are_the_same_verdicts(burnin_child, monkeypatch):
    import json

    bad = dict(CHILD_OK, hbm={"read_gbps": 900.0, "write_gbps": 1.0, "copy_gbps": 1.0},
               gemm_first_bad={"tflops": 1400.0, "ms": 1, "bad_columns": 2, "bad_rows": 1, "first_bad_column": 7,
                               "first_bad_row": 3, "max_norm_error": 9.0},
               memtest=dict(CHILD_OK["memtest"], errors=12))
    monkeypatch.setenv("FAKE_CHILD_DOC", json.dumps(bad))
    res = probe.run_burnin(0, "full")
    assert not res.ok
    text = "; ".join(res.failures)
    assert "HBM read 900 GB/s below" in text and "memtest: 12 mismatching words" in text
    assert "GEMM checksum mismatch: 1 rows / 2 columns (first at row 3, column 7)" in text
    monkeypatch.setenv("FAKE_CHILD_DOC", json.dumps({"ok": False, "error": "hipMalloc: out of memory"}))
    with pytest.raises(probe.ProbeError, match="out of memory"):
        probe.run_burnin(0, "quick")
    monkeypatch.setenv("FAKE_CHILD_DOC", json.dumps({"level": "full", "gpus": [], "ok": True}))  # a stale binary
    with pytest.raises(probe.ProbeError, match="no burn-in verdict"):
        probe.run_burnin(0, "quick")


def test_partitions_of_one_pool_burn_in_in_process(burnin_child, monkeypatch):
    """Concurrent partitions share an HBM pool: the span is sized per partition here, so
    they keep the in-process path (the child tests a whole GPU's HBM)."""
    called = []
    monkeypatch.setattr(probe, "_burnin_child", lambda *a, **k: called.append(a))
    monkeypatch.setattr(probe, "device_info", lambda dev: (_ for _ in ()).throw(RuntimeError("in-process")))
    with pytest.raises(RuntimeError, match="in-process"):
        probe.run_burnin(0, "full", probe.Thresholds.for_partition("cpx", "nps2"))
    assert not called


def test_child_releases_its_hbm_only_when_the_hold_says(burnin_child, monkeypatch, tmp_path):
    """The agent's release hold (node/agent_gate.py:_await_rccl_inits): the child gets
    --hold-stdin and frees what it tested when its stdin closes, not at its verdict."""
    import json
    import sys
    import threading
    import time

    exe = tmp_path / "gpu-burnin"
    released = tmp_path / "released"
    exe.write_text(f"""#!{sys.executable}
import os, sys
open(os.environ["FAKE_CHILD_ARGV"], "w").write(" ".join(sys.argv[1:]))
print(os.environ["FAKE_CHILD_DOC"], flush=True)
if "--hold-stdin" in sys.argv:
    sys.stdin.read()  # until the parent closes the pipe
open({str(released)!r}, "w").write("freed")
""")
    monkeypatch.setenv("FAKE_CHILD_DOC", json.dumps(CHILD_OK))
    go = threading.Event()
    probe.set_release_hold(go.wait)
    try:
        res = probe.run_burnin(0, "full")
        assert res.ok
        argv = burnin_child.read_text().split()
        assert "--hold-stdin" in argv and argv[argv.index("--hold-max-ms") + 1] == str(probe.RELEASE_HOLD_MAX_MS)
        time.sleep(0.3)
        assert not released.exists()  # verdict in hand, HBM still held
        go.set()
        probe.wait_frees()
        assert released.read_text() == "freed"
    finally:
        go.set()
        probe.set_release_hold(None)
    released.unlink()
    assert probe.run_burnin(0, "full").ok  # no hold: released right after the verdict
    probe.wait_frees()
    assert released.exists() and "--hold-stdin" not in burnin_child.read_text()


def test_agent_release_hold_waits_for_running_rccl_inits(monkeypatch):
    import time

    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.ops import rccl

    running = [2]

    def inits():
        running[0] = max(0, running[0] - 1)
        return running[0]

    monkeypatch.setattr(rccl, "inits_running", inits)
    monkeypatch.setattr(rccl, "preloads_running", lambda: 0)
    a = NodeAgent(name="h", mode="sim", token="t" * 20)
    a._await_rccl_inits()
    assert running[0] == 0
    monkeypatch.setattr(rccl, "inits_running", lambda: 1)  # an init that never finishes: bounded
    monkeypatch.setattr(NodeAgent, "RELEASE_HOLD_S", 0.05)
    t0 = time.monotonic()
    a._await_rccl_inits()
    assert time.monotonic() - t0 < 1.0


def test_inits_running_is_zero_without_loading_libtk_rccl(monkeypatch):
    from triton_kubernetes_amd.ops import native, rccl

    monkeypatch.delitem(native._cache, "libtk_rccl.so", raising=False)
    assert rccl.inits_running() == 0 and "libtk_rccl.so" not in native._cache


def test_agent_stop_leaves_burnin_children_to_finish_their_release(monkeypatch):
    """A child still freeing the HBM it tested finishes on its own (its stdin closes with the
    agent); stopping the agent waits only for this process's own releases."""
    from triton_kubernetes_amd.node.agent import NodeAgent

    calls = []
    monkeypatch.setattr(probe, "wait_frees", lambda children=True: calls.append(children))
    a = NodeAgent(name="h", mode="sim", devices=[0], token="t" * 20)
    a.stop()
    assert calls == [False]


def test_link_matrix_in_a_child_process(burnin_child, monkeypatch, tmp_path):
    """The agent's gpu_links step measures the peer-read matrix in ``gpu-burnin --p2p-child``
    (beside its RCCL start, as the burn-in): same result form as the in-process matrix."""
    import json
    import sys

    exe = tmp_path / "gpu-burnin"
    exe.write_text(f"""#!{sys.executable}
import json, os, sys
open(os.environ["FAKE_CHILD_ARGV"], "w").write(" ".join(sys.argv[1:]))
print(json.dumps({{"ok": True, "pairs": {{"0-1": 51.5, "1-0": 50.9}}, "peer_access": {{"0-1": True, "1-0": True}},
                  "errors": [], "bytes": 67108864, "method": "kernel-read", "data_errors": {{"1-0": 3}}}}), flush=True)
""")
    got = probe.link_matrix_process([0, 1])
    assert burnin_child.read_text().split() == ["--p2p-child", "--devices", "0,1", "--bytes", str(64 << 20),
                                                "--iters", "3", "--p2p-method", "kernel-read"]
    assert got == {"pairs": {"0-1": 51.5, "1-0": 50.9}, "peer_access": {"0-1": True, "1-0": True}, "errors": [],
                   "bytes": 64 << 20, "method": "kernel-read", "data_errors": {"1-0": 3}}
    from triton_kubernetes_amd.node.labels import link_labels

    verdict = link_labels(got, 0.5, 38.0)
    assert verdict["status"] == "degraded"  # the corrupted pair fails the node, as in process
    exe.write_text(f"#!{sys.executable}\nprint('{{\"ok\": false, \"error\": \"hipSetDevice: invalid device\"}}')\n")
    with pytest.raises(probe.ProbeError, match="invalid device"):
        probe.link_matrix_process([0, 7])


def test_agent_links_step_uses_the_child(monkeypatch):
    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.node.plan import Step

    used = []
    monkeypatch.setattr(probe, "_BURNIN_PROCESS", True)
    monkeypatch.setattr(probe, "link_matrix_process", lambda devs, method: used.append(("child", devs)) or {
        "pairs": {"0-1": 50.0, "1-0": 50.0}, "peer_access": {}, "errors": [], "data_errors": {}})
    monkeypatch.setattr(probe, "link_matrix", lambda devs, method: used.append(("here", devs)))
    a = NodeAgent(name="h", mode="sim", devices=[0, 1], token="t" * 20)
    step = Step("gpu_links", "gpu_links", "", {"min_frac": 0.5, "min_gbps": 38.0, "method": "kernel-read"})
    ctx = {"labels": {}, "capacity": {}, "taints": []}
    out = a._run_step(None, step, ctx)
    assert used == [("child", [0, 1])] and out["status"] == "passed", (used, out)


def test_release_hold_also_waits_for_the_plans_link_matrix(monkeypatch):
    import threading
    import time

    from triton_kubernetes_amd.node.agent import NodeAgent
    from triton_kubernetes_amd.ops import rccl

    monkeypatch.setattr(rccl, "inits_running", lambda: 0)
    monkeypatch.setattr(rccl, "preloads_running", lambda: 0)
    a = NodeAgent(name="h", mode="sim", token="t" * 20)
    a._links_pending = True
    done = threading.Event()
    t = threading.Thread(target=lambda: (a._await_rccl_inits(), done.set()), daemon=True)
    t.start()
    time.sleep(0.2)
    assert not done.is_set()  # still held: the link matrix is yet to be measured
    a._links_pending = False
    assert done.wait(2.0)


def test_preload_exports_and_stub_abi():
    """libtk_rccl exports the device-code preload and its counter; the ABI stub answers
    "nothing to preload" (no RCCL device code behind it)."""
    import ctypes
    import os

    from triton_kubernetes_amd.ops import native

    stub = ctypes.CDLL(os.path.join(native.LIB_DIR, "libtk_rccl_stub.so"))
    assert stub.tkr_preload_device_code(1, (ctypes.c_int * 1)(0)) == 1
    assert stub.tkr_preloads_running() == 0
    out = __import__("subprocess").run(["nm", "-D", os.path.join(native.LIB_DIR, "libtk_rccl.so")],
                                       capture_output=True, text=True).stdout
    assert " T tkr_preload_device_code" in out and " T tkr_preloads_running" in out and " T tkr_inits_running" in out
    assert " T tkr_preload_symbol" in out and " T tkr_elf_kernel_symbol" in out


def _elf_scan(path: str) -> str:
    import ctypes
    import os

    from triton_kubernetes_amd.ops import native

    stub = ctypes.CDLL(os.path.join(native.LIB_DIR, "libtk_rccl_stub.so"))
    stub.tkr_elf_kernel_symbol.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
    buf = ctypes.create_string_buffer(1024)
    n = stub.tkr_elf_kernel_symbol(path.encode(), buf, len(buf))
    assert n == len(buf.value)
    return buf.value.decode()


def test_preload_scan_finds_a_kernel_handle_in_every_librccl_on_this_image():
    """the preload looked up two mangled names only.  /opt/rocm's librccl
    exports them; the librccl torch ships (the one a process that imported torch first has
    loaded) names its kernels ``rcclGenericKernel<...>`` -- there the lookup found nothing
    and the preload silently did nothing.  The scan (tk_elf_scan.h) finds an exported
    device-kernel handle in both, and never a debug variant."""
    import glob
    import os

    import torch

    rocm = os.path.realpath("/opt/rocm/lib/librccl.so.1")
    torch_rccl = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    checked = 0
    for path in (rocm, torch_rccl):
        if not os.path.exists(path):
            continue
        name = _elf_scan(path)
        assert "ncclDevKernelArgsStorage" in name and "Debug" not in name, (path, name)
        out = __import__("subprocess").run(["nm", "-D", "--defined-only", path], capture_output=True,
                                           text=True).stdout
        assert f" {name}" in out  # an exported, defined symbol: dlsym finds it
        checked += 1
    assert checked >= 1
    if os.path.exists(rocm):
        assert _elf_scan(rocm) == "_Z23ncclDevKernel_Generic_124ncclDevKernelArgsStorageILm4096EE"
    if os.path.exists(torch_rccl):
        assert _elf_scan(torch_rccl).startswith("_Z17rcclGenericKernel")


def test_preload_scan_refuses_what_is_not_a_librccl(tmp_path):
    import os

    from triton_kubernetes_amd.ops import native

    assert _elf_scan(os.path.join(native.LIB_DIR, "libtk_topo.so")) == ""  # an ELF without RCCL kernels
    junk = tmp_path / "junk.so"
    junk.write_bytes(b"\x7fELF" + b"\x02" + b"\x00" * 200)  # a truncated header
    assert _elf_scan(str(junk)) == ""
    assert _elf_scan(str(tmp_path / "missing.so")) == ""
    (tmp_path / "empty.so").write_bytes(b"")
    assert _elf_scan(str(tmp_path / "empty.so")) == ""


def test_eight_gpus_burn_in_concurrently_and_release_together(burnin_child, monkeypatch, tmp_path):
    """An 8-GPU node: one child per GPU at once (the agent's pool), each told its own device,
    each holding what it tested until the release hold lets go -- then all release."""
    import concurrent.futures as cf
    import json
    import sys
    import threading
    import time

    exe = tmp_path / "gpu-burnin"
    exe.write_text(f"""#!{sys.executable}
import json, os, sys, time
dev = sys.argv[sys.argv.index("--device") + 1]
doc = json.loads(os.environ["FAKE_CHILD_DOC"]); doc["device"] = int(dev)
open(os.path.join({str(tmp_path)!r}, "started-" + dev), "w").write(str(time.monotonic()))
print(json.dumps(doc), flush=True)
if "--hold-stdin" in sys.argv:
    sys.stdin.read()
open(os.path.join({str(tmp_path)!r}, "released-" + dev), "w").write(str(time.monotonic()))
""")
    monkeypatch.setenv("FAKE_CHILD_DOC", json.dumps(CHILD_OK))
    go = threading.Event()
    probe.set_release_hold(go.wait)
    try:
        with cf.ThreadPoolExecutor(8) as pool:
            results = list(pool.map(lambda d: probe.run_burnin(d, "full"), range(8)))
        assert all(r.ok for r in results) and sorted(r.device.index for r in results) == list(range(8))
        assert len(list(tmp_path.glob("started-*"))) == 8
        time.sleep(0.2)
        assert not list(tmp_path.glob("released-*"))  # every GPU's HBM still held
        go.set()
        probe.wait_frees()
        assert sorted(p.name for p in tmp_path.glob("released-*")) == [f"released-{d}" for d in range(8)]
    finally:
        go.set()
        probe.set_release_hold(None)


def test_gpu_burnin_all_runs_the_same_levels_as_the_agent():
    """``gpu-burnin --all`` (SSH / Terraform nodes) hard-codes its levels; the agent path takes
    them from ``probe.LEVELS``.  Both must burn in the same way: the constants in the C++
    source are read here and compared."""
    import os
    import re

    from triton_kubernetes_amd.ops import probe

    src = open(os.path.join(os.path.dirname(probe.__file__), "csrc", "tk_gpu_probe.hip"), encoding="utf-8").read()
    body = src[src.index('const bool full = !strcmp(level, "full");'):]
    body = body[:6000]  # the --all path: levels, then the per-GPU screens
    hbm = re.search(r"hbm_bytes = full \? \((\d+)ull << (\d+)\) : \((\d+)ull << (\d+)\)", body)
    mfma = re.search(r"mfma_iters = full \? (\d+) : (\d+);", body)
    hbm_iters = re.search(r"tkp_hbm_bandwidth\(d, hbm_bytes, (\d+),", body)
    passes = re.search(r"tkp_memtest_span\(d, mt_bytes, [^,]+, [^,]+, full \? (\d+) : (\d+)", body)
    assert hbm and mfma and hbm_iters and passes
    for level, k in (("full", 0), ("quick", 1)):
        hb, hi, mi, mt_bytes, mp = probe.LEVELS[level]
        assert hb == int(hbm.group(1 + 2 * k)) << int(hbm.group(2 + 2 * k)), level
        assert hi == int(hbm_iters.group(1)), level
        assert mi == int(mfma.group(1 + k)), level
        assert mp == int(passes.group(1 + k)), level


def _matrix(n=4, gbps=50.0, slow=None, corrupt=None, errors=()):
    pairs = {f"{i}-{j}": gbps for i in range(n) for j in range(n) if i != j}
    for p, v in (slow or {}).items():
        pairs[p] = v
    return {"pairs": pairs, "peer_access": {p: True for p in pairs}, "errors": list(errors),
            "data_errors": dict(corrupt or {}), "method": "kernel-read", "bytes": 64 << 20}


def test_a_link_that_read_slow_once_is_measured_again():
    """The burn-in's rule for throughput gates applies to the xGMI link matrix: a pair below
    half the node's median is measured again (best of up to 3) before it fails the node --
    the first 8-GPU run must not fail on one noisy read."""
    from triton_kubernetes_amd.node.labels import best_link_verdict

    runs = iter([_matrix(slow={"2-3": 12.0}), _matrix()])
    got = best_link_verdict(lambda: next(runs), 0.5, 0.0)
    assert got["status"] == "passed" and got["remeasured"] == 1 and got["matrix"]["pairs"]["2-3"] == 50.0


def test_a_link_slow_every_time_still_fails_and_wrong_data_is_never_retried():
    from triton_kubernetes_amd.node.labels import best_link_verdict

    calls = []

    def slow():
        calls.append(1)
        return _matrix(slow={"1-3": 10.0})

    got = best_link_verdict(slow, 0.5, 0.0)
    assert got["status"] == "degraded" and got["degraded"] == ["1-3"] and got["remeasured"] == 2 and len(calls) == 3
    calls.clear()

    def corrupt():
        calls.append(1)
        return _matrix(corrupt={"0-1": 7})

    got = best_link_verdict(corrupt, 0.5, 0.0)
    assert got["status"] == "degraded" and got["corrupt"] == ["0-1"] and len(calls) == 1
    calls.clear()

    def broken():
        calls.append(1)
        return _matrix(errors=["2->3: peer read failed"])

    got = best_link_verdict(broken, 0.5, 0.0)
    assert got["status"] == "error" and len(calls) == 1
    # a pair that corrupted data in a retry stays corrupt after a faster read
    runs = iter([_matrix(slow={"1-2": 10.0}), _matrix(corrupt={"1-2": 1})])
    got = best_link_verdict(lambda: next(runs), 0.5, 0.0)
    assert got["status"] == "degraded" and got["corrupt"] == ["1-2"] and got["remeasured"] == 1
