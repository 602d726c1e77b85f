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
