"""`gpu-burnin`'s command line (ops/csrc/tk_gpu_probe.hip:main), checked on the CPU: every
option and value is read before the first HIP call, so a refusal needs no GPU.

A threshold that does not parse used to read as 0 (``atof``), which switched its check
off; an unknown option or level was ignored.  Both are now a usage error (exit 64) with
one JSON line, the form the node scripts and ops/probe.py read.
"""

import json
import subprocess

import pytest

from triton_kubernetes_amd.ops.native import NativeUnavailable, executable


@pytest.fixture(scope="module")
def burnin():
    try:
        return executable("gpu-burnin")
    except NativeUnavailable as exc:
        pytest.skip(f"gpu-burnin not buildable here: {exc}")


def _run(exe, args):
    return subprocess.run([exe] + args, capture_output=True, text=True, timeout=60)


@pytest.mark.parametrize("args,opt", [
    (["--level", "bogus"], "--level"), (["--level", "off"], "--level"), (["--level"], "--level"),
    (["--min-link-gbps", "abc"], "--min-link-gbps"), (["--min-link-gbps", "-1"], "--min-link-gbps"),
    (["--min-link-frac", "nan"], "--min-link-frac"), (["--min-read-gbps", "inf"], "--min-read-gbps"),
    (["--min-bf16-tflops", "1e3x"], "--min-bf16-tflops"), (["--device", "-1"], "--device"),
    (["--device", "99999999999"], "--device"), (["--span-chunk", "0"], "--span-chunk"),
    (["--span-passes", "0"], "--span-passes"), (["--span-bytes", "1G"], "--span-bytes"),
    (["--hold-max-ms", "99999999999"], "--hold-max-ms"), (["--compute-partition", "SPX"], "--compute-partition"),
    (["--memory-partition", "nps8"], "--memory-partition"), (["--p2p-method", "dma"], "--p2p-method"),
    (["--all", "--frobnicate"], "--frobnicate"), (["--labels"], "--labels"),
])
def test_bad_options_are_usage_errors(burnin, args, opt):
    run = _run(burnin, args)
    assert run.returncode == 64, (run.returncode, run.stdout, run.stderr)
    doc = json.loads(run.stdout)
    assert doc["ok"] is False and doc["error"].startswith("usage:") and f"'{opt}'" in doc["error"]


@pytest.mark.parametrize("args", [
    ["--all", "--level", "quick", "--compute-partition", "cpx", "--memory-partition", "nps2", "--labels", "/dev/null"],
    ["--all", "--level", "full", "--compute-partition", "spx", "--memory-partition", "nps1"],
    ["--p2p", "--min-link-frac", "0.5", "--min-link-gbps", "38.0", "--labels", "/dev/null"],
    ["--p2p", "--p2p-method", "sdma-copy", "--min-link-gbps", "0"],
    ["--memtest-span", "--device", "0", "--span-bytes", "0", "--span-headroom", "4294967296", "--span-passes", "3",
     "--span-chunk", "17179869184", "--hold-stdin", "--hold-max-ms", "30000"],
    ["--device", "0", "--level", "quick", "--min-read-gbps", "3780", "--min-gemm-fp8-tflops", "1500.5"],
])
def test_what_the_callers_pass_is_accepted(burnin, args):
    """The command lines of node/plan.py, the install script and ops/probe.py parse; on this
    CPU-only container the run then stops at the first HIP call (exit 2), not at the parser."""
    run = _run(burnin, args)
    assert run.returncode != 64, run.stdout
    if run.returncode == 2:
        assert "usage:" not in run.stdout


# ---- rccl-ready (ops/csrc/tk_rccl_probe.hip:main): the same rule, errors on stderr ----------

@pytest.fixture(scope="module")
def rccl_ready():
    try:
        return executable("rccl-ready")
    except NativeUnavailable as exc:
        pytest.skip(f"rccl-ready not buildable here: {exc}")


@pytest.mark.parametrize("args,opt", [
    (["--min-busbw", "abc"], "--min-busbw"), (["--min-busbw", "-3"], "--min-busbw"), (["--ngpus", "0"], "--ngpus"),
    (["--ngpus", "2x"], "--ngpus"), (["--iters", "0"], "--iters"), (["--timeout-s", "0"], "--timeout-s"),
    (["--timeout-s", "inf"], "--timeout-s"), (["--world", "0"], "--world"), (["--rank-base", "-8"], "--rank-base"),
    (["--max-mib", "0"], "--max-mib"), (["--uid"], "--uid"), (["--cluster", "--bogus"], "--bogus"),
])
def test_rccl_ready_bad_options_are_usage_errors(rccl_ready, args, opt):
    run = _run(rccl_ready, args)
    assert run.returncode == 64, (run.returncode, run.stdout, run.stderr)
    doc = json.loads(run.stderr)
    assert doc["error"].startswith("usage:") and f"'{opt}'" in doc["error"]


def test_rccl_ready_accepts_the_gate_scripts_command_line(rccl_ready):
    """The command line readiness/process_gate.py writes for both ends of the SSH gate
    parses; here the run then stops at the first HIP call (exit 3, no devices)."""
    import shlex

    from triton_kubernetes_amd.readiness.process_gate import gate_script

    for uid in (None, "ab" * 128):
        script = gate_script("/opt/tk", 16, 8 if uid else 0, 8, [1 << 20, 64 << 20], 5, uid, min_busbw=12.5)
        args = shlex.split(script.split('"$t" ', 1)[1].split(" </dev/null", 1)[0])
        run = _run(rccl_ready, args + ["--bf16", "--preload"])
        assert run.returncode == 3 and "no HIP devices" in run.stderr, (args, run.stderr)
