"""RCCL communicator-init cost on one MI355X: repeated world=1 gate inits, with RCCL's own
INIT debug timing lines captured, under a few environment variants.  Each variant runs in a
fresh child process.  Output: one JSON line per variant (+ raw RCCL timing lines)."""

import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys, time
if os.environ.get("TK_TORCH_FIRST"):
    import torch  # binds librccl.so.1 to torch's bundled RCCL, as in bench.py
if os.environ.get("TK_RSMI_PREINIT"):
    import ctypes
    _rsmi = ctypes.CDLL("librocm_smi64.so.1", mode=ctypes.RTLD_GLOBAL)
    _t = time.perf_counter(); _rc = _rsmi.rsmi_init(ctypes.c_uint64(0))
    print("RSMI_PREINIT rc=%d ms=%.1f" % (_rc, (time.perf_counter() - _t) * 1e3), flush=True)
from triton_kubernetes_amd.ops import rccl
if os.environ.get("TK_TEARDOWN_ABORT"):
    rccl._lib().tkr_set_teardown_abort(1)
out = []
for i in range(int(os.environ.get("TK_N", "5"))):
    g = rccl.GateComm(rccl.unique_id(), 1, 0, [0], blocking=True)
    r = g.sweep([1 << 20], iters=2, warmup=1, async_teardown=False)
    out.append(r.phase_ms)
print("RESULT " + json.dumps(out), flush=True)
'''

VARIANTS = {
    "baseline": {},
    "no_rocm_smi": {"RCCL_USE_ROCM_SMI_LIB": "0"},
    "rsmi_preinit": {"TK_RSMI_PREINIT": "1"},
    "ignore_cpu_affinity": {"NCCL_IGNORE_CPU_AFFINITY": "1"},
    "teardown_abort": {"TK_TEARDOWN_ABORT": "1"},
    "no_msccl_no_plugin": {"RCCL_MSCCL_ENABLE": "0", "RCCL_MSCCLPP_ENABLE": "0", "NCCL_NET_PLUGIN": "none"},
    "ib_off": {"NCCL_IB_DISABLE": "1"},
    "topo_file": {"NCCL_TOPO_FILE": "/tmp/tk_topo.xml"},
}


def run(name, extra, torch_first):
    env = dict(os.environ, PYTHONPATH=HERE, NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT", **extra)
    if torch_first:
        env["TK_TORCH_FIRST"] = "1"
    proc = subprocess.run(["timeout", "-k", "5", "120", sys.executable, "-c", CHILD], capture_output=True, text=True,
                          env=env, cwd=HERE)
    lines = (proc.stdout + proc.stderr).splitlines()
    res = [json.loads(ln[7:]) for ln in lines if ln.startswith("RESULT ")]
    timing = [ln.split("NCCL INFO", 1)[-1].strip() for ln in lines
              if "Init timings" in ln or "Init COMPLETE" in ln or "RSMI_PREINIT" in ln]
    print(json.dumps({"variant": name, "torch_first": torch_first, "rc": proc.returncode,
                      "phases": res[0] if res else None, "rccl_timing": timing[-6:],
                      "tail": [] if res else lines[-15:]}), flush=True)
    return proc.returncode


def main():
    # dump a topology file first (used by the topo_file variant)
    env = dict(os.environ, PYTHONPATH=HERE, NCCL_TOPO_DUMP_FILE="/tmp/tk_topo.xml", TK_N="1")
    subprocess.run(["timeout", "-k", "5", "120", sys.executable, "-c", CHILD], env=env, cwd=HERE,
                   capture_output=True, text=True)
    for torch_first in (True, False):
        for name, extra in VARIANTS.items():
            if run(name, extra, torch_first) in (124, 137, 134, 139):
                return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
