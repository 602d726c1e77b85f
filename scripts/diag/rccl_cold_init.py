#!/usr/bin/env python3
"""Diagnostic (not product code): where a COLD node agent spends its first RCCL init.

The cold-create bench (bench.py) starts a fresh agent process per step; its critical
path is the first communicator init in that process (~1.8 s against ~45 ms warm).
Each variant runs in a fresh child process (``--child``) that times, in order:

  import     importing the package's ctypes layers
  dlopen     loading libtk_rccl.so (+ librccl, HIP runtime) and libtk_gpu_probe.so
  hip_init   first HIP call (device count) and a device allocation (scratch arena)
  uid        ncclGetUniqueId
  init1      first 1-rank communicator init (blocking)
  sweep1     first verified all-reduce (1 MiB)
  init2      second init + sweep (the warm cost, for reference)

With ``TK_SAMPLE=1`` the child samples every thread during ``init1`` with
scripts/diag/native/tk_sampler.so and reports the top frames per shared object.
Parent mode runs every variant and writes one JSON line each to stdout.
"""

import collections
import ctypes
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

VARIANTS = {
    "base": {},
    "no_msccl_no_plugin": {"RCCL_MSCCL_ENABLE": "0", "RCCL_MSCCLPP_ENABLE": "0", "NCCL_NET_PLUGIN": "none"},
    "ib_disable": {"NCCL_IB_DISABLE": "1"},
    "all_off": {"RCCL_MSCCL_ENABLE": "0", "RCCL_MSCCLPP_ENABLE": "0", "NCCL_NET_PLUGIN": "none",
                "NCCL_IB_DISABLE": "1"},
    "eager_code_objects": {"HIP_ENABLE_DEFERRED_LOADING": "0"},
    "no_smi": {"RCCL_USE_ROCM_SMI_LIB": "0"},
    "debug_init": {"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "INIT"},
    "sampled": {"TK_SAMPLE": "1"},
    "torch_runtime": {"TK_HIP_RUNTIME": "torch"},
    # comgr's on-disk cache of actions (the compressed-bundle UNBUNDLE among them): the first
    # run fills it, later processes would read the extracted gfx950 code object back
    "comgr_cache_fill": {"AMD_COMGR_CACHE": "1", "AMD_COMGR_CACHE_DIR": "/tmp/tk-comgr-cache"},
    "comgr_cache_hit": {"AMD_COMGR_CACHE": "1", "AMD_COMGR_CACHE_DIR": "/tmp/tk-comgr-cache"},
    "comgr_cache_hit2": {"AMD_COMGR_CACHE": "1", "AMD_COMGR_CACHE_DIR": "/tmp/tk-comgr-cache"},
    "base2": {},
    # ncclCommAbort instead of ncclCommDestroy once the verified sweep has drained the streams
    "teardown_abort": {"TK_TEARDOWN_ABORT": "1"},
    "teardown_abort2": {"TK_TEARDOWN_ABORT": "1"},
    # ops/rccl_slim.py: gfx950-only, uncompressed device code (the parent prepares it first)
    "slim": {"TK_HIP_RUNTIME": "@slim"},
    "slim2": {"TK_HIP_RUNTIME": "@slim"},
    "torch_runtime2": {"TK_HIP_RUNTIME": "torch"},
    "slim_system": {"TK_HIP_RUNTIME": "@slim:/opt/rocm/lib"},
    # the shell form (terraform/scripts.py tk_rccl_slim), prepared by scripts/gpu_check.sh shslim
    "shslim": {"TK_HIP_RUNTIME": "/tmp/tk-shslim/rocm"},
    "shslim2": {"TK_HIP_RUNTIME": "/tmp/tk-shslim/rocm"},
    "system": {"TK_HIP_RUNTIME": "system"},
    "system2": {"TK_HIP_RUNTIME": "system"},
    "torch_runtime_all_off": {"TK_HIP_RUNTIME": "torch", "RCCL_MSCCL_ENABLE": "0", "RCCL_MSCCLPP_ENABLE": "0",
                              "NCCL_NET_PLUGIN": "none"},
}


def child() -> None:
    t = {}
    t0 = time.perf_counter()

    def mark(k):
        nonlocal t0
        now = time.perf_counter()
        t[k] = round((now - t0) * 1e3, 1)
        t0 = now

    from triton_kubernetes_amd.ops import probe, rccl

    mark("import")
    rccl._lib()
    if os.environ.get("TK_TEARDOWN_ABORT") == "1":
        rccl._lib().tkr_set_teardown_abort(1)
    probe._lib()
    mark("dlopen")
    probe.device_count()
    probe.prealloc_scratch(0, "quick")
    mark("hip_init")
    uid = rccl.unique_id()
    mark("uid")
    sampler = None
    if os.environ.get("TK_SAMPLE") == "1":
        sampler = ctypes.CDLL(os.path.join(HERE, "native", "tk_sampler.so"))
        sampler.tks_start.argtypes = [ctypes.c_int, ctypes.c_int]
        sampler.tks_stop.argtypes = [ctypes.c_char_p]
        sampler.tks_start(0, 1000)
        t0 = time.perf_counter()
    g = rccl.GateComm(uid, 1, 0, [0], blocking=True)
    mark("init1")
    out_path = ""
    if sampler is not None:
        out_path = os.path.join(ROOT, "gpurun_out", "cold_init_samples.txt")
        os.makedirs(os.path.dirname(out_path), exist_ok=True)
        sampler.tks_stop(out_path.encode())
        t0 = time.perf_counter()
    res = g.sweep([1 << 20], iters=2, warmup=1, async_teardown=False)
    mark("sweep1")
    g2 = rccl.GateComm(rccl.unique_id(), 1, 0, [0], blocking=True)
    g2.sweep([1 << 20], iters=2, warmup=1, async_teardown=False)
    mark("init2")
    from triton_kubernetes_amd.ops.native import runtime_dir

    doc = {"ms": t, "ok": res.ok, "runtime": runtime_dir(), "rccl_version": rccl.version()}
    if out_path:
        doc["top"] = summarize(out_path)
    print(json.dumps(doc), flush=True)


def summarize(path: str):
    """Per sample: the deepest frame inside a GPU/RCCL library, counted by object!symbol."""
    libs = ("librccl", "libamdhip64", "libhsa-runtime64", "librocm_smi", "libamd_smi", "libibverbs", "libmlx5",
            "libdrm", "libnuma", "libc.so", "ld-linux", "libstdc++")
    leaf = collections.Counter()
    first_lib = collections.Counter()
    total = 0
    for line in open(path, encoding="utf-8"):
        _, _, stack = line.strip().partition(" ")
        frames = stack.split(";") if stack else []
        if not frames or not any(f.startswith(("librccl", "libamdhip64", "libhsa")) for f in frames):
            continue
        total += 1
        leaf[frames[0].split("+")[0]] += 1
        gpu = next((f.split("+")[0] for f in frames if f.startswith(libs[:7])), "other")
        first_lib[gpu] += 1
    return {"samples": total, "leaf": leaf.most_common(15), "first_gpu_lib_frame": first_lib.most_common(25)}


def parent() -> None:
    names = sys.argv[1:] or list(VARIANTS)
    for name in names:
        env = dict(os.environ, **VARIANTS[name])
        if env.get("TK_HIP_RUNTIME", "").startswith("@slim"):
            from triton_kubernetes_amd.ops import native, rccl_slim

            meta = rccl_slim.prepare(env["TK_HIP_RUNTIME"].partition(":")[2] or native._torch_lib_dir())
            print(json.dumps({"slim_prepare": meta}), flush=True)
            env["TK_HIP_RUNTIME"] = meta["dir"]
        t0 = time.perf_counter()
        proc = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True,
                              text=True, timeout=300, check=False)
        wall = round((time.perf_counter() - t0) * 1e3, 1)
        line = next((ln for ln in proc.stdout.splitlines() if ln.startswith("{")), "{}")
        doc = {"variant": name, "rc": proc.returncode, "process_wall_ms": wall, **json.loads(line)}
        if name == "debug_init":
            doc["rccl_init_lines"] = [ln for ln in (proc.stdout + proc.stderr).splitlines()
                                      if "Init" in ln or "init" in ln][-12:]
        if proc.returncode:
            doc["stderr"] = proc.stderr[-1500:]
        print(json.dumps(doc), flush=True)
        if proc.returncode not in (0, 1):
            break  # a crash: stop the GPU work here


if __name__ == "__main__":
    if "--child" in sys.argv:
        child()
    else:
        parent()
