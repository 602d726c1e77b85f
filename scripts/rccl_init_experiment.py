#!/usr/bin/env python3
"""Measure RCCL communicator-init cost under environment variants (GPU box).

Each variant runs in its own subprocess (RCCL reads its environment once):
three back-to-back single-rank gates, reporting comm-init ms and total ms.
Output: one JSON line per variant.
"""

import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, time
sys.path.insert(0, %r)
if %r:
    import torch  # noqa: F401  (loads torch's bundled librccl first)
from triton_kubernetes_amd.ops import rccl
out = []
for i in range(3):
    t0 = time.perf_counter()
    r = rccl.sweep_rank(0, 1, rccl.unique_id(), 0, [1 << 20, 64 << 20], iters=5, warmup=2)
    out.append({"init_ms": round(r.init_ms, 1), "total_ms": round((time.perf_counter() - t0) * 1e3, 1), "ok": r.ok})
print(json.dumps(out))
"""

VARIANTS = {
    "baseline": {},
    "debug_warn": {"NCCL_DEBUG": "WARN"},
    "no_msccl": {"RCCL_MSCCL_ENABLE": "0", "RCCL_MSCCLPP_ENABLE": "0"},
    "no_ib_net": {"NCCL_IB_DISABLE": "1", "NCCL_NET_PLUGIN": "none"},
    "few_channels": {"NCCL_MAX_NCHANNELS": "4"},
    "combined": {"NCCL_DEBUG": "WARN", "RCCL_MSCCL_ENABLE": "0", "RCCL_MSCCLPP_ENABLE": "0", "NCCL_IB_DISABLE": "1",
                 "NCCL_NET_PLUGIN": "none"},
}


def main() -> int:
    for torch_first in (False, True):
        for name, env in VARIANTS.items():
            if torch_first and name not in ("baseline", "combined"):
                continue
            e = dict(os.environ)
            e.update(env)
            proc = subprocess.run([sys.executable, "-c", CHILD % (HERE, torch_first)], env=e, capture_output=True,
                                  text=True, timeout=300)
            lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("[")]
            print(json.dumps({"variant": name, "torch_first": torch_first, "rc": proc.returncode,
                              "runs": json.loads(lines[-1]) if lines else None,
                              "stderr": proc.stderr[-300:] if proc.returncode else ""}), flush=True)
            if proc.returncode not in (0, 1):
                return proc.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
