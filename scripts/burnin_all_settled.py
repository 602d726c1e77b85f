"""GPU box: ``gpu-burnin --all --level <level>`` (the SSH / Terraform path) on a card the
driver has finished clearing, then once more right after (no wait): per-phase times from the
verdict, the process wall, and the settle before each run.  One JSON line per run."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from triton_kubernetes_amd.ops import hbm  # noqa: E402

level = sys.argv[1] if len(sys.argv) > 1 else "full"
p = torch.cuda.get_device_properties(0)
cards = hbm.cards_for_pci([(p.pci_domain_id, p.pci_bus_id, p.pci_device_id)])
floor = None
# runs: (settle first, extra env)
RUNS = [(True, {}), (False, {}), (True, {"TK_BURNIN_EXIT": "normal"}), (True, {})]
for run, (wait, extra) in enumerate(RUNS):
    s = hbm.settle(cards=cards, floor=floor, quiet_s=3.0) if wait else {"waited_s": 0.0, "reached_floor": None}
    if wait:
        floor = s["floor"] if floor is None else min(floor, s["floor"])
    t0 = time.monotonic()
    out = subprocess.run(["timeout", "-k", "10", "120", os.path.join(ROOT, "triton_kubernetes_amd/ops/lib/gpu-burnin"),
                          "--all", "--level", level], capture_output=True, text=True,
                         env=dict(os.environ, TK_BURNIN_TRACE="1", **extra))
    wall = (time.monotonic() - t0) * 1e3
    doc = json.loads(out.stdout.strip().splitlines()[-1]) if out.stdout.strip() else {}
    g = (doc.get("gpus") or [{}])[0]
    main_ms = [ln for ln in out.stderr.splitlines() if "ms to the verdict" in ln]
    print(json.dumps({"run": run, "settled_first": wait, "env": extra, "main_trace": main_ms, "settle_s": s["waited_s"], "clean": s.get("reached_floor"),
                      "rc": out.returncode, "wall_ms": round(wall, 1), "ok": doc.get("ok"),
                      "memtest_gib": round(g.get("memtest_bytes", 0) / 2**30, 1), "phase_ms": g.get("phase_ms")}),
          flush=True)
    if out.returncode != 0:
        sys.exit(out.returncode)
