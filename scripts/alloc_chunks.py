"""GPU box: the full memtest's allocation time by chunk size, on a card the driver has
finished clearing.  For each chunk size: wait for this GPU's VRAM to settle to its clean
level (ops/hbm.py), run ``alloc_probe fresh <chunk GiB>`` (scripts/alloc_probe.hip: every free
byte but 8 GiB in chunks, touched, freed) in a fresh process, then time how long the driver
takes to clear what it released.  One JSON line per run to stdout."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from triton_kubernetes_amd.ops import hbm  # noqa: E402

p = torch.cuda.get_device_properties(0)
cards = hbm.cards_for_pci([(p.pci_domain_id, p.pci_bus_id, p.pci_device_id)])
floor = None
for chunk in [int(c) for c in (sys.argv[1:] or ["1", "16", "4", "2", "1", "16"])]:
    s = hbm.settle(cards=cards, floor=floor, quiet_s=3.0)
    floor = s["floor"] if floor is None else min(floor, s["floor"])
    t0 = time.monotonic()
    out = subprocess.run(["timeout", "-k", "10", "120", os.path.join(ROOT, "scripts/native/alloc_probe"), "fresh",
                          str(chunk)], capture_output=True, text=True)
    wall = (time.monotonic() - t0) * 1e3
    if out.returncode != 0:
        print(json.dumps({"chunk_gib": chunk, "rc": out.returncode, "stderr": out.stderr[-500:]}), flush=True)
        sys.exit(out.returncode)
    doc = json.loads(out.stdout.strip().splitlines()[-1])
    per = doc.pop("per_chunk_ms")
    after = hbm.settle(cards=cards, floor=floor, quiet_s=3.0)
    doc.update(process_wall_ms=round(wall, 1), settled_before_s=s["waited_s"], clean_before=s["reached_floor"],
               per_chunk_ms_max=max(per), per_chunk_ms_median=sorted(per)[len(per) // 2],
               release_clear_s=after["waited_s"], released_gib=after["released_gib"])
    print(json.dumps(doc), flush=True)
