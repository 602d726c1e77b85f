"""GPU box: which DRM card is this process's GPU, and does mem_info_vram_used show a
release backlog?  Allocates 64 GiB with torch, frees it, samples every card."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from triton_kubernetes_amd.ops import hbm  # noqa: E402


def snap(tag):
    print(json.dumps({"t": round(time.monotonic() - T0, 3), "tag": tag,
                      "gib": {k: round(v / 2**30, 1) for k, v in hbm.vram_used().items()}}), flush=True)


T0 = time.monotonic()
p = torch.cuda.get_device_properties(0)
print(json.dumps({"domain": p.pci_domain_id, "bus": p.pci_bus_id, "dev": p.pci_device_id,
                  "mapped": hbm.cards_for_pci([(p.pci_domain_id, p.pci_bus_id, p.pci_device_id)]),
                  "free_total": [x / 2**30 for x in torch.cuda.mem_get_info()],
                  "cards": {c: os.path.basename(os.path.realpath(f"/sys/class/drm/{c}/device"))
                            for c in sorted(hbm.vram_used())}}), flush=True)
snap("start")
xs = [torch.empty(16 << 30, dtype=torch.uint8, device="cuda") for _ in range(4)]
for x in xs:
    x.fill_(1)
torch.cuda.synchronize()
snap("allocated64")
del xs
torch.cuda.empty_cache()
torch.cuda.synchronize()
snap("freed")
for i in range(40):
    time.sleep(0.05)
    snap(f"after{i}")
