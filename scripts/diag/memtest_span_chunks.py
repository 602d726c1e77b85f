"""Diagnostic: where the full burn-in's span memtest spends its time (allocation, fill +
verify, release) for three chunk sizes (profiles/round2/memtest_span_chunks.jsonl)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from triton_kubernetes_amd.ops import probe
for chunk in (16 << 30, 64 << 30, 8 << 30):
    t = time.perf_counter()
    r = probe.memtest_span(0, 0, chunk=chunk, headroom=4 << 30, passes=1)
    print(json.dumps(dict(r, chunk_gib=chunk >> 30, wall_ms=round((time.perf_counter() - t) * 1e3, 1))), flush=True)
