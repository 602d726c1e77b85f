#!/bin/bash
# One cold create with the full burn-in under kernel + HIP-runtime traces (every process:
# the bench and its agents), to see which runtime calls the gate's sweep waits in.
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"
mkdir -p "$ROOT/gpurun_out/prof_bench_full"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv \
  -d "$ROOT/gpurun_out/prof_bench_full" -o "b_%pid%" -- \
  python3 "$ROOT/bench.py" --steps 1 --warmup 1 --burnin full --warm-steps 0 \
  --report "$ROOT/gpurun_out/prof_bench_full/report.json" > "$ROOT/gpurun_out/prof_bench_full/bench.log" 2>&1
