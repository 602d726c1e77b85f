#!/bin/bash
# Where a full burn-in's wall-clock goes: kernel time vs HIP runtime calls (allocation,
# frees, synchronisation).  Kernel + HIP-runtime traces only (no counters).
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"
mkdir -p "$ROOT/gpurun_out/prof_burnin"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv \
  -d "$ROOT/gpurun_out/prof_burnin" -o "full_%pid%" -- \
  "$ROOT/triton_kubernetes_amd/ops/lib/gpu-burnin" --device 0 --level "${1:-full}" \
  > "$ROOT/gpurun_out/prof_burnin/burnin.json" 2> "$ROOT/gpurun_out/prof_burnin/burnin.err"
