#!/bin/bash
# GPU-box: does keeping the burn-in buffers allocated remove the occasional bring-up stall?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
for c in 1 0 1 0; do
  TK_PROBE_SCRATCH_CACHE=$c timeout -k 10 240 python bench.py --steps 20 --warmup 2 --report gpurun_out/exp4_c${c}_$RANDOM.json > gpurun_out/exp4_c$c.log 2>&1
  rc=$?; echo "cache=$c rc=$rc" >> gpurun_out/exp4.log
  case $rc in 0) ;; *) exit $rc;; esac
done
