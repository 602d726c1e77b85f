#!/bin/bash
# GPU-box: does deferring communicator teardowns to quiet periods remove the one-per-run stall?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
for q in 0 1000 0 1000; do
  TK_TEARDOWN_QUIET_MS=$q timeout -k 10 240 python bench.py --steps 20 --warmup 2 --report gpurun_out/exp3_q${q}_$RANDOM.json > gpurun_out/exp3_q$q.log 2>&1
  rc=$?; echo "quiet=$q rc=$rc" >> gpurun_out/exp3.log
  case $rc in 0) ;; *) exit $rc;; esac
done
