#!/bin/bash
# GPU-box: are the occasional ~120 ms bring-up stalls Python garbage collections?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
for g in default off default off; do
  mode=$g; [ "$g" = default ] && mode=""
  TK_BENCH_GC=$mode timeout -k 10 240 python bench.py --steps 20 --warmup 2 --report gpurun_out/exp5_${g}_$RANDOM.json > gpurun_out/exp5_$g.log 2>&1
  rc=$?; echo "gc=$g rc=$rc" >> gpurun_out/exp5.log
  case $rc in 0) ;; *) exit $rc;; esac
done
