#!/bin/bash
# GPU-box: does the burn-in slow the overlapped RCCL init?  burn-in off / low-priority
# streams (default) / normal-priority streams, 20 steps each, twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 2 ${BENCH_ARGS} --report gpurun_out/exp12_$name.json > gpurun_out/exp12_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> gpurun_out/exp12.log
  return $rc
}
BENCH_ARGS="--burnin off" run off1 && run low1 && run normal1 TKP_STREAM_PRIORITY=normal && \
BENCH_ARGS="--burnin off" run off2 && run low2 && run normal2 TKP_STREAM_PRIORITY=normal
