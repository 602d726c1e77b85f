#!/bin/bash
# GPU-box: bring-up stall mitigations, 30 steps each: burn-in scratch cache, quiet-period
# teardown scheduling, both.  Stacks of every thread when a step overruns 90 ms.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
run() {
  local name=$1; shift
  env TK_BENCH_STEP_WATCHDOG=0.09 TKP_TRACE_MS=5 "$@" timeout -k 10 240 python bench.py --steps 30 --warmup 2 --report gpurun_out/exp8_$name.json > gpurun_out/exp8_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> gpurun_out/exp8.log
  return $rc
}
run base && run cache TK_PROBE_SCRATCH_CACHE=1 && run quiet TK_TEARDOWN_QUIET_MS=1000 && \
run both TK_PROBE_SCRATCH_CACHE=1 TK_TEARDOWN_QUIET_MS=1000
