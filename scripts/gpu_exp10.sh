#!/bin/bash
# GPU-box: fd-table presizing on/off (RCU-synchronized fd table resizes as the stall source?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 30 --warmup 2 --report gpurun_out/exp10_$name.json > gpurun_out/exp10_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> gpurun_out/exp10.log
  return $rc
}
run off1 TK_FD_TABLE=0 && run on1 TK_FD_TABLE=16384 && run off2 TK_FD_TABLE=0 && run on2 TK_FD_TABLE=16384
