#!/bin/bash
# GPU-box: Python stacks of every thread when a bring-up step overruns 80 ms.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
TK_BENCH_STEP_WATCHDOG=0.08 TKP_TRACE_MS=2 timeout -k 10 240 python bench.py --steps 40 --warmup 2 --report gpurun_out/exp7.json > gpurun_out/exp7.log 2>&1
echo "exp7 rc=$?" >> gpurun_out/exp7_rc.log
