#!/bin/bash
# GPU-box: CPU accounting per bring-up step (cgroup throttling, PSI, process CPU time).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
(cat /proc/self/cgroup; nproc; cat /proc/pressure/cpu; cat /sys/fs/cgroup/cpu.max; cat /sys/fs/cgroup/cpu/cpu.cfs_quota_us) > gpurun_out/exp9_env.txt 2>&1
TK_BENCH_STEP_WATCHDOG=0.09 timeout -k 10 240 python bench.py --steps 30 --warmup 2 --report gpurun_out/exp9.json > gpurun_out/exp9.log 2>&1
echo "exp9 rc=$?" >> gpurun_out/exp9_rc.log
