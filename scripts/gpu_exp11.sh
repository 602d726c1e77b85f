#!/bin/bash
# GPU-box: GPU tests, then the default bench (fd table presized, resident burn-in arena) twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/exp11_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/exp11.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 240 python bench.py --steps 30 --warmup 2 --report gpurun_out/exp11_b$i.json > gpurun_out/exp11_b$i.log 2>&1
  rc=$?; echo "bench$i rc=$rc" >> gpurun_out/exp11.log; [ $rc -eq 0 ] || exit $rc
done
