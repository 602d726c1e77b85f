#!/bin/bash
# GPU-box check: GPU test suite, bench (1 GPU), smoke, burn-in levels timed.
# Every GPU step has its own time limit; the script stops at the first fault.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
LOG="$GRAFT_REPO_ROOT/gpurun_out/check.log"
echo "# mode=${1:-all} $(date -u +%FT%TZ)" >> $LOG  # appended: chained modes keep every step's line
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2  # env assignments before "step" apply to the command
  local t0=$(date +%s%N)
  timeout -k 10 "$secs" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc wall_ms=$(( ($(date +%s%N) - t0) / 1000000 ))" >> $LOG
  echo "$name rc=$rc"
  case $rc in 0) return 0;; *) exit $rc;; esac
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py --steps 5 --warmup 1 --report gpurun_out/bench_report.json
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = burnin ]; then
  step burnin_quick 120 triton_kubernetes_amd/ops/lib/gpu-burnin --all --level quick
  step burnin_full 600 triton_kubernetes_amd/ops/lib/gpu-burnin --all --level full
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  cd /tmp && export TMPDIR=/tmp
  step prof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" -o "bench_%pid%" -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --warm-steps 0
fi
