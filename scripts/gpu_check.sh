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
if [ "$MODE" = coldinit ]; then
  step rccl_cold_init 600 python scripts/diag/rccl_cold_init.py ${COLD_VARIANTS:-}
fi
if [ "$MODE" = runtime ]; then
  # cold bench on the system ROCm runtime vs the PyTorch-ROCm bundled runtime, alternating
  step bench_sys1 300 python bench.py --steps 5 --warmup 1 --warm-steps 0
  TK_HIP_RUNTIME=torch step bench_torch1 300 python bench.py --steps 5 --warmup 1 --warm-steps 0
  step bench_sys2 300 python bench.py --steps 5 --warmup 1 --warm-steps 0
  TK_HIP_RUNTIME=torch step bench_torch2 300 python bench.py --steps 5 --warmup 1 --warm-steps 0
fi
if [ "$MODE" = kload ]; then
  step rccl_kernel_load 300 python scripts/diag/rccl_kernel_load.py
fi
if [ "$MODE" = full ]; then
  step bench_full 600 python bench.py --steps 3 --warmup 1 --warm-steps 0 --burnin full
  TK_HIP_RUNTIME=system step bench_system 300 python bench.py --steps 5 --warmup 1 --warm-steps 0
fi
if [ "$MODE" = steps ]; then
  step bench_steps 300 python bench.py --steps 3 --warmup 1 --warm-steps 0
  step bench_steps_full 600 python bench.py --steps 2 --warmup 1 --warm-steps 0 --burnin full
fi
if [ "$MODE" = slim ]; then
  # single-target RCCL (ops/rccl_slim.py): GPU test, then the cold bench with / without it, alternating
  step slim_test 300 python -u -m pytest tests/test_gpu_probes.py -k slim -x -v -s --timeout 120 --timeout-method thread
  step bench_slim1 300 python bench.py --steps 5 --warmup 1 --report gpurun_out/bench_slim1.json
  step bench_noslim1 300 python bench.py --steps 5 --warmup 1 --warm-steps 0 --rccl-slim off --report gpurun_out/bench_noslim1.json
  step bench_slim2 300 python bench.py --steps 5 --warmup 1 --warm-steps 0 --report gpurun_out/bench_slim2.json
  step bench_noslim2 300 python bench.py --steps 5 --warmup 1 --warm-steps 0 --rccl-slim off --report gpurun_out/bench_noslim2.json
fi
if [ "$MODE" = shslim ]; then
  # shell form (SSH / Terraform nodes): e2e scripts with the rccl_slim step, then rccl-ready's
  # process wall on /opt/rocm's full bundle vs the shell-made single-target copy, alternating
  step shslim_tests 600 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_probes.py -k "rendered_shell or terraform_mi355x or slim" -x -v -s --timeout 280 --timeout-method thread
  python -c "from triton_kubernetes_amd.terraform.scripts import RCCL_SLIM_FN as f; print(f)" > /tmp/tk-slim-fn.sh
  step shslim_prep 300 bash -c '. /tmp/tk-slim-fn.sh; tk_rccl_slim /tmp/tk-shslim /opt/rocm'
  step shslim_cold_init 600 python scripts/diag/rccl_cold_init.py system shslim system2 shslim2
fi
if [ "$MODE" = span ]; then
  step memtest_span 300 python scripts/diag/memtest_span_chunks.py
fi
