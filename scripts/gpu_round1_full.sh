#!/bin/bash
# GPU-box run: all GPU tests, bench (1 GPU) with and without the RCCL gate, smoke, profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
LOG=gpurun_out/run.log
fatal() { case "$1" in 0|1|2) return 1;; esac; return 0; }

timeout -k 10 600 python -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc" >> $LOG; if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 2 --report gpurun_out/bench_report.json > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $LOG; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $LOG; if fatal $rc; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
TK_BENCH_WATCHDOG=60 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log" 2>&1
echo "prof_bench rc=$?" >> "$GRAFT_REPO_ROOT/$LOG"
