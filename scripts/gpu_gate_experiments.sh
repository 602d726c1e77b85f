#!/bin/bash
# GPU-box: gate tests, RCCL init breakdown, rocprof of the bench without and with the
# pipelined gate (the latter with a Python stack watchdog; last, since it may hang).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
LOG=gpurun_out/exp.log
stop() { case "$1" in 0|1) return 1;; esac; return 0; }
timeout -k 10 300 python -m pytest tests/test_gpu_probes.py -k "gate or rccl" -q -s -p no:cacheprovider > gpurun_out/gate_tests.log 2>&1
rc=$?; echo "gate_tests rc=$rc" >> $LOG; if stop $rc; then exit $rc; fi
timeout -k 10 900 python scripts/rccl_init_breakdown.py > gpurun_out/rccl_init_breakdown.jsonl 2> gpurun_out/rccl_init_breakdown.err
rc=$?; echo "init_breakdown rc=$rc" >> $LOG; if stop $rc; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_nopipe" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-gate-pipeline > "$GRAFT_REPO_ROOT/gpurun_out/prof_nopipe.log" 2>&1
rc=$?; echo "prof_nopipe rc=$rc" >> "$GRAFT_REPO_ROOT/$LOG"; if stop $rc; then exit $rc; fi
TK_BENCH_WATCHDOG=40 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_pipe" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_pipe.log" 2>&1
echo "prof_pipe rc=$?" >> "$GRAFT_REPO_ROOT/$LOG"
