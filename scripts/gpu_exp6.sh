#!/bin/bash
# GPU-box: where do the occasional ~150 ms burn-in stalls go?  Slow-call trace of the
# probe's runtime calls (TKP_TRACE_MS) + per-probe spans, with the pipelined gate on
# and off, and with the scratch cache on.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
run() {  # name, extra env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 2 --report gpurun_out/exp6_$name.json ${BENCH_ARGS} > gpurun_out/exp6_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> gpurun_out/exp6.log
  return $rc
}
run pipe TKP_TRACE_MS=2 && \
BENCH_ARGS=--no-gate-pipeline run nopipe TKP_TRACE_MS=2 && \
run pipe_cache TKP_TRACE_MS=2 TK_PROBE_SCRATCH_CACHE=1 && \
BENCH_ARGS=--no-rccl-gate run nogate TKP_TRACE_MS=2
