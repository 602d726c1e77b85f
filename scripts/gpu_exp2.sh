#!/bin/bash
# GPU-box: RCCL init/teardown variants (incl. rocm_smi pre-init, abort-teardown).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 1000 python scripts/rccl_init_breakdown.py > gpurun_out/rccl_init_breakdown2.jsonl 2> gpurun_out/rccl_init_breakdown2.err
echo "init_breakdown rc=$?" >> gpurun_out/exp2.log
