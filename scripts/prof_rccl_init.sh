#!/bin/bash
# GPU box: where a fresh process's first RCCL communicator init goes, with comgr's cache
# warm (a first run fills it): HIP and HSA API statistics from rocprofv3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH="$GRAFT_REPO_ROOT"
timeout -k 10 120 python3 scripts/rccl_init_once.py > gpurun_out/rccl_init_warmup.json || exit $?
timeout -k 10 120 python3 scripts/rccl_init_once.py > gpurun_out/rccl_init_plain.json || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --hsa-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_rccl_init" -o init -- python3 "$GRAFT_REPO_ROOT/scripts/rccl_init_once.py" > "$GRAFT_REPO_ROOT/gpurun_out/rccl_init_prof.log" 2>&1 || exit $?
cat "$GRAFT_REPO_ROOT"/gpurun_out/rccl_init_warmup.json "$GRAFT_REPO_ROOT"/gpurun_out/rccl_init_plain.json
grep '^{' "$GRAFT_REPO_ROOT/gpurun_out/rccl_init_prof.log" | tail -1
