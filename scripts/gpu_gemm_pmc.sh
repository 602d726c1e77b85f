#!/bin/bash
# GPU-box: rocprofv3 counter passes over the GEMM screen (each pass its own run).
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmc/$name" -o gemm -- python3 "$R/scripts/gemm_profile.py" > "$R/gpurun_out/pmc/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc" >> "$R/gpurun_out/pmc/rc.log"; return $rc
}
pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE && \
pass mem FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE
