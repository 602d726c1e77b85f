#!/bin/bash
# GPU-box: where the GEMM's waves wait (second set of counter passes).
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmc2"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmc2/$name" -o gemm -- python3 "$R/scripts/gemm_profile.py" > "$R/gpurun_out/pmc2/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc" >> "$R/gpurun_out/pmc2/rc.log"; return $rc
}
pass wait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_BUSY_CYCLES && \
pass lds SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM
