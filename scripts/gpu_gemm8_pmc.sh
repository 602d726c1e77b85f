#!/bin/bash
# GPU-box: counter passes over the staggered GEMM schedule (TKG_SCHED=1), each pass its own run.
# TK_GEMM_DTYPE=fp8 profiles the fp8 screen; PMC_OUT names the output directory.
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="${PMC_OUT:-pmc8}"
mkdir -p "$R/gpurun_out/$OUT"
cd /tmp && export TMPDIR=/tmp
export TKG_SCHED=1
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/$OUT/$name" -o gemm -- python3 "$R/scripts/gemm_profile.py" > "$R/gpurun_out/$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc" >> "$R/gpurun_out/$OUT/rc.log"; return $rc
}
pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE && \
pass wait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_BUSY_CYCLES && \
pass lds SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM && \
pass mem FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE
