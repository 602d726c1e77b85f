#!/bin/bash
# GPU-box: staggered wave-group GEMM (TKG_STAGGER=1) vs the single-group pipeline: tests + throughput.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TKG_STAGGER=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_gemm.py -m gpu -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gemm_stagger_tests.log 2>&1 && \
timeout -k 10 200 python scripts/gemm_ab.py base=triton_kubernetes_amd/ops/lib/libtk_gemm.so > gpurun_out/gemm_stagger_base.json 2>&1 && \
TKG_STAGGER=1 timeout -k 10 200 python scripts/gemm_ab.py stagger=triton_kubernetes_amd/ops/lib/libtk_gemm.so > gpurun_out/gemm_stagger_on.json 2>&1
