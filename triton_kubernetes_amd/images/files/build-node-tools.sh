#!/bin/bash
# Build the MI355X node tools for gfx950 from /opt/triton-kubernetes/src into
# /opt/triton-kubernetes/bin (same flags as triton_kubernetes_amd/ops/build.py).
set -euo pipefail
S=${TK_SRC:-/opt/triton-kubernetes/src}
T=${TK_BIN:-/opt/triton-kubernetes/bin}
ROCM=${ROCM_PATH:-/opt/rocm}
HIPCC=$ROCM/bin/hipcc
HIP_FLAGS=(-O3 -std=c++17 --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value)
mkdir -p "$T"
"$HIPCC" "${HIP_FLAGS[@]}" -mllvm -amdgpu-mfma-vgpr-form -DTK_PROBE_MAIN "$S/tk_gpu_probe.hip" "$S/tk_gemm_screen.hip" -o "$T/gpu-burnin" -Wl,-rpath,"$ROCM/lib" &
"$HIPCC" "${HIP_FLAGS[@]}" -DTK_RCCL_MAIN "$S/tk_rccl_probe.hip" -o "$T/rccl-ready" -L"$ROCM/lib" -lrccl -Wl,-rpath,"$ROCM/lib" &
g++ -O2 -std=c++17 -DTK_TOPO_MAIN -DTK_TOPO_AMDSMI -I"$ROCM/include" "$S/tk_topo.cpp" -o "$T/amdgpu-topo-labeller" -L"$ROCM/lib" -lamd_smi -Wl,-rpath,"$ROCM/lib" &
rc=0
for job in $(jobs -p); do wait "$job" || rc=$?; done
[ "$rc" = 0 ] || { echo "node tool build failed" >&2; exit "$rc"; }
"$T/amdgpu-topo-labeller" --labels
