#!/bin/bash
# Round 6's native host code under ASan/UBSan on the MI355X (device code not instrumented):
# the gate path of rccl-ready (--cluster: tkr_gate_begin_ex -> init_body with the footprint
# measurement, proc_vram's KFD lookup and its device-wide fallback) and the preload's symbol
# lookup (--preload).  (.gpurunignore lists the -asan-r6 binary: drop that line to send it with a
# gpurun call.)  Build (CPU container):
#   hipcc -O1 -g -std=c++17 --offload-arch=gfx950 -DTK_RCCL_MAIN -Xarch_host -fsanitize=address \
#     -Xarch_host -fsanitize=undefined -fno-gpu-sanitize ops/csrc/tk_rccl_probe.hip \
#     -o scripts/native/rccl-ready-asan-r6 -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
B=scripts/native/rccl-ready-asan-r6
timeout -k 10 120 $B --cluster --world 1 --ngpus 1 --uid-out --max-mib 64 --iters 3 \
    > gpurun_out/r6/asan_rccl_gate.log 2>&1 \
  && timeout -k 10 120 $B --ngpus 1 --iters 3 --max-mib 8 --preload > gpurun_out/r6/asan_rccl_preload.log 2>&1
rc=$?
echo "host_asan_r6 rc=$rc"
exit $rc
