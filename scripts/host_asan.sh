#!/bin/bash
# Host-code sanitizers on the MI355X: rccl-ready and gpu-burnin built with ASan/UBSan on the
# host side only (device code is not instrumented), run against the real GPU.
#   (.gpurunignore lists the two -asan binaries: drop those lines to send them with a gpurun call)
#   build (CPU container): hipcc ... -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined
#                          -fno-gpu-sanitize  -> scripts/native/{rccl-ready,gpu-burnin}-asan
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export TK_BURNIN_EXIT=normal  # the whole exit path runs under the sanitizers (gpu-burnin otherwise leaves with _exit)
B=scripts/native
timeout -k 10 120 $B/rccl-ready-asan --ngpus 1 --iters 3 --max-mib 8 > gpurun_out/asan_rccl_ready.log 2>&1 \
  && timeout -k 10 300 $B/gpu-burnin-asan --device 0 --level quick > gpurun_out/asan_burnin_quick.log 2>&1 \
  && timeout -k 10 300 $B/gpu-burnin-asan --memtest-span --device 0 --span-bytes 34359738368 \
       --span-chunk 1073741824 > gpurun_out/asan_memtest_span.log 2>&1 \
  && timeout -k 10 300 $B/gpu-burnin-asan --burnin-child --device 0 --hbm-bytes 17179869184 --hbm-iters 3 \
       --mfma-iters 2000 --gemm 4096,4096,4096,2 --memtest-bytes 0 --memtest-passes 1 --span-chunk 1073741824 \
       > gpurun_out/asan_burnin_child_full.log 2>&1 \
  && timeout -k 10 120 $B/gpu-burnin-asan --p2p-child --devices 0 > gpurun_out/asan_p2p_child.log 2>&1 \
  && timeout -k 10 120 $B/rccl-ready-asan --ngpus 1 --iters 3 --max-mib 8 --preload \
       > gpurun_out/asan_rccl_ready_preload.log 2>&1 \
  && timeout -k 10 300 $B/gpu-burnin-asan --all --level full > gpurun_out/asan_burnin_all_full.log 2>&1
rc=$?
echo "host_asan rc=$rc"
exit $rc
