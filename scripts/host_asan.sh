#!/bin/bash
# Host-code sanitizers on the MI355X: rccl-ready and gpu-burnin built with ASan/UBSan on the
# host side only (device code is not instrumented), run against the real GPU.
#   (.gpurunignore lists ./scripts/bin: drop that line to send the binaries with a gpurun call)
#   build (CPU container): hipcc ... -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined
#                          -fno-gpu-sanitize  -> scripts/bin/{rccl-ready,gpu-burnin}-asan
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export TK_BURNIN_EXIT=normal  # the whole exit path runs under the sanitizers (gpu-burnin otherwise leaves with _exit)
timeout -k 10 120 scripts/bin/rccl-ready-asan --ngpus 1 --iters 3 --max-mib 8 > gpurun_out/asan_rccl_ready.log 2>&1 \
  && timeout -k 10 300 scripts/bin/gpu-burnin-asan --device 0 --level quick > gpurun_out/asan_burnin_quick.log 2>&1 \
  && timeout -k 10 300 scripts/bin/gpu-burnin-asan --memtest-span --device 0 --span-bytes 34359738368 \
       --span-chunk 1073741824 > gpurun_out/asan_memtest_span.log 2>&1
rc=$?
echo "host_asan rc=$rc"
exit $rc
