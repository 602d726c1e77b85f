set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export PYTHONPATH="$GRAFT_REPO_ROOT"
O=gpurun_out/kernels_head.jsonl; : > $O
run() { timeout -k 10 "$1" "${@:2}" >> $O 2>> gpurun_out/kernels_head.err || exit $?; echo >> $O; }
run 120 python -m triton_kubernetes_amd.ops.cli hbm --gib 8
run 120 python -m triton_kubernetes_amd.ops.cli mfma --dtype bf16
run 120 python -m triton_kubernetes_amd.ops.cli mfma --dtype fp8
run 180 python -m triton_kubernetes_amd.ops.cli gemm --size 8192 --dtype bf16
run 180 python -m triton_kubernetes_amd.ops.cli gemm --size 8192 --dtype fp8
echo done
