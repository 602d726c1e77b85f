#!/bin/bash
# The driver's multi-rank launch rehearsed on a one-GPU box: torchrun with N ranks, each rank
# owning a 1-GPU agent (TK_BENCH_ASSUME_MASKED=1), all sharing GPU 0.  The cluster RCCL gate
# is off (ranks of one communicator cannot share a GPU); everything else -- gloo control
# plane, N agents, real burn-ins on the GPU, N-worker create and readiness -- runs.
# Not a scaling measurement: N agents contend for one GPU.  The burn-in is `quick` by default
# (REHEARSE_BURNIN): N full spans cannot each hold every free byte of the one shared card.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in ${REHEARSE_RANKS:-2 4}; do
  TK_BENCH_ASSUME_MASKED=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus "$n" --steps 3 --warmup 1 \
    --warm-steps 0 --no-rccl-gate --burnin "${REHEARSE_BURNIN:-quick}" > "gpurun_out/rehearse_masked_$n.jsonl" 2> "gpurun_out/rehearse_masked_$n.err" || exit $?
  echo "ranks=$n rc=0"
done
