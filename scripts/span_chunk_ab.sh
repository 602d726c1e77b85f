#!/bin/bash
# Full-burnin bench with the agent's span child at different chunk sizes (TK_SPAN_CHUNK_GIB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for gib in ${@:-16 4 1}; do
  TK_SPAN_CHUNK_GIB=$gib timeout -k 10 400 python bench.py --steps 3 --warmup 1 --burnin full --warm-steps 0 \
    --report gpurun_out/bench_full_chunk${gib}.json > gpurun_out/bench_full_chunk${gib}.log 2>&1 || exit $?
  echo "chunk ${gib} GiB done"
done
