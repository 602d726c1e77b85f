#!/bin/bash
# GPU box: does comgr's cache (AMD_COMGR_CACHE / AMD_COMGR_CACHE_DIR) carry RCCL's unbundled
# gfx950 code object from one process to the next?  rccl-ready's first communicator init,
# in fresh processes: cache off, then cache on (cold dir), then on again (warm dir).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/comgr_cache_ab.jsonl
: > $OUT
R=triton_kubernetes_amd/ops/lib/rccl-ready
CACHE=$(mktemp -d /tmp/tk-comgr-XXXX)
one() {  # one <tag> <env...>
  local tag=$1; shift
  local t0=$(date +%s%N)
  local line
  line=$(env "$@" timeout -k 10 120 $R --ngpus 1 --iters 3 --max-mib 8 2>/dev/null | grep '^{' | tail -1) || exit 1
  echo "{\"tag\": \"$tag\", \"wall_ms\": $(( ($(date +%s%N) - t0) / 1000000 )), \"cache_files\": $(find $CACHE -type f | wc -l), \"cache_mb\": $(du -sm $CACHE | cut -f1), \"out\": $line}" >> $OUT
}
one off AMD_COMGR_CACHE=0
one off2 AMD_COMGR_CACHE=0
one cold AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=$CACHE
one warm AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=$CACHE
one warm2 AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=$CACHE
one default TK_NOTHING=1
cat $OUT
