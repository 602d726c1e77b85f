#!/bin/bash
# Run every allocation scenario of alloc_probe in its own process (scripts/alloc_probe.hip).
set -o pipefail
OUT="$GRAFT_REPO_ROOT/gpurun_out/alloc_probe.jsonl"
: > "$OUT"
for s in fresh prefree presync untouched fresh; do
  t0=$(date +%s%N)
  timeout -k 10 120 "$GRAFT_REPO_ROOT/scripts/native/alloc_probe" "$s" 16 >> "$OUT" || exit $?
  echo "{\"scenario\": \"$s\", \"process_wall_ms\": $(( ($(date +%s%N) - t0) / 1000000 ))}" >> "$OUT"
done
timeout -k 10 120 "$GRAFT_REPO_ROOT/scripts/native/alloc_probe" fresh 64 >> "$OUT"
