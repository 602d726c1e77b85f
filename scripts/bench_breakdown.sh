#!/bin/bash
# GPU box: where the full burn-in's cold create goes.  The default line, then the same
# without the cluster RCCL gate (no communicator init beside the burn-in), then with the
# opt-in single-target RCCL, the quick level, and (nohold) the burn-in child releasing its HBM
# right after the verdict instead of after the agent's RCCL init.  One JSON line each under
# gpurun_out/breakdown/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/breakdown
mkdir -p $OUT
export PYTHONPATH="$GRAFT_REPO_ROOT"
run() {  # run <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 500 env ${RUN_ENV:-TK_BREAKDOWN=1} python3 bench.py --steps ${STEPS:-3} --warmup 1 --warm-steps 0 "$@" \
    --report $OUT/$tag.report.json > $OUT/$tag.json 2> $OUT/$tag.err || exit $?
  python3 - "$OUT/$tag.json" "$tag" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pm = d["phase_ms_per_step"]
print(sys.argv[2], d["value"], "burnin", d["gpu_burnin_ms"], "rccl_init", pm.get("rccl.init_total_max_rank"),
      "settle", d["hbm_settle_s"])
for b in d["burnin_phase_ms"]:
    print("   ", b)
EOF
}
run default
run nogate --no-rccl-gate
run slim --rccl-slim on
run quick --burnin quick
RUN_ENV=TK_BURNIN_RELEASE_HOLD=0 run nohold
