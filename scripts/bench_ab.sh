#!/bin/bash
# GPU box: alternating A/B of bench.py arms, one JSON line each under gpurun_out/ab/.
#   bash scripts/bench_ab.sh <tag>=<ENV=VAL[,ENV=VAL]> ...      (tag=- for no extra env)
# e.g.  bash scripts/bench_ab.sh base=- preload=TK_RCCL_PRELOAD=1 base2=- preload2=TK_RCCL_PRELOAD=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab
mkdir -p $OUT
export PYTHONPATH="$GRAFT_REPO_ROOT"
for arm in "$@"; do
  tag=${arm%%=*}; envs=${arm#*=}
  [ "$envs" = "-" ] && envs="TK_AB=1"
  timeout -k 10 400 env ${envs//,/ } python3 bench.py --steps ${STEPS:-3} --warmup 1 > $OUT/$tag.json 2> $OUT/$tag.err || exit $?
  python3 - "$OUT/$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pm = d["phase_ms_per_step"]
print(sys.argv[2], d["value"], d["create_to_ready_s"], "init", pm.get("rccl.init_total_max_rank"),
      "agents_start", d.get("agents_start_s_mean"), "burnin", d["gpu_burnin_ms"])
PY
done
