#!/bin/bash
# GPU box: the headline bench at its defaults (burn-in full, HBM settle on) and the A/B
# with the settle wait off; sysfs VRAM used sampled around each run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/settle_ab
export PYTHONPATH="$GRAFT_REPO_ROOT"
OUT=gpurun_out/settle_ab
vram() { python3 -c "from triton_kubernetes_amd.ops import hbm; import json; print(json.dumps(hbm.vram_used()))"; }
echo "before $(vram)" >> $OUT/vram.log
timeout -k 10 600 python3 bench.py --steps ${STEPS:-5} --warmup 1 --warm-steps 0 --report $OUT/settle_on_report.json \
  > $OUT/settle_on.json 2> $OUT/settle_on.err || exit $?
echo "after_on $(vram)" >> $OUT/vram.log
timeout -k 10 600 python3 bench.py --steps ${STEPS:-5} --warmup 1 --warm-steps 0 --hbm-settle off \
  --report $OUT/settle_off_report.json > $OUT/settle_off.json 2> $OUT/settle_off.err || exit $?
echo "after_off $(vram)" >> $OUT/vram.log
python3 - <<'EOF'
import json
for tag in ("on", "off"):
    d = json.loads(open(f"gpurun_out/settle_ab/settle_{tag}.json").read().strip().splitlines()[-1])
    print(tag, d["value"], d["ms_per_step"], d["config"]["burnin"], d["gpu_burnin_ms"], d["hbm_settle_s"],
          d["hbm_settle_released_gib"])
EOF
