#!/bin/bash
# A/B: the bench with and without the agent applying the node's RCCL env at start.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for mode in 1 0 1 0; do
  TK_AGENT_RCCL_ENV=$mode timeout -k 10 300 python bench.py --steps 5 --warmup 1 --warm-steps 0 \
    --report gpurun_out/ab_env$mode.json > gpurun_out/ab_env$mode.log 2>&1 || exit $?
  python3 -c "import json;r=json.load(open('gpurun_out/ab_env$mode.json'));l=r['line'];print('env=$mode', l['value'], l['create_to_ready_s'], l['phase_ms_per_step'].get('rccl.init_total_max_rank'))" >> gpurun_out/ab_env.txt
done
python3 - <<'PY' >> gpurun_out/ab_env.txt
import json, os
from triton_kubernetes_amd.node.agent import NodeAgent
a = NodeAgent(name="probe", mode="sim", devices=[0])
try:
    import triton_kubernetes_amd.parallel.rccl_env as re_
    print("site env from topology:", re_.site_env_from_topology(a._topology()))
finally:
    a.stop()
PY
