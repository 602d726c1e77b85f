#!/bin/bash
# GPU-box run: native probe tests, per-probe sweeps, and a rocprofv3 kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH="$GRAFT_REPO_ROOT"
LOG=gpurun_out/gpu_tests.log
fatal() { case "$1" in 0|1|2) return 1;; esac; return 0; }

# isolate the exit-time heap corruption seen in the first run
timeout -k 10 120 python -c "from triton_kubernetes_amd.ops import topo; d=topo.amdsmi_topology_inprocess(); print(len(d['gpus']))" > gpurun_out/diag_topo_inproc.log 2>&1
echo "diag_topo_inproc rc=$?" >> $LOG
timeout -k 10 120 python -c "from triton_kubernetes_amd.ops import rccl; r=rccl.sweep_rank(0,1,rccl.unique_id(),0,[1<<20],3,1); print(r.to_json())" > gpurun_out/diag_rccl.log 2>&1
rc=$?; echo "diag_rccl rc=$rc" >> $LOG
timeout -k 10 120 python -c "from triton_kubernetes_amd.ops import probe; print(probe.memtest(0, 1<<28, 1))" > gpurun_out/diag_memtest.log 2>&1
rc=$?; echo "diag_memtest rc=$rc" >> $LOG

timeout -k 10 600 python -m pytest tests/test_gpu_probes.py -m gpu -q -s -p no:cacheprovider >> $LOG 2>&1
rc=$?; echo "pytest_rc=$rc" >> $LOG
if fatal $rc; then exit $rc; fi

for args in "hbm --gib 4" "hbm --gib 4 --blocks-per-cu 8" "hbm --gib 4 --blocks-per-cu 32" \
            "mfma --dtype bf16 --blocks-per-cu 1" "mfma --dtype bf16 --blocks-per-cu 2" \
            "mfma --dtype bf16 --blocks-per-cu 4" "mfma --dtype fp8 --blocks-per-cu 1" "mfma --dtype fp8 --blocks-per-cu 2" \
            "mfma --dtype f32 --iters 4000" "topology"; do
  name=$(echo "$args" | tr ' ' '_' | tr -d '-')
  timeout -k 10 120 python -m triton_kubernetes_amd.ops.cli $args > "gpurun_out/$name.json" 2>&1
  rc=$?; if fatal $rc; then echo "$args rc=$rc" >> $LOG; exit $rc; fi
done

cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_burnin" -o burnin -- python3 -m triton_kubernetes_amd.ops.cli burnin --level quick > "$GRAFT_REPO_ROOT/gpurun_out/prof_burnin.log" 2>&1
echo "prof_rc=$?" >> "$GRAFT_REPO_ROOT/gpurun_out/prof_burnin.log"
