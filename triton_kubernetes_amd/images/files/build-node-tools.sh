#!/bin/bash
# Build the MI355X node tools for gfx950 from /opt/triton-kubernetes/src into
# /opt/triton-kubernetes/bin, each stamped with the sha256 of the sources it was built
# from.  tk_node_tools is the function the Terraform host module runs
# (triton_kubernetes_amd/node/tools.py, which writes this file), so a node made from this
# image keeps these tools at bring-up: nothing is uploaded or compiled again while the
# shipped sources match.
set -euo pipefail
S=${TK_SRC:-/opt/triton-kubernetes/src}
T=${TK_BIN:-/opt/triton-kubernetes/bin}
ROCM=${ROCM_PATH:-/opt/rocm}
tk_libs_resolve() { # <binary>: every shared library it needs is on this host
  case "$(ldd "$1" 2>/dev/null || true)" in *'not found'*) return 1 ;; esac
}
tk_node_tool() { # <tools dir> <sources dir> <prebuilt dir> <name> "<sources>" <compiler> <flags...>
  local T=$1 S=$2 P=$3 name=$4 srcs=$5 want
  shift 5
  want=$( { printf 'tool %s\n' "$name"; cd "$S" && sha256sum $srcs; } | sha256sum | cut -d' ' -f1)
  [ -n "$want" ] || { echo "$name: cannot hash its sources in $S" >&2; return 1; }
  if [ -x "$T/$name" ] && [ "$(cat "$T/.stamps/$name.sha256" 2>/dev/null)" = "$want" ]; then
    echo "$name: installed copy is current"
    return 0
  fi
  if [ -x "$P/$name" ] && [ "$(cat "$P/$name.sha256" 2>/dev/null)" = "$want $(sha256sum < "$P/$name" | cut -d' ' -f1)" ] \
      && tk_libs_resolve "$P/$name"; then
    sudo install -m 0755 "$P/$name" "$T/$name" || return 1
    echo "$name: prebuilt binary installed"
  elif command -v "$1" >/dev/null 2>&1; then
    echo "$name: no matching prebuilt binary; building with $1"
    sudo "$@" -o "$T/$name" || { echo "$name: build failed" >&2; return 1; }
  else
    echo "$name: no prebuilt binary for the shipped sources was uploaded and $1 is not on this node" >&2
    return 1
  fi
  echo "$want" | sudo tee "$T/.stamps/$name.sha256" >/dev/null
}
tk_node_tools() { # <tools dir> <sources dir> <prebuilt dir> <rocm dir>
  local T=$1 S=$2 P=$3 R=$4 pids='' p rc=0 t0
  t0=$(date +%s%N)
  sudo mkdir -p "$T/.stamps" || return 1
  tk_node_tool "$T" "$S" "$P" amdgpu-topo-labeller "tk_topo.cpp" g++ -O2 -std=c++17 -DTK_TOPO_MAIN -DTK_TOPO_AMDSMI -I$R/include $S/tk_topo.cpp -L$R/lib -lamd_smi -Wl,-rpath,$R/lib &
  pids="$pids $!"
  tk_node_tool "$T" "$S" "$P" gpu-burnin "tk_gpu_probe.hip tk_gemm_screen.hip tk_link_verdict.h" $R/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -DTK_PROBE_MAIN $S/tk_gpu_probe.hip $S/tk_gemm_screen.hip -Wl,-rpath,$R/lib &
  pids="$pids $!"
  tk_node_tool "$T" "$S" "$P" rccl-ready "tk_rccl_probe.hip tk_rccl_verify.h tk_rccl_group.h tk_elf_scan.h" $R/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -DTK_RCCL_MAIN $S/tk_rccl_probe.hip -L$R/lib -lrccl -Wl,-rpath,$R/lib &
  pids="$pids $!"
  for p in $pids; do wait "$p" || rc=1; done
  echo "node tools: $(( ($(date +%s%N) - t0) / 1000000 )) ms"
  return $rc
}
tk_node_tools "$T" "$S" /nonexistent "$ROCM"
"$T/amdgpu-topo-labeller" --labels
