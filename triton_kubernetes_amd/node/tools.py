"""The MI355X node tools, shipped prebuilt and stamped with the sources they come from.

The reference installs no GPU tooling at all (its host modules only run the Rancher agent
container, ``terraform/modules/bare-metal-rancher-k8s-host/main.tf``).  Here an MI355X host
gets three tools in ``/opt/triton-kubernetes/bin``: ``amdgpu-topo-labeller`` (N1),
``gpu-burnin`` (the HBM/MFMA/memtest/GEMM screen) and ``rccl-ready`` (N2).  Building them on
every node with ``hipcc`` costs ~40 s of a cold create per node (two gfx950 compiles) and needs
the ROCm compiler on production hosts, so:

* the CLI stages the in-tree build (``ops/build.py``; rebuilt first when stale) into the
  Terraform work dir, each binary next to ``<tool>.sha256``, its **node stamp**: a sha256
  over the tool's name and the sha256 of every source it is built from (:func:`node_stamp`);
* the host module uploads that directory (``tk_prebuilt_tools``) beside the shipped sources,
  and its install script (``tk_node_tools``, :data:`NODE_TOOLS_FN`) computes the same stamp
  from the sources it was shipped.  Per tool: kept when the installed copy carries that
  stamp (a re-apply compiles nothing); else the uploaded binary when its stamp matches, its
  own sha256 is the one staged with it (it arrived whole) and its shared libraries resolve on
  the node; else built on the node (``hipcc``/``g++`` only
  as this fallback, the builds in parallel); with no compiler there either, the node fails
  naming the tool.

The stamp is over the sources, not mtimes (an upload resets those), so a binary built from
other sources than the ones shipped is never installed.  The other two delivery paths use
the same stamp: the DirectExecutor uploads a tool over SSH only when the host's stamp for
it differs (:data:`REMOTE_STAMPS`), and the machine image (``images/files/build-node-tools.sh``)
builds with this same ``tk_node_tools``, so a node made from the image keeps its tools.
"""

import hashlib
import os
import shutil
import sys
from typing import Callable, Dict, List, Optional

from ..ops.build import CSRC

# tool -> the shipped sources it is built from (basenames under the module's files/src)
TOOL_SOURCES: Dict[str, List[str]] = {
    "amdgpu-topo-labeller": ["tk_topo.cpp"],
    "gpu-burnin": ["tk_gpu_probe.hip", "tk_gemm_screen.hip", "tk_link_verdict.h"],
    "rccl-ready": ["tk_rccl_probe.hip", "tk_rccl_verify.h", "tk_rccl_group.h", "tk_elf_scan.h"],
}
PREBUILT_DIR = "/opt/triton-kubernetes/prebuilt"
SOURCES_DIR = "/opt/triton-kubernetes/src"


def node_stamp(name: str, src_dir: str = CSRC) -> str:
    """What ``tk_node_tools`` computes on the node: sha256 of ``tool <name>`` and
    ``sha256sum``'s lines for the tool's sources (in :data:`TOOL_SOURCES` order)."""
    lines = [f"tool {name}\n"]
    for src in TOOL_SOURCES[name]:
        with open(os.path.join(src_dir, src), "rb") as fh:
            lines.append(f"{hashlib.sha256(fh.read()).hexdigest()}  {src}\n")
    return hashlib.sha256("".join(lines).encode()).hexdigest()


def _in_tree(name: str) -> str:
    from ..ops.native import executable

    return executable(name)


def stage(dest: str, binary: Optional[Callable[[str], str]] = None, log=None) -> Dict[str, str]:
    """Copy each node tool built from this tree's sources into ``dest`` with its node
    stamp.  A tool that cannot be built here (no ROCm compiler on the operator's machine) is
    left out: the node builds that one.  Returns ``{tool: "prebuilt" | "<why not>"}``."""
    from ..ops.native import NativeUnavailable

    binary = binary or _in_tree
    log = log or (lambda msg: sys.stderr.write(msg + "\n"))
    os.makedirs(dest, exist_ok=True)
    out: Dict[str, str] = {}
    for name in TOOL_SOURCES:
        try:
            path = binary(name)
        except NativeUnavailable as exc:
            out[name] = f"not staged: {exc}"
            log(f"{name}: no gfx950 build on this machine ({exc}); MI355X nodes build it themselves")
            continue
        shutil.copyfile(path, os.path.join(dest, name))
        os.chmod(os.path.join(dest, name), 0o755)
        with open(os.path.join(dest, name), "rb") as fh:
            binary_sum = hashlib.sha256(fh.read()).hexdigest()
        # "<source stamp> <sha256 of the binary>": the node installs it only when both hold
        # (the shipped sources are the ones it was built from; it arrived whole)
        with open(os.path.join(dest, name + ".sha256"), "w", encoding="ascii") as fh:
            fh.write(f"{node_stamp(name)} {binary_sum}\n")
        out[name] = "prebuilt"
    return out


# Installed by the MI355X host module's script (terraform/scripts.py INSTALL_MI355X_NODE);
# no "${" or "%{" so it reads the same inside a Terraform template and on its own.
NODE_TOOLS_FN = r"""tk_libs_resolve() { # <binary>: every shared library it needs is on this host
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
}"""

def image_build_script() -> str:
    """``images/files/build-node-tools.sh``: the machine image's tool build (packer), on this
    same ``tk_node_tools``.  ``python -m triton_kubernetes_amd.node.tools`` rewrites the file."""
    return ("#!/bin/bash\n"
            "# Build the MI355X node tools for gfx950 from /opt/triton-kubernetes/src into\n"
            "# /opt/triton-kubernetes/bin, each stamped with the sha256 of the sources it was built\n"
            "# from.  tk_node_tools is the function the Terraform host module runs\n"
            "# (triton_kubernetes_amd/node/tools.py, which writes this file), so a node made from this\n"
            "# image keeps these tools at bring-up: nothing is uploaded or compiled again while the\n"
            "# shipped sources match.\n"
            "set -euo pipefail\n"
            "S=${TK_SRC:-/opt/triton-kubernetes/src}\n"
            "T=${TK_BIN:-/opt/triton-kubernetes/bin}\n"
            "ROCM=${ROCM_PATH:-/opt/rocm}\n"
            + NODE_TOOLS_FN + "\n"
            'tk_node_tools "$T" "$S" /nonexistent "$ROCM"\n'
            '"$T/amdgpu-topo-labeller" --labels\n')


# "<tool> <stamp>" for every node tool installed with a stamp (DirectExecutor uploads)
REMOTE_STAMPS = """for f in {tools}/.stamps/*.sha256; do
  n=$(basename "$f" .sha256)
  [ -f "$f" ] && [ -x "{tools}/$n" ] && echo "$n $(cat "$f")"
done
true
"""

if __name__ == "__main__":
    from ..images import packer

    with open(os.path.join(packer.FILES_DIR, "build-node-tools.sh"), "w", encoding="utf-8") as out:
        out.write(image_build_script())
    print("wrote", os.path.join(packer.FILES_DIR, "build-node-tools.sh"))

__all__ = ["NODE_TOOLS_FN", "REMOTE_STAMPS", "image_build_script", "PREBUILT_DIR", "SOURCES_DIR", "TOOL_SOURCES", "node_stamp", "stage"]
