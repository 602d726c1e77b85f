"""Build the native MI355X components in-tree (``triton_kubernetes_amd/ops/lib``).

Targets (gfx950 only; ``hipcc`` cross-compiles without a GPU):

=============================  ==========================================  =========
artifact                       source                                      toolchain
=============================  ==========================================  =========
``libtk_gpu_probe.so``         ``csrc/tk_gpu_probe.hip`` (HBM/MFMA/memtest)  hipcc
``libtk_gemm.so``              ``csrc/tk_gemm_screen.hip`` (ABFT GEMM screen)  hipcc
``libtk_rccl.so``              ``csrc/tk_rccl_probe.hip`` (N2, RCCL)          hipcc
``rccl-ready``                 same, ``-DTK_RCCL_MAIN``                     hipcc
``libtk_rccl_stub.so``         ``csrc/tk_rccl_stub.cpp`` (the ABI, no GPU)    g++
``libtk_topo.so``              ``csrc/tk_topo.cpp`` (N1, sysfs collector)    g++
``amdgpu-topo-labeller``       same + amd_smi, ``-DTK_TOPO_MAIN``           g++
=============================  ==========================================  =========

Usage: ``python -m triton_kubernetes_amd.ops.build [--force] [-j N]``.
Rebuilds only targets that are not current.  Every artifact gets a stamp
(``lib/.stamps/<name>.sha256``): a sha256 over its sources' contents and its build command
(paths made relative), written after a successful build.  An artifact is current when its
stamp matches its sources -- not their mtimes, which a copy or an upload resets -- so a
node tool can be checked against the sources it must have been built from (the MI355X
host module's prebuilt tools, ``ops/probe.py``'s ``gpu-burnin`` child).
"""

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from dataclasses import dataclass
from typing import List, Sequence

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

HIP_FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result", "-Wno-unused-value",
             "-Wno-unused-command-line-argument"]
RPATH = [f"-Wl,-rpath,{ROCM}/lib"]
# VGPR-form MFMA accumulators: see the note at the top of csrc/tk_gpu_probe.hip
MFMA_FLAGS = ["-mllvm", "-amdgpu-mfma-vgpr-form"]


@dataclass
class Target:
    name: str
    sources: List[str]
    cmd: List[str]

    @property
    def output(self) -> str:
        return os.path.join(LIB, self.name)

    @property
    def stamp_path(self) -> str:
        return os.path.join(LIB, ".stamps", self.name + ".sha256")

    def source_hash(self) -> str:
        """sha256 over the build command (locations replaced by placeholders, so the same
        tree hashes the same wherever it is unpacked) and every source's name and bytes."""
        return source_hash(self.name, self.sources, self.cmd)

    def stamp(self) -> str:
        try:
            with open(self.stamp_path, "r", encoding="ascii") as fh:
                return fh.read().strip()
        except OSError:
            return ""

    def stale(self) -> bool:
        return not os.path.exists(self.output) or self.stamp() != self.source_hash()

    def write_stamp(self) -> None:
        os.makedirs(os.path.dirname(self.stamp_path), exist_ok=True)
        tmp = self.stamp_path + ".tmp"
        with open(tmp, "w", encoding="ascii") as fh:
            fh.write(self.source_hash() + "\n")
        os.replace(tmp, self.stamp_path)


def source_hash(name: str, sources: Sequence[str], cmd: Sequence[str]) -> str:
    h = hashlib.sha256()
    h.update(name.encode() + b"\0")
    for i, arg in enumerate(cmd):
        # the compiler driver by name (hipcc is on PATH or under ROCm, either is the same)
        arg = os.path.basename(arg) if i == 0 else arg.replace(LIB, "<lib>").replace(CSRC, "<csrc>").replace(
            ROCM, "<rocm>")
        h.update(arg.encode() + b"\0")
    for src in sources:
        h.update(os.path.basename(src).encode() + b"\0")
        with open(src, "rb") as fh:
            h.update(hashlib.sha256(fh.read()).digest())
    return h.hexdigest()


def target(name: str) -> "Target":
    for t in targets():
        if t.name == name:
            return t
    raise KeyError(name)


def current(name: str) -> bool:
    """The artifact ``name`` exists and was built from the sources in this tree."""
    return not target(name).stale()


def _hipcc() -> str:
    return shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")


def targets() -> List[Target]:
    hipcc = _hipcc()
    probe = os.path.join(CSRC, "tk_gpu_probe.hip")
    rccl = os.path.join(CSRC, "tk_rccl_probe.hip")
    gemm = os.path.join(CSRC, "tk_gemm_screen.hip")
    topo = os.path.join(CSRC, "tk_topo.cpp")
    stub = os.path.join(CSRC, "tk_rccl_stub.cpp")
    rccl_h = [os.path.join(CSRC, "tk_rccl_group.h"), os.path.join(CSRC, "tk_rccl_verify.h"),
              os.path.join(CSRC, "tk_elf_scan.h")]
    link_h = os.path.join(CSRC, "tk_link_verdict.h")
    out = lambda n: os.path.join(LIB, n)  # noqa: E731
    return [
        Target("libtk_gpu_probe.so", [probe, link_h],
               [hipcc, *HIP_FLAGS, *MFMA_FLAGS, "-fPIC", "-shared", probe, "-o", out("libtk_gpu_probe.so"), *RPATH]),
        Target("gpu-burnin", [probe, gemm, link_h],
               [hipcc, *HIP_FLAGS, *MFMA_FLAGS, "-DTK_PROBE_MAIN", probe, gemm, "-o", out("gpu-burnin"), *RPATH]),
        Target("libtk_gemm.so", [gemm],
               [hipcc, *HIP_FLAGS, "-fPIC", "-shared", gemm, "-o", out("libtk_gemm.so"), *RPATH]),
        Target("libtk_rccl.so", [rccl, *rccl_h],
               [hipcc, *HIP_FLAGS, "-fPIC", "-shared", rccl, "-o", out("libtk_rccl.so"), f"-L{ROCM}/lib",
                "-lrccl", *RPATH]),
        # /opt/rocm's RCCL (RUNPATH).  The opt-in single-target copy (rccl_slim) is reached
        # only through the rccl-ready-slim wrapper, which checks it is verified and current
        Target("rccl-ready", [rccl, *rccl_h],
               [hipcc, *HIP_FLAGS, "-DTK_RCCL_MAIN", rccl, "-o", out("rccl-ready"), f"-L{ROCM}/lib", "-lrccl",
                *RPATH]),
        # the libtk_rccl C ABI without GPUs or RCCL: dry runs of the cluster gate (TK_RCCL_LIB)
        Target("libtk_rccl_stub.so", [stub, *rccl_h],
               ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", f"-I{CSRC}", stub, "-o", out("libtk_rccl_stub.so"),
                "-lpthread"]),
        # in-process library: sysfs collector only, no libamd_smi (see csrc/tk_topo.cpp)
        Target("libtk_topo.so", [topo],
               ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", topo, "-o", out("libtk_topo.so")]),
        Target("amdgpu-topo-labeller", [topo],
               ["g++", "-O2", "-std=c++17", "-DTK_TOPO_MAIN", "-DTK_TOPO_AMDSMI", f"-I{ROCM}/include", topo, "-o",
                out("amdgpu-topo-labeller"), f"-L{ROCM}/lib", "-lamd_smi", *RPATH]),
    ]


def _run(t: Target) -> str:
    proc = subprocess.run(t.cmd, capture_output=True, text=True, check=False)
    if proc.returncode != 0:
        raise RuntimeError(f"building {t.name} failed:\n$ {' '.join(t.cmd)}\n{proc.stdout}\n{proc.stderr}")
    t.write_stamp()
    return t.name


def build(force: bool = False, jobs: int = 4, only: Sequence[str] = ()) -> List[str]:
    os.makedirs(LIB, exist_ok=True)
    todo = [t for t in targets() if (force or t.stale()) and (not only or t.name in only)]
    built: List[str] = []
    if not todo:
        return built
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as pool:
        for name in pool.map(_run, todo):
            built.append(name)
    return built


def main(argv: Sequence[str] = ()) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("targets", nargs="*")
    args = ap.parse_args(list(argv) or sys.argv[1:])
    built = build(args.force, args.jobs, args.targets)
    print(f"built: {', '.join(built) if built else '(up to date)'} -> {LIB}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
