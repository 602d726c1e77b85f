"""``python -m triton_kubernetes_amd.release.build``: the release directory.

Mirrors the reference's ``make build`` + ``build-rpm`` + ``build-deb`` +
``sha256-checksums.txt`` (``Makefile:1-79``):

* ``triton-kubernetes-<version>.pyz`` -- the CLI as one file (git sha injected as
  ``CLI_VERSION``, like ``-ldflags -X cmd.cliVersion``);
* ``triton-kubernetes_<version>-1_all.deb`` / ``triton-kubernetes-<version>-1.noarch.rpm``
  -- that file at ``/usr/bin/triton-kubernetes``; depends on python3, openssh-client
  and openssl (the reference's only dependency was ``jq``, which this CLI does not need);
* ``triton-kubernetes-node_<version>-1_amd64.deb`` / ``…-node-<version>-1.x86_64.rpm`` --
  the gfx950 node tools, their sources, the node agent and its systemd unit;
* ``sha256-checksums.txt`` over all of them.
"""

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import zipapp
from typing import List, Optional

from .. import __version__
from .packages import Package, PkgFile, build_deb, build_rpm, tree_files, write_checksums

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROOT = os.path.dirname(PKG_DIR)
NODE_TOOLS = ("amdgpu-topo-labeller", "gpu-burnin", "rccl-ready")


def git_sha() -> str:
    try:
        return subprocess.run(["git", "rev-parse", "--short", "HEAD"], cwd=ROOT, capture_output=True, text=True,
                              check=True).stdout.strip() or "local"
    except (OSError, subprocess.CalledProcessError):
        return "local"


def build_pyz(out_dir: str, sha: str) -> str:
    with tempfile.TemporaryDirectory(prefix="tk-pyz-") as tmp:
        dst = os.path.join(tmp, "triton_kubernetes_amd")
        shutil.copytree(PKG_DIR, dst, ignore=shutil.ignore_patterns("__pycache__", "*.pyc", "lib"))
        with open(os.path.join(dst, "_build_info.py"), "w", encoding="utf-8") as fh:
            fh.write(f'CLI_VERSION = "{sha}"\n')
        out = os.path.join(out_dir, f"triton-kubernetes-v{__version__}.pyz")
        zipapp.create_archive(tmp, out, interpreter="/usr/bin/env python3", main="triton_kubernetes_amd.cli.main:main")
    return out


def cli_package(pyz: str) -> Package:
    with open(pyz, "rb") as fh:
        data = fh.read()
    return Package("triton-kubernetes", __version__, arch="all",
                   summary="Multi-cloud Kubernetes (Rancher/RKE) provisioning CLI with an MI355X bare-metal path",
                   description="create|destroy|get manager/cluster/node over Terraform or the native executor.",
                   depends=["python3 (>= 3.10)", "openssh-client", "openssl"],
                   files=[PkgFile("/usr/bin/triton-kubernetes", data, 0o755)])


def node_package() -> Package:
    from ..ops.native import LIB_DIR

    files: List[PkgFile] = []
    for tool in NODE_TOOLS:
        path = os.path.join(LIB_DIR, tool)
        if not os.path.exists(path):
            raise SystemExit(f"{path} missing: build the native tools first (make native)")
        with open(path, "rb") as fh:
            files.append(PkgFile(f"/opt/triton-kubernetes/bin/{tool}", fh.read(), 0o755))
    images = os.path.join(PKG_DIR, "images", "files")
    files += tree_files(os.path.join(images, "src"), "/opt/triton-kubernetes/src", lambda rel: 0o644)
    with open(os.path.join(images, "tk-node-agent.service"), "rb") as fh:
        files.append(PkgFile("/lib/systemd/system/tk-node-agent.service", fh.read(), 0o644))
    files += tree_files(PKG_DIR, "/usr/lib/python3/dist-packages/triton_kubernetes_amd", lambda rel: 0o644)
    files = [f for f in files if "/ops/lib/" not in f.path]
    return Package("triton-kubernetes-node", __version__, arch="amd64",
                   summary="MI355X node tools: topology labeller, burn-in, RCCL readiness probe, node agent",
                   description="gfx950 executables built from the shipped sources, plus the tk-node-agent daemon.",
                   depends=["python3 (>= 3.10)", "rocm-hip-runtime", "rccl", "amd-smi-lib"], files=files)


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="python -m triton_kubernetes_amd.release.build")
    ap.add_argument("--out", default=os.path.join(ROOT, "build"))
    ap.add_argument("--formats", default="pyz,deb,rpm")
    ap.add_argument("--no-node", action="store_true", help="skip the node-tools package")
    args = ap.parse_args(argv)
    os.makedirs(args.out, exist_ok=True)
    fmts = set(args.formats.split(","))
    sha = git_sha()
    made = [build_pyz(args.out, sha)]
    pkgs = [cli_package(made[0])] + ([] if args.no_node else [node_package()])
    for pkg in pkgs:
        if "deb" in fmts:
            path = os.path.join(args.out, f"{pkg.name}_{pkg.version}-{pkg.release}_{pkg.arch}.deb")
            with open(path, "wb") as fh:
                fh.write(build_deb(pkg))
            made.append(path)
        if "rpm" in fmts:
            arch = {"amd64": "x86_64", "all": "noarch"}.get(pkg.arch, pkg.arch)
            path = os.path.join(args.out, f"{pkg.name}-{pkg.version}-{pkg.release}.{arch}.rpm")
            with open(path, "wb") as fh:
                fh.write(build_rpm(pkg))
            made.append(path)
    made.append(write_checksums(made, os.path.join(args.out, "sha256-checksums.txt")))
    print(json.dumps({"artifacts": made}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
