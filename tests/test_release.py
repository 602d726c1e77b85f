"""Release artefacts (reference Makefile build-deb / build-rpm / sha256-checksums.txt):
stdlib .deb and .rpm writers, read back with dpkg-deb and the module's own rpm reader."""

import hashlib
import os
import subprocess

import pytest

from triton_kubernetes_amd.release import build
from triton_kubernetes_amd.release.packages import Package, PkgFile, build_deb, build_rpm, read_rpm

from helpers import have


def _pkg():
    return Package("tk-demo", "1.2.3", arch="amd64", summary="demo", description="line one\n\nline three",
                   depends=["python3 (>= 3.10)", "jq"],
                   files=[PkgFile("/usr/bin/tk-demo", b"#!/bin/sh\necho hi\n", 0o755),
                          PkgFile("/opt/tk/share/data.txt", b"x" * 1001)], mtime=1700000000)


@pytest.mark.skipif(not have("dpkg-deb"), reason="dpkg-deb not installed")
def test_deb_reads_back_with_dpkg(tmp_path):
    deb = tmp_path / "tk-demo.deb"
    deb.write_bytes(build_deb(_pkg()))
    info = subprocess.run(["dpkg-deb", "--field", str(deb), "Package", "Version", "Architecture", "Depends"],
                          capture_output=True, text=True, check=True).stdout
    assert "Package: tk-demo" in info and "Version: 1.2.3-1" in info and "Depends: python3 (>= 3.10), jq" in info
    out = tmp_path / "x"
    subprocess.run(["dpkg-deb", "-x", str(deb), str(out)], check=True)
    exe = out / "usr/bin/tk-demo"
    assert exe.read_bytes() == b"#!/bin/sh\necho hi\n" and os.access(exe, os.X_OK)
    assert (out / "opt/tk/share/data.txt").stat().st_size == 1001
    ctl = tmp_path / "c"
    subprocess.run(["dpkg-deb", "-e", str(deb), str(ctl)], check=True)
    md5 = (ctl / "md5sums").read_text()
    assert f"{hashlib.md5(b'x' * 1001).hexdigest()}  opt/tk/share/data.txt" in md5


def test_rpm_structure_and_digests():
    data = build_rpm(_pkg())
    doc = read_rpm(data)
    h = doc["header"]
    assert (h["NAME"], h["VERSION"], h["RELEASE"], h["ARCH"], h["OS"]) == ("tk-demo", "1.2.3", "1", "x86_64", "linux")
    assert h["REQUIRENAME"] == ["python3", "jq"] and h["PAYLOADCOMPRESSOR"] == "gzip"
    paths = [h["DIRNAMES"][i] + b for i, b in zip(h["DIRINDEXES"], h["BASENAMES"])]
    assert paths == ["/opt/tk/share/data.txt", "/usr/bin/tk-demo"]
    for p, digest, size in zip(paths, h["FILEDIGESTS"], h["FILESIZES"]):
        body, mode = doc["files"][p]
        assert hashlib.sha256(body).hexdigest() == digest and len(body) == size
    assert doc["files"]["/usr/bin/tk-demo"][1] & 0o777 == 0o755
    sig = doc["signature"]
    assert sig[1004] == hashlib.md5(doc["header_bytes"] + doc["payload"]).digest()  # RPMSIGTAG_MD5
    assert sig[1000] == [len(doc["header_bytes"]) + len(doc["payload"])]  # RPMSIGTAG_SIZE
    assert sig[273] == hashlib.sha256(doc["header_bytes"]).hexdigest()  # RPMSIGTAG_SHA256


def test_packages_are_reproducible():
    assert build_deb(_pkg()) == build_deb(_pkg()) and build_rpm(_pkg()) == build_rpm(_pkg())


def test_release_build_writes_checksummed_artifacts(tmp_path, monkeypatch):
    monkeypatch.setenv("SOURCE_DATE_EPOCH", "1700000000")
    from triton_kubernetes_amd.ops.native import LIB_DIR

    node = all(os.path.exists(os.path.join(LIB_DIR, t)) for t in build.NODE_TOOLS)
    assert build.main(["--out", str(tmp_path)] + ([] if node else ["--no-node"])) == 0
    names = sorted(os.listdir(tmp_path))
    assert "triton-kubernetes_0.8.2-1_all.deb" in names and "triton-kubernetes-0.8.2-1.noarch.rpm" in names
    sums = dict(reversed(ln.split("  ")) for ln in (tmp_path / "sha256-checksums.txt").read_text().splitlines())
    for name, digest in sums.items():
        assert hashlib.sha256((tmp_path / name).read_bytes()).hexdigest() == digest
    assert len(sums) == len(names) - 1
    rpm = read_rpm((tmp_path / "triton-kubernetes-0.8.2-1.noarch.rpm").read_bytes())
    pyz = rpm["files"]["/usr/bin/triton-kubernetes"][0]
    assert pyz == (tmp_path / "triton-kubernetes-v0.8.2.pyz").read_bytes()
    out = subprocess.run(["python3", str(tmp_path / "triton-kubernetes-v0.8.2.pyz"), "version"], capture_output=True,
                         text=True, check=True).stdout
    assert out.startswith("triton-kubernetes v0.8.2 (")
    if node:
        rpm = read_rpm((tmp_path / "triton-kubernetes-node-0.8.2-1.x86_64.rpm").read_bytes())
        assert {"/opt/triton-kubernetes/bin/rccl-ready", "/lib/systemd/system/tk-node-agent.service"} <= set(rpm["files"])
