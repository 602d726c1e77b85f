"""Single-target RCCL preparation (ops/rccl_slim.py) and its runtime selection (ops/native.py).

CPU only: the in-tree gfx950 libraries stand in for ``librccl.so`` (their ``.hip_fatbin`` is
an uncompressed host+gfx950 bundle); a compressed multi-target source is made from them with
``clang-offload-bundler --compress``, the format of the PyTorch-ROCm and /opt/rocm RCCL builds.
The GPU side (the slim library loads, and the first communicator init gets faster) is
``tests/test_gpu_probes.py::test_slim_rccl_runtime_gate`` and ``profiles/round2/rccl_slim_ab.md``.
"""

import json
import os
import shutil
import subprocess
import sys

import pytest

from triton_kubernetes_amd.ops import native, rccl_slim

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GFX950 = rccl_slim.device_triple("gfx950")


def _lib(name="libtk_gpu_probe.so"):
    path = os.path.join(native.LIB_DIR, name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not built")
    return path


def _section(path):
    off, size = rccl_slim.elf_section(path, ".hip_fatbin")
    with open(path, "rb") as fh:
        fh.seek(off)
        return off, size, fh.read(size)


def _fake_runtime(tmp_path, lib):
    """A runtime dir: ``librccl.so`` (a copy of ``lib``) plus a dependency next to it."""
    src = tmp_path / "src"
    src.mkdir()
    shutil.copyfile(lib, src / "librccl.so")
    (src / "libamdhip64.so").write_bytes(b"not really a library")
    return str(src)


def test_bundle_round_trip_and_alignment():
    co = b"\x7fELF" + bytes(range(256)) * 40
    data = rccl_slim.make_bundle([(rccl_slim.HOST_TRIPLE, b""), (GFX950, co)])
    entries = rccl_slim.parse_bundle(data)
    assert [e[0] for e in entries] == [rccl_slim.HOST_TRIPLE, GFX950]
    _, off, size = entries[1]
    assert off % rccl_slim.ALIGN == 0 and size == len(co) and data[off:off + size] == co
    assert entries[0][1:] == (0, 0)


def test_in_tree_library_sections_parse():
    _, _, data = _section(_lib())
    triples = [t for t, _, _ in rccl_slim.parse_bundle(data)]
    assert GFX950 in triples


def test_prepare_from_plain_bundle(tmp_path):
    lib = _lib()
    src = _fake_runtime(tmp_path, lib)
    meta = rccl_slim.prepare(src, root=str(tmp_path / "cache"), strip=False, verify_with_gpu=False)
    out = meta["dir"]
    assert not meta["cached"] and meta["source_format"] == "bundle"
    assert os.path.exists(os.path.join(out, "slim.json"))
    # same size and section placement; a single device entry holding the original code object
    assert os.path.getsize(os.path.join(out, "librccl.so")) == os.path.getsize(lib)
    off0, size0, orig = _section(lib)
    off1, size1, new = _section(os.path.join(out, "librccl.so"))
    assert (off0, size0) == (off1, size1)
    entries = rccl_slim.parse_bundle(new)
    assert [t for t, _, _ in entries] == [rccl_slim.HOST_TRIPLE, GFX950]
    want = next(orig[o:o + s] for t, o, s in rccl_slim.parse_bundle(orig) if t == GFX950)
    _, o, s = entries[1]
    assert new[o:o + s] == want
    assert new[meta["bundle_bytes"]:] == b"\0" * (size1 - meta["bundle_bytes"])
    # bytes outside the section are untouched
    with open(lib, "rb") as a, open(os.path.join(out, "librccl.so"), "rb") as b:
        x, y = a.read(), b.read()
    assert x[:off0] == y[:off0] and x[off0 + size0:] == y[off0 + size0:]
    # the rest of the runtime is linked in; a second prepare is a cache hit
    assert os.path.islink(os.path.join(out, "libamdhip64.so"))
    assert rccl_slim.prepare(src, root=str(tmp_path / "cache"), strip=False, verify_with_gpu=False)["cached"] is True
    assert rccl_slim.cached(src, root=str(tmp_path / "cache")) == ""  # the stripped entry is another key


@pytest.mark.skipif(not rccl_slim.find_tool("clang-offload-bundler"), reason="no ROCm LLVM bundler")
def test_prepare_from_compressed_multi_target_bundle(tmp_path):
    """The shape of the real RCCL builds: one compressed bundle of many targets."""
    lib = _lib()
    _, _, orig = _section(lib)
    co = next(orig[o:o + s] for t, o, s in rccl_slim.parse_bundle(orig) if t == GFX950)
    (tmp_path / "gfx950.co").write_bytes(co)
    (tmp_path / "other.co").write_bytes(co[::-1])
    (tmp_path / "host").write_bytes(b"")
    bundler = rccl_slim.find_bundler()
    targets = ",".join([rccl_slim.HOST_TRIPLE, rccl_slim.device_triple("gfx942"), GFX950])
    subprocess.run([bundler, "--compress", "--type=o", f"--targets={targets}",
                    f"--input={tmp_path / 'host'}", f"--input={tmp_path / 'other.co'}",
                    f"--input={tmp_path / 'gfx950.co'}", f"--output={tmp_path / 'fat.bin'}"], check=True,
                   capture_output=True)
    fat = (tmp_path / "fat.bin").read_bytes()
    assert fat.startswith(rccl_slim.COMPRESSED_MAGIC)
    src = _fake_runtime(tmp_path, lib)
    off, size, _ = _section(os.path.join(src, "librccl.so"))
    assert len(fat) <= size
    with open(os.path.join(src, "librccl.so"), "r+b") as fh:
        fh.seek(off)
        fh.write(fat + b"\0" * (size - len(fat)))
    meta = rccl_slim.prepare(src, root=str(tmp_path / "cache"), verify_with_gpu=False)
    assert meta["source_format"] == "compressed"
    _, _, new = _section(os.path.join(meta["dir"], "librccl.so"))
    entries = rccl_slim.parse_bundle(new)
    assert [t for t, _, _ in entries] == [rccl_slim.HOST_TRIPLE, GFX950]
    _, o, s = entries[1]
    got = new[o:o + s]
    assert got[:4] == b"\x7fELF" and s == meta["loaded_code_object_bytes"] <= len(co)
    # a target the bundle lacks is an error, and no partial entry is left behind
    with pytest.raises(rccl_slim.SlimError, match="gfx1234"):
        rccl_slim.prepare(src, arch="gfx1234", root=str(tmp_path / "cache2"), verify_with_gpu=False)
    assert not os.path.exists(tmp_path / "cache2") or os.listdir(tmp_path / "cache2") == []


def test_partial_entry_is_never_used(tmp_path):
    src = _fake_runtime(tmp_path, _lib())
    d = rccl_slim.entry_dir(src, root=str(tmp_path / "cache"))
    os.makedirs(d)
    shutil.copyfile(os.path.join(src, "librccl.so"), os.path.join(d, "librccl.so"))
    assert rccl_slim.cached(src, root=str(tmp_path / "cache")) == ""


def test_source_change_invalidates_the_entry(tmp_path):
    src = _fake_runtime(tmp_path, _lib())
    root = str(tmp_path / "cache")
    rccl_slim.prepare(src, root=root, strip=False, verify_with_gpu=False)
    k1 = rccl_slim.entry_dir(src, root=root)
    os.utime(os.path.join(src, "librccl.so"), ns=(1, 1))
    assert rccl_slim.entry_dir(src, root=root) != k1


def test_non_elf_is_refused(tmp_path):
    src = tmp_path / "src"
    src.mkdir()
    (src / "librccl.so").write_bytes(b"MZ" + b"\0" * 100)
    with pytest.raises(rccl_slim.SlimError, match="not an ELF64"):
        rccl_slim.prepare(str(src), root=str(tmp_path / "cache"), verify_with_gpu=False)


def _select(env):
    code = "from triton_kubernetes_amd.ops import native; print(native.select_runtime())"
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT, timeout=120,
                       env=dict(os.environ, **env))
    assert p.returncode == 0, p.stderr
    return p.stdout.strip()


def test_slim_runtime_is_opt_in_and_verified_only(tmp_path):
    """An unverified entry is never selected; TK_HIP_RUNTIME=slim (the opt-in) picks a
    verified one; without the opt-in nothing picks it."""
    root = str(tmp_path / "cache")
    d = rccl_slim.entry_dir(native.SYSTEM_LIB_DIR, root=root)
    os.makedirs(d)
    with open(os.path.join(d, "slim.json"), "w", encoding="utf-8") as fh:
        json.dump({"dir": d}, fh)
    assert rccl_slim.cached(native.SYSTEM_LIB_DIR, root=root) == ""
    with open(os.path.join(d, "slim.json"), "w", encoding="utf-8") as fh:
        json.dump({"dir": d, "verified": {"time": 1}}, fh)
    assert rccl_slim.cached(native.SYSTEM_LIB_DIR, root=root) == d
    assert _select({"TK_HIP_RUNTIME": "slim", "TK_RCCL_SLIM_DIR": root}) == d
    assert _select({"TK_HIP_RUNTIME": "system", "TK_RCCL_SLIM_DIR": root}) == "system"


def test_failed_verification_removes_the_entry(tmp_path, monkeypatch):
    src = _fake_runtime(tmp_path, _lib())
    root = str(tmp_path / "cache")

    def boom(entry, timeout=180.0):
        raise rccl_slim.SlimError("verifying: allreduce mismatch")

    monkeypatch.setattr(rccl_slim, "verify", boom)
    with pytest.raises(rccl_slim.SlimError, match="mismatch"):
        rccl_slim.prepare(src, root=root, strip=False)
    assert not os.path.exists(rccl_slim.entry_dir(src, root=root, strip=False))
    assert [n for n in os.listdir(root) if not n.startswith(".")] == []
    monkeypatch.setattr(rccl_slim, "verify", lambda entry, timeout=180.0: {"ok": True, "init_ms": 1.0,
                                                                          "mapped": [entry + "/librccl.so"]})
    meta = rccl_slim.prepare(src, root=root, strip=False)
    assert meta["verified"]["mapped"] and meta["dir"] == rccl_slim.entry_dir(src, root=root, strip=False)


def test_verify_child_without_gpu_reports_failure(tmp_path):
    """On a machine without a GPU the verification child fails (it never passes by default)."""
    src = _fake_runtime(tmp_path, _lib())
    meta = rccl_slim.prepare(src, root=str(tmp_path / "cache"), strip=False, verify_with_gpu=False)
    env = dict(os.environ, TK_FORCE_NO_GPU="1")
    with pytest.raises(rccl_slim.SlimError):
        old = os.environ.copy()
        try:
            os.environ.update(env)
            rccl_slim.verify(str(meta["dir"]), timeout=120)
        finally:
            os.environ.clear()
            os.environ.update(old)


def test_cli_reports_errors_as_json(tmp_path):
    p = subprocess.run([sys.executable, "-m", "triton_kubernetes_amd.ops.rccl_slim", "--source", str(tmp_path),
                        "--root", str(tmp_path / "c")], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert p.returncode == 1 and "librccl.so missing" in json.loads(p.stdout)["error"]


@pytest.mark.skipif(not rccl_slim.find_tool("clang-offload-bundler"), reason="no ROCm LLVM bundler")
def test_shell_form_matches_the_python_form(tmp_path):
    """terraform/scripts.py tk_rccl_slim (SSH / Terraform nodes) on a fake ROCm tree whose
    librccl carries a compressed 2-target bundle: one aligned gfx950 entry, soname aliases
    on the copy, cached on a re-run; no link anything loads by default."""
    from triton_kubernetes_amd.terraform.scripts import RCCL_SLIM_FN

    lib = _lib()
    _, _, orig = _section(lib)
    co = next(orig[o:o + s] for t, o, s in rccl_slim.parse_bundle(orig) if t == GFX950)
    for name, data in (("gfx950.co", co), ("other.co", co[::-1]), ("host", b"")):
        (tmp_path / name).write_bytes(data)
    targets = ",".join([rccl_slim.HOST_TRIPLE, rccl_slim.device_triple("gfx942"), GFX950])
    subprocess.run([rccl_slim.find_bundler(), "--compress", "--type=o", f"--targets={targets}",
                    f"--input={tmp_path / 'host'}", f"--input={tmp_path / 'other.co'}",
                    f"--input={tmp_path / 'gfx950.co'}", f"--output={tmp_path / 'fat.bin'}"], check=True,
                   capture_output=True)
    fat = (tmp_path / "fat.bin").read_bytes()
    rocm = tmp_path / "rocm"
    (rocm / "lib" / "llvm").mkdir(parents=True)
    os.symlink(os.path.dirname(rccl_slim.find_bundler()), rocm / "lib" / "llvm" / "bin")
    real = rocm / "lib" / "librccl.so.1.0.1"
    shutil.copyfile(lib, real)
    os.symlink("librccl.so.1.0.1", rocm / "lib" / "librccl.so")
    os.symlink("librccl.so.1.0.1", rocm / "lib" / "librccl.so.1")
    (rocm / "lib" / "libamdhip64.so.7").write_bytes(b"x")
    off, size, _ = _section(str(real))
    with open(real, "r+b") as fh:  # a compressed bundle shorter than its section
        fh.seek(off)
        fh.write(fat + b"\0" * (size - len(fat)))
    root = tmp_path / "cache"
    script = RCCL_SLIM_FN + f"\ntk_rccl_slim {root} {rocm}\n"
    p = subprocess.run(["bash", "-c", script], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    out = p.stdout.strip()
    assert not os.path.exists(root / "rocm")  # nothing points the node tools at it
    new_lib = os.path.join(out, "librccl.so")
    assert os.path.getsize(new_lib) == os.path.getsize(real)
    _, _, new = _section(new_lib)
    entries = [(t, o, s) for t, o, s in rccl_slim.parse_bundle(new) if s]
    assert [t for t, _, _ in entries] == [GFX950] and entries[0][1] % 4096 == 0
    assert new[entries[0][1]:entries[0][1] + 4] == b"\x7fELF"
    assert os.readlink(os.path.join(out, "librccl.so.1")) == "librccl.so"
    assert os.path.realpath(os.path.join(out, "libamdhip64.so.7")) == os.path.realpath(rocm / "lib" / "libamdhip64.so.7")
    assert json.loads(open(os.path.join(out, "slim.json"), encoding="utf-8").read())["form"] == "shell"
    again = subprocess.run(["bash", "-c", script], capture_output=True, text=True, timeout=120)
    assert again.returncode == 0 and again.stdout.strip() == out


def test_python_form_links_every_librccl_alias_to_the_copy(tmp_path):
    src = _fake_runtime(tmp_path, _lib())
    os.symlink("librccl.so", os.path.join(src, "librccl.so.1"))
    meta = rccl_slim.prepare(src, root=str(tmp_path / "cache"), strip=False, verify_with_gpu=False)
    assert os.readlink(os.path.join(meta["dir"], "librccl.so.1")) == "librccl.so"
    path = rccl_slim.link(str(tmp_path / "cache"), "rocm", str(meta["dir"]))
    assert os.path.realpath(path) == os.path.realpath(meta["dir"])


def test_gpu_cli_prepares_and_reports(tmp_path):
    src = _fake_runtime(tmp_path, _lib())
    p = subprocess.run([sys.executable, "-m", "triton_kubernetes_amd", "gpu", "rccl-slim", "--source", src, "--root",
                        str(tmp_path / "c"), "--no-verify"], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert p.returncode == 0, p.stderr
    meta = json.loads(p.stdout.strip().splitlines()[-1])
    assert os.path.exists(os.path.join(meta["dir"], "slim.json")) and meta["cached"] is False
    assert "verified" not in meta and rccl_slim.cached(src, root=str(tmp_path / "c")) == ""


def test_shell_enable_verifies_then_wraps_and_falls_back_when_stale(tmp_path):
    """The opt-in on SSH / Terraform nodes: the copy is enabled only after rccl-ready ran a
    one-rank all-reduce that mapped it; the wrapper uses it while the installed librccl is
    unchanged and falls back (with a warning) after a ROCm upgrade."""
    from triton_kubernetes_amd.terraform.scripts import RCCL_SLIM_ENABLE_FN

    rocm, tools, copy = tmp_path / "rocm", tmp_path / "bin", tmp_path / "copy"
    (rocm / "lib").mkdir(parents=True)
    tools.mkdir()
    copy.mkdir()
    (rocm / "lib" / "librccl.so").write_bytes(b"installed")
    (copy / "librccl.so").write_bytes(b"copy")
    # stand-in rccl-ready: prints the LD_LIBRARY_PATH it ran with; --expect-rccl passes only
    # when that library is first on the path (the real tool reads /proc/self/maps)
    (tools / "rccl-ready").write_text(
        '#!/bin/sh\nfor a in "$@"; do case $prev in --expect-rccl) exp=$a;; esac; prev=$a; done\n'
        'echo "LD=$LD_LIBRARY_PATH"\n'
        'if [ -n "$exp" ]; then [ "$(dirname "$exp")" = "${LD_LIBRARY_PATH%%:*}" ] && [ "$FAIL" != 1 ] || exit 1; fi\n')
    (tools / "rccl-ready").chmod(0o755)
    stub = f"tk_rccl_slim() {{ echo {copy}; }}\n"
    run = lambda extra_env=None: subprocess.run(  # noqa: E731
        ["bash", "-c", stub + RCCL_SLIM_ENABLE_FN + f"\ntk_rccl_slim_enable {tmp_path}/c {rocm} {tools}\n"],
        capture_output=True, text=True, timeout=60, env=dict(os.environ, **(extra_env or {})))
    p = run({"FAIL": "1"})
    assert p.returncode != 0 and "failed its one-rank verified all-reduce" in p.stderr
    assert not (tools / "rccl-ready-slim").exists() and not (tools / "rccl-slim.env").exists()
    p = run()
    assert p.returncode == 0, p.stderr
    assert (tools / "rccl-ready-slim").exists()
    env = dict(os.environ, ROCM_PATH=str(rocm))
    env.pop("LD_LIBRARY_PATH", None)
    w = subprocess.run([str(tools / "rccl-ready-slim"), "--ngpus", "8"], capture_output=True, text=True, env=env)
    assert w.returncode == 0 and w.stdout.strip() == f"LD={copy}"
    os.utime(rocm / "lib" / "librccl.so", ns=(10**9, 10**9))  # "upgraded"
    w = subprocess.run([str(tools / "rccl-ready-slim"), "--ngpus", "8"], capture_output=True, text=True, env=env)
    assert w.returncode == 0 and w.stdout.strip() == "LD=" and "librccl changed" in w.stderr
