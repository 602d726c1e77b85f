"""Single-target RCCL for a node's cold communicator init.

Why.  A fresh process's first RCCL communicator init on MI355X is dominated by
loading RCCL's device code, not by the init itself (``profiles/round2/
cold_rccl_init.md``): ``librccl.so`` carries its kernels for every GPU target
(13 on the PyTorch-ROCm build) as ONE compressed offload bundle (``CCOB``), and
the HIP runtime decompresses the whole bundle to find the gfx950 code object the
first time a kernel is touched.  Every node agent, every ``rccl-ready`` gate and
every cold create pays that again.

What.  :func:`prepare` makes, once per node and per RCCL build, a copy of
``librccl.so`` whose ``.hip_fatbin`` section holds an UNCOMPRESSED bundle with only
the node's target (gfx950).  The section keeps its address and size (the new
bundle is smaller and zero-padded), so nothing else in the ELF moves; the HIP
runtime then maps the gfx950 code object straight out of the file.  The other
libraries of the source directory are symlinked next to it (``librccl.so`` finds
its dependencies through ``$ORIGIN``), so the directory is a drop-in runtime for
``ops/native.py:select_runtime``.

Opt-in.  The copy is a modified vendor binary, so nothing uses it by default: the
node tools and agents load ``/opt/rocm/lib/librccl.so``.  A node opts in with
``rccl_slim = "on"`` (MI355X host module / node plan) or ``TK_HIP_RUNTIME=slim``
(agent), and an entry is only ever used after :func:`verify` ran a one-rank
all-reduce on it in a fresh process, checked the result and checked that the process
really mapped the copy (``slim.json`` ``verified``).

Cache.  ``$TK_RCCL_SLIM_DIR`` (default ``/var/lib/triton-kubernetes/rccl-slim``
when writable, else ``~/.cache/triton-kubernetes/rccl-slim``), one subdirectory
per source build (keyed by path, size, mtime and a hash of its first MiB).  A
finished entry holds ``slim.json``; a partial one is never used.

The compressed bundle is unpacked with ``clang-offload-bundler`` from the ROCm
LLVM toolchain (``/opt/rocm/lib/llvm/bin`` or ``/opt/rocm/llvm/bin``); an
already-uncompressed bundle is split here without it.
"""

import hashlib
import json
import os
import shutil
import struct
import subprocess
import tempfile
import time
from typing import Dict, List, Optional, Tuple

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
COMPRESSED_MAGIC = b"CCOB"
HOST_TRIPLE = "host-x86_64-unknown-linux-gnu-"
ALIGN = 4096
_BUNDLER_DIRS = ("/opt/rocm/lib/llvm/bin", "/opt/rocm/llvm/bin")


class SlimError(RuntimeError):
    pass


def device_triple(arch: str = "gfx950") -> str:
    return f"hipv4-amdgcn-amd-amdhsa--{arch}"


def cache_root() -> str:
    env = os.environ.get("TK_RCCL_SLIM_DIR")
    if env:
        return env
    system = "/var/lib/triton-kubernetes/rccl-slim"
    parent = os.path.dirname(system)
    if os.access(parent, os.W_OK) or (not os.path.exists(parent) and os.access(os.path.dirname(parent), os.W_OK)):
        return system
    return os.path.join(os.path.expanduser("~"), ".cache", "triton-kubernetes", "rccl-slim")


def elf_section(path: str, name: str) -> Tuple[int, int]:
    """(file offset, size) of section ``name`` in the ELF64 little-endian file ``path``."""
    with open(path, "rb") as fh:
        ident = fh.read(64)
        if ident[:4] != b"\x7fELF" or ident[4] != 2 or ident[5] != 1:
            raise SlimError(f"{path}: not an ELF64 little-endian file")
        e_shoff, = struct.unpack_from("<Q", ident, 0x28)
        e_shentsize, e_shnum, e_shstrndx = struct.unpack_from("<HHH", ident, 0x3A)
        fh.seek(e_shoff)
        table = fh.read(e_shentsize * e_shnum)
        shdrs = [struct.unpack_from("<IIQQQQIIQQ", table, i * e_shentsize) for i in range(e_shnum)]
        str_off, str_size = shdrs[e_shstrndx][4], shdrs[e_shstrndx][5]
        fh.seek(str_off)
        strtab = fh.read(str_size)
    for sh_name, sh_type, _flags, _addr, sh_offset, sh_size, *_ in shdrs:
        end = strtab.index(b"\0", sh_name)
        if strtab[sh_name:end].decode() == name:
            if sh_type == 8:  # SHT_NOBITS: no file bytes to rewrite
                raise SlimError(f"{path}: section {name} has no file contents")
            return sh_offset, sh_size
    raise SlimError(f"{path}: no {name} section")


def parse_bundle(data: bytes) -> List[Tuple[str, int, int]]:
    """Entries (triple, offset, size) of an uncompressed offload bundle."""
    if not data.startswith(BUNDLE_MAGIC):
        raise SlimError("not an uncompressed offload bundle")
    n, = struct.unpack_from("<Q", data, len(BUNDLE_MAGIC))
    pos = len(BUNDLE_MAGIC) + 8
    out = []
    for _ in range(n):
        off, size, tlen = struct.unpack_from("<QQQ", data, pos)
        pos += 24
        triple = data[pos:pos + tlen].decode()
        pos += tlen
        out.append((triple, off, size))
    return out


def bundle_layout(entries: List[Tuple[str, int]]) -> Tuple[bytes, List[int], int]:
    """Header bytes, payload offsets and total size of an uncompressed offload bundle whose
    entries are (triple, payload size); payloads 4 KiB aligned (as hipcc lays them out)."""
    header_len = len(BUNDLE_MAGIC) + 8 + sum(24 + len(t.encode()) for t, _ in entries)
    offsets, pos = [], header_len
    for _, n in entries:
        if n:
            pos = (pos + ALIGN - 1) // ALIGN * ALIGN
        offsets.append(pos)
        pos += n
    head = bytearray(BUNDLE_MAGIC + struct.pack("<Q", len(entries)))
    for (triple, n), off in zip(entries, offsets):
        t = triple.encode()
        head += struct.pack("<QQQ", off if n else 0, n, len(t)) + t
    return bytes(head), offsets, pos


def make_bundle(entries: List[Tuple[str, bytes]]) -> bytes:
    """Uncompressed offload bundle of ``entries`` (triple, payload) in memory."""
    head, offsets, total = bundle_layout([(t, len(p)) for t, p in entries])
    buf = bytearray(total)
    buf[:len(head)] = head
    for (_, payload), off in zip(entries, offsets):
        buf[off:off + len(payload)] = payload
    return bytes(buf)


def _copy_range(src: str, offset: int, length: int, dst: str) -> None:
    with open(src, "rb") as fi, open(dst, "wb") as fo:
        fi.seek(offset)
        while length > 0:
            chunk = fi.read(min(length, 16 << 20))
            if not chunk:
                raise SlimError(f"{src}: short read")
            fo.write(chunk)
            length -= len(chunk)


def find_tool(name: str) -> str:
    """``name`` from the ROCm LLVM toolchain (then PATH), or ``""``."""
    for d in _BUNDLER_DIRS:
        cand = os.path.join(d, name)
        if os.access(cand, os.X_OK):
            return cand
    return shutil.which(name) or ""


def find_bundler() -> str:
    exe = find_tool("clang-offload-bundler")
    if not exe:
        raise SlimError("clang-offload-bundler not found (ROCm LLVM toolchain)")
    return exe


def strip_debug(src: str, dst: str) -> bool:
    """``llvm-objcopy --strip-debug src dst``; False (nothing written) when the tool is
    missing.  RCCL's gfx950 code object is 277 MB of which 50 MB load onto the GPU; the rest
    is DWARF the runtime would read for nothing (only a GPU debugger uses it, and none runs
    on a gated node)."""
    tool = find_tool("llvm-objcopy")
    if not tool:
        return False
    run = subprocess.run([tool, "--strip-debug", src, dst], capture_output=True, text=True, check=False)
    if run.returncode != 0:
        raise SlimError(f"llvm-objcopy --strip-debug: {run.stderr.strip()}")
    return True


def compressed_size(head: bytes, section_size: int) -> int:
    """Bytes of the compressed bundle starting a ``section_size`` byte section (which may be
    padded past it), from its header ``head``: magic, u16 version, u16 method, then the
    total size as u32 (v2) or u64 (v3); v1 has none, so the whole section is the bundle."""
    version, = struct.unpack_from("<H", head, 4)
    if version == 2:
        total, = struct.unpack_from("<I", head, 8)
    elif version >= 3:
        total, = struct.unpack_from("<Q", head, 8)
    else:
        return section_size
    if not 16 <= total <= section_size:
        raise SlimError(f"compressed bundle header gives {total} bytes in a {section_size} byte section")
    return total


def extract_code_object(lib: str, offset: int, size: int, arch: str, dst: str) -> None:
    """Write the ``arch`` code object of the (compressed or plain) offload bundle at
    ``lib[offset:offset+size]`` to ``dst``, streaming (the sections run to 0.5 GB)."""
    triple = device_triple(arch)
    with open(lib, "rb") as fh:
        fh.seek(offset)
        head = fh.read(min(size, 1 << 16))
    if head.startswith(BUNDLE_MAGIC):
        for t, off, n in parse_bundle(head):
            if t == triple:
                _copy_range(lib, offset + off, n, dst)
                break
        else:
            raise SlimError(f"bundle has no {triple} entry")
    elif head.startswith(COMPRESSED_MAGIC):
        src = dst + ".fatbin"
        _copy_range(lib, offset, compressed_size(head, size), src)
        try:
            run = subprocess.run([find_bundler(), "--unbundle", "--type=o", f"--input={src}", f"--targets={triple}",
                                  f"--output={dst}"], capture_output=True, text=True, check=False)
        finally:
            os.unlink(src)
        if run.returncode != 0:
            # (a target the bundle lacks fails here: "Can't find bundles for ...")
            raise SlimError(f"clang-offload-bundler --unbundle {triple}: {run.stderr.strip()}")
    else:
        raise SlimError("unknown .hip_fatbin format")
    with open(dst, "rb") as fh:
        if fh.read(4) != b"\x7fELF":
            raise SlimError(f"extracted {triple} code object is not an ELF file")


def source_key(lib: str) -> str:
    st = os.stat(lib)
    h = hashlib.sha256(f"{os.path.realpath(lib)}|{st.st_size}|{st.st_mtime_ns}".encode())
    with open(lib, "rb") as fh:
        h.update(fh.read(1 << 20))
    return h.hexdigest()[:20]


def entry_dir(src_dir: str, arch: str = "gfx950", root: Optional[str] = None, strip: bool = True) -> str:
    key = source_key(os.path.join(src_dir, "librccl.so"))
    return os.path.join(root or cache_root(), f"{arch}-{key}" + ("" if strip else "-debug"))


def _meta(d: str) -> Dict[str, object]:
    try:
        with open(os.path.join(d, "slim.json"), "r", encoding="utf-8") as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return {}


def cached(src_dir: str, arch: str = "gfx950", root: Optional[str] = None) -> str:
    """The finished *and verified* slim runtime directory for ``src_dir``, or ``""``
    (keyed by the current source library: a ROCm upgrade never reuses an old copy)."""
    try:
        d = entry_dir(src_dir, arch, root)
    except OSError:
        return ""
    return d if _meta(d).get("verified") else ""


VERIFY_BYTES = 4 << 20


def verify(entry: str, timeout: float = 180.0) -> Dict[str, object]:
    """One-rank verified all-reduce against the copy in ``entry``, in a fresh process
    (``TK_HIP_RUNTIME=<entry>``): the child must map ``<entry>/librccl.so`` and the
    all-reduce result must check.  Raises :class:`SlimError` otherwise."""
    import sys

    env = dict(os.environ, TK_HIP_RUNTIME=entry)
    try:
        proc = subprocess.run([sys.executable, "-m", "triton_kubernetes_amd.ops.rccl_slim", "--verify-child", entry],
                              capture_output=True, text=True, timeout=timeout, env=env,
                              cwd=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    except subprocess.TimeoutExpired as exc:
        raise SlimError(f"verifying {entry}: timed out after {timeout:.0f} s") from exc
    line = (proc.stdout.strip().splitlines() or [""])[-1]
    try:
        res = json.loads(line)
    except ValueError:
        res = {}
    if proc.returncode != 0 or not res.get("ok"):
        raise SlimError(f"verifying {entry} failed (exit {proc.returncode}): "
                        f"{res.get('error') or proc.stderr.strip()[-400:]}")
    return res


def _verify_child(entry: str) -> int:
    """Child side of :func:`verify` (the runtime was selected from ``TK_HIP_RUNTIME``)."""
    out: Dict[str, object] = {"entry": entry}
    try:
        from . import native, rccl

        native.runtime_dir()
        res = rccl.sweep_local(1, sizes=(VERIFY_BYTES,), iters=2, warmup=1)
        with open("/proc/self/maps", "r", encoding="utf-8") as fh:
            maps = {ln.split()[-1] for ln in fh if "librccl" in ln and "/" in ln}
        want = os.path.realpath(os.path.join(entry, "librccl.so"))
        mapped = sorted(maps)
        out.update(allreduce_ok=res.ok, errors=res.errors, init_ms=round(res.init_ms, 3), mapped=mapped,
                   ok=res.ok and any(os.path.realpath(m) == want for m in mapped))
        if res.ok and not out["ok"]:
            out["error"] = f"the process mapped {mapped}, not {want}"
    except Exception as exc:  # noqa: BLE001 - reported to the parent
        out.update(ok=False, error=f"{type(exc).__name__}: {exc}")
    print(json.dumps(out), flush=True)
    return 0 if out.get("ok") else 1


def _record_verified(d: str, result: Dict[str, object]) -> Dict[str, object]:
    meta = _meta(d)
    meta["verified"] = {"time": time.time(), "init_ms": result.get("init_ms"), "mapped": result.get("mapped")}
    tmp = os.path.join(d, f".slim.json.{os.getpid()}")
    with open(tmp, "w", encoding="utf-8") as fh:
        json.dump(meta, fh, indent=1)
    os.replace(tmp, os.path.join(d, "slim.json"))
    return meta


def prepare(src_dir: str, arch: str = "gfx950", root: Optional[str] = None, strip: bool = True,
            verify_with_gpu: bool = True) -> Dict[str, object]:
    """Build (or find) the slim runtime directory for the RCCL in ``src_dir`` and (unless
    ``verify_with_gpu`` is False — CPU tests of the ELF surgery) :func:`verify` it before
    it may be used.

    Returns the entry's metadata (``dir``, sizes, ``prepare_s``; ``cached`` True when it
    already existed).  Raises :class:`SlimError` when the library cannot be slimmed or
    the copy fails verification (the entry is then removed)."""
    t0 = time.perf_counter()
    lib = os.path.join(src_dir, "librccl.so")
    if not os.path.exists(lib):
        raise SlimError(f"{lib} missing")
    out = entry_dir(src_dir, arch, root, strip)
    meta_path = os.path.join(out, "slim.json")
    if os.path.exists(meta_path):
        meta = _meta(out)
        if verify_with_gpu and not meta.get("verified"):
            try:
                meta = _record_verified(out, verify(out))
            except SlimError:
                shutil.rmtree(out, ignore_errors=True)
                raise
        meta["cached"] = True
        return meta
    real = os.path.realpath(lib)
    offset, size = elf_section(real, ".hip_fatbin")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = tempfile.mkdtemp(prefix=os.path.basename(out) + ".tmp-", dir=os.path.dirname(out))
    os.chmod(tmp, 0o755)  # agents may run as another user than the one that prepared it
    try:
        full, stripped = os.path.join(tmp, "full.co"), os.path.join(tmp, "stripped.co")
        extract_code_object(real, offset, size, arch, full)
        full_bytes = os.path.getsize(full)
        co_path = stripped if strip and strip_debug(full, stripped) else full
        co_bytes = os.path.getsize(co_path)
        head, offsets, total = bundle_layout([(HOST_TRIPLE, 0), (device_triple(arch), co_bytes)])
        if total > size:
            raise SlimError(f"{arch} code object ({co_bytes} B) does not fit the {size} B .hip_fatbin section")
        dst = os.path.join(tmp, "librccl.so")
        shutil.copyfile(real, dst)
        with open(dst, "r+b") as fo, open(co_path, "rb") as fi:
            fo.seek(offset)
            fo.write(head)
            fo.write(b"\0" * (offsets[1] - len(head)))
            shutil.copyfileobj(fi, fo, 16 << 20)
            fo.write(b"\0" * (size - total))
        for p in (full, stripped):
            if os.path.exists(p):
                os.unlink(p)
        os.chmod(dst, 0o755)
        # the rest of the runtime: librccl resolves libamdhip64 & co. through $ORIGIN
        for name in sorted(os.listdir(src_dir)):
            if not name.startswith("lib") or ".so" not in name or name == "librccl.so":
                continue
            # every soname / version alias of librccl is the copy (an executable's NEEDED
            # librccl.so.1 resolves here through RUNPATH or LD_LIBRARY_PATH)
            target = "librccl.so" if name.startswith("librccl.so") else os.path.realpath(os.path.join(src_dir, name))
            os.symlink(target, os.path.join(tmp, name))
        with open(real, "rb") as fh:
            fh.seek(offset)
            fmt = "compressed" if fh.read(4) == COMPRESSED_MAGIC else "bundle"
        meta = {"dir": out, "source": real, "arch": arch, "source_fatbin_bytes": size, "source_format": fmt,
                "code_object_bytes": full_bytes, "loaded_code_object_bytes": co_bytes,
                "debug_stripped": co_bytes < full_bytes, "bundle_bytes": total,
                "prepare_s": round(time.perf_counter() - t0, 3)}
        with open(os.path.join(tmp, "slim.json"), "w", encoding="utf-8") as fh:
            json.dump(meta, fh, indent=1)
        if verify_with_gpu:  # before the entry exists under its final name
            meta = _record_verified(tmp, verify(tmp))
            meta["dir"] = out
        try:
            os.rename(tmp, out)
        except OSError:
            if not os.path.exists(meta_path):  # lost a race to a finished entry: use it
                raise
            shutil.rmtree(tmp, ignore_errors=True)
        meta["cached"] = False
        return meta
    except BaseException:
        shutil.rmtree(tmp, ignore_errors=True)
        raise


def link(root: str, name: str, target: str) -> str:
    """Point ``root/name`` at ``target`` atomically (``rocm``: the entry the node tools'
    RUNPATH names)."""
    path = os.path.join(root, name)
    tmp = f"{path}.tmp-{os.getpid()}"
    os.symlink(target, tmp)
    os.replace(tmp, path)
    return path


def main(argv=None) -> int:
    import argparse

    ap = argparse.ArgumentParser(description="Prepare the single-target (gfx950) RCCL runtime directory")
    ap.add_argument("--source", default="", help="directory holding librccl.so (default: /opt/rocm/lib)")
    ap.add_argument("--arch", default="gfx950")
    ap.add_argument("--root", default="", help="cache root (default: TK_RCCL_SLIM_DIR or the node default)")
    ap.add_argument("--no-verify", action="store_true", help="skip the GPU verification (the copy is then unusable)")
    ap.add_argument("--verify-child", default="", help=argparse.SUPPRESS)
    args = ap.parse_args(argv)
    if args.verify_child:
        return _verify_child(args.verify_child)
    from .native import SYSTEM_LIB_DIR

    sources = [args.source or (SYSTEM_LIB_DIR if os.path.exists(SYSTEM_LIB_DIR) else "")]
    if not any(sources):
        print(json.dumps({"error": "no RCCL source directory (pass --source)"}))
        return 2
    rc = 0
    for src in sources:
        try:
            meta = prepare(src, args.arch, args.root or None, verify_with_gpu=not args.no_verify)
            if os.path.realpath(src) == os.path.realpath(SYSTEM_LIB_DIR):
                meta["link"] = link(os.path.dirname(str(meta["dir"])), "rocm", str(meta["dir"]))
        except (SlimError, OSError) as exc:
            meta, rc = {"source": src, "error": str(exc)}, 1
        print(json.dumps(meta))
    return rc


if __name__ == "__main__":
    raise SystemExit(main())
