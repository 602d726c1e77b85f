"""``.deb`` and ``.rpm`` packages written with the standard library.

The reference builds its release packages with ``fpm`` (``Makefile:43-79``:
``build-rpm`` / ``build-deb``, ``--depends jq``, then ``sha256-checksums.txt``).
``fpm`` is a Ruby gem that is not available here, so this module writes both formats
directly:

* **deb** -- an ``ar`` archive of ``debian-binary`` (``2.0``), ``control.tar.gz``
  (``control``, ``md5sums``) and ``data.tar.gz`` (``dpkg-deb --info/--contents`` read it);
* **rpm** -- the v3 lead, a signature header (``SIZE``, ``MD5``, ``PAYLOADSIZE``) and a
  main header (name/version/release/arch, file list as dirnames/basenames/dirindexes with
  sizes, modes, SHA-256 digests, owners, requires) followed by a gzip'd ``newc`` cpio
  payload.  :func:`read_rpm` parses them back (tests; no ``rpm`` binary here).

Two packages, like the two things a site installs:

* ``triton-kubernetes`` -- the CLI (single-file ``.pyz`` at ``/usr/bin/triton-kubernetes``);
* ``triton-kubernetes-node`` -- MI355X node tools: the gfx950 executables
  (``amdgpu-topo-labeller``, ``gpu-burnin``, ``rccl-ready``) under
  ``/opt/triton-kubernetes/bin``, their sources (for on-node rebuilds), the node agent
  (package + ``tk-node-agent.service``).
"""

import gzip
import hashlib
import io
import os
import stat
import struct
import tarfile
import time
from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple


@dataclass
class PkgFile:
    path: str  # absolute install path
    data: bytes
    mode: int = 0o644


@dataclass
class Package:
    name: str
    version: str  # upstream version, e.g. 0.8.2
    release: str = "1"
    arch: str = "amd64"  # deb name; rpm uses x86_64 / noarch
    summary: str = ""
    description: str = ""
    maintainer: str = "triton-kubernetes maintainers"
    url: str = ""
    license: str = "MPL-2.0"
    depends: List[str] = field(default_factory=list)
    files: List[PkgFile] = field(default_factory=list)
    mtime: int = 0  # reproducible builds: fixed timestamps (0 -> SOURCE_DATE_EPOCH or now)

    def when(self) -> int:
        return self.mtime or int(os.environ.get("SOURCE_DATE_EPOCH", time.time()))


# --- deb ------------------------------------------------------------------------------------------------
def _ar(members: Sequence[Tuple[str, bytes]], mtime: int) -> bytes:
    out = io.BytesIO()
    out.write(b"!<arch>\n")
    for name, data in members:
        hdr = f"{name:<16}{mtime:<12}{0:<6}{0:<6}{0o100644:<8o}{len(data):<10}`\n".encode()
        assert len(hdr) == 60
        out.write(hdr + data + (b"\n" if len(data) % 2 else b""))
    return out.getvalue()


def _tar_gz(entries: Sequence[Tuple[str, bytes, int]], mtime: int) -> bytes:
    raw = io.BytesIO()
    with tarfile.open(fileobj=raw, mode="w", format=tarfile.GNU_FORMAT) as tar:
        dirs = set()
        for path, _, _ in entries:
            parts = path.strip("./").split("/")[:-1]
            for i in range(1, len(parts) + 1):
                dirs.add("./" + "/".join(parts[:i]))
        for d in sorted(dirs):
            ti = tarfile.TarInfo(d)
            ti.type, ti.mode, ti.mtime, ti.uname, ti.gname = tarfile.DIRTYPE, 0o755, mtime, "root", "root"
            tar.addfile(ti)
        for path, data, mode in entries:
            ti = tarfile.TarInfo(path)
            ti.size, ti.mode, ti.mtime, ti.uname, ti.gname = len(data), mode, mtime, "root", "root"
            tar.addfile(ti, io.BytesIO(data))
    return gzip.compress(raw.getvalue(), mtime=mtime)


def build_deb(pkg: Package) -> bytes:
    mtime = pkg.when()
    size_kib = (sum(len(f.data) for f in pkg.files) + 1023) // 1024
    control = [f"Package: {pkg.name}", f"Version: {pkg.version}-{pkg.release}", f"Architecture: {pkg.arch}",
               f"Maintainer: {pkg.maintainer}", f"Installed-Size: {size_kib}"]
    if pkg.depends:
        control.append("Depends: " + ", ".join(pkg.depends))
    if pkg.url:
        control.append(f"Homepage: {pkg.url}")
    desc = pkg.description.strip().splitlines() or [""]
    control.append(f"Description: {pkg.summary}")
    control += [" " + (ln if ln.strip() else ".") for ln in desc if desc != [""]]
    md5sums = "".join(f"{hashlib.md5(f.data).hexdigest()}  {f.path.lstrip('/')}\n" for f in pkg.files)
    ctl = _tar_gz([("./control", ("\n".join(control) + "\n").encode(), 0o644),
                   ("./md5sums", md5sums.encode(), 0o644)], mtime)
    data = _tar_gz([("./" + f.path.lstrip("/"), f.data, f.mode) for f in pkg.files], mtime)
    return _ar([("debian-binary", b"2.0\n"), ("control.tar.gz", ctl), ("data.tar.gz", data)], mtime)


# --- rpm ------------------------------------------------------------------------------------------------
# header tag types
_INT16, _INT32, _STRING, _BIN, _STRING_ARRAY, _I18N = 3, 4, 6, 7, 8, 9
RPM_TAGS = {
    "NAME": 1000, "VERSION": 1001, "RELEASE": 1002, "SUMMARY": 1004, "DESCRIPTION": 1005, "BUILDTIME": 1006,
    "SIZE": 1009, "LICENSE": 1014, "GROUP": 1016, "URL": 1020, "OS": 1021, "ARCH": 1022,
    "FILESIZES": 1028, "FILEMODES": 1030, "FILERDEVS": 1033, "FILEMTIMES": 1034, "FILEDIGESTS": 1035,
    "FILELINKTOS": 1036, "FILEFLAGS": 1037, "FILEUSERNAME": 1039, "FILEGROUPNAME": 1040,
    "REQUIREFLAGS": 1048, "REQUIRENAME": 1049, "REQUIREVERSION": 1050, "FILEINODES": 1096,
    "FILELANGS": 1097, "DIRINDEXES": 1116, "BASENAMES": 1117, "DIRNAMES": 1118,
    "PAYLOADFORMAT": 1124, "PAYLOADCOMPRESSOR": 1125, "PAYLOADFLAGS": 1126, "FILEDIGESTALGO": 5011,
}
SIG_SIZE, SIG_MD5, SIG_PAYLOADSIZE, SIG_SHA256 = 1000, 1004, 1007, 273
_HEADER_MAGIC = b"\x8e\xad\xe8\x01\x00\x00\x00\x00"


def _header(entries: List[Tuple[int, int, object]], region_tag: int = 63) -> bytes:
    """An rpm header structure (index + data store), with the immutable-region trailer."""
    index, store = [], bytearray()
    align = {_INT16: 2, _INT32: 4}

    def put(tag: int, typ: int, value: object) -> None:
        a = align.get(typ, 1)
        while len(store) % a:
            store.append(0)
        off = len(store)
        if typ == _INT32:
            vals = list(value) if isinstance(value, (list, tuple)) else [value]
            store.extend(struct.pack(f">{len(vals)}i", *vals))
            count = len(vals)
        elif typ == _INT16:
            vals = list(value) if isinstance(value, (list, tuple)) else [value]
            store.extend(struct.pack(f">{len(vals)}H", *[v & 0xFFFF for v in vals]))
            count = len(vals)
        elif typ in (_STRING, _I18N):
            store.extend(str(value).encode() + b"\0")
            count = 1
        elif typ == _STRING_ARRAY:
            for v in value:  # type: ignore[union-attr]
                store.extend(str(v).encode() + b"\0")
            count = len(value)  # type: ignore[arg-type]
        elif typ == _BIN:
            store.extend(value)  # type: ignore[arg-type]
            count = len(value)  # type: ignore[arg-type]
        else:
            raise ValueError(typ)
        index.append((tag, typ, off, count))

    for tag, typ, value in entries:
        put(tag, typ, value)
    # region trailer: a negative offset covering the whole index (rpm >= 4 expects it)
    n = len(index) + 1
    trailer = struct.pack(">iiii", region_tag, _BIN, -16 * n, 16)
    region_off = len(store)
    store.extend(trailer)
    idx = [struct.pack(">iiii", region_tag, _BIN, region_off, 16)]
    idx += [struct.pack(">iiii", t, ty, o, c) for t, ty, o, c in index]
    return _HEADER_MAGIC + struct.pack(">ii", n, len(store)) + b"".join(idx) + bytes(store)


def _cpio_newc(entries: Sequence[Tuple[str, bytes, int, int]]) -> bytes:
    out = io.BytesIO()

    def rec(name: str, data: bytes, mode: int, mtime: int, ino: int, nlink: int = 1) -> None:
        nb = name.encode() + b"\0"
        hdr = "070701" + "".join(f"{v:08x}" for v in (ino, mode, 0, 0, nlink, mtime, len(data), 0, 0, 0, 0,
                                                           len(nb), 0))
        out.write(hdr.encode() + nb)
        out.write(b"\0" * ((4 - (110 + len(nb)) % 4) % 4))
        out.write(data)
        out.write(b"\0" * ((4 - len(data) % 4) % 4))

    for i, (name, data, mode, mtime) in enumerate(entries, 1):
        rec(name, data, mode, mtime, i)
    rec("TRAILER!!!", b"", 0, 0, 0)
    return out.getvalue()


def build_rpm(pkg: Package) -> bytes:
    mtime = pkg.when()
    arch = {"amd64": "x86_64", "all": "noarch"}.get(pkg.arch, pkg.arch)
    files = sorted(pkg.files, key=lambda f: f.path)
    dirs: List[str] = []
    dirindex, basenames = [], []
    for f in files:
        d, b = os.path.dirname(f.path) + "/", os.path.basename(f.path)
        if d not in dirs:
            dirs.append(d)
        dirindex.append(dirs.index(d))
        basenames.append(b)
    payload = gzip.compress(_cpio_newc([("." + f.path, f.data, stat.S_IFREG | f.mode, mtime) for f in files]),
                            mtime=mtime)
    reqs = [r.split()[0] for r in pkg.depends]
    n = len(files)
    main = [
        (RPM_TAGS["NAME"], _STRING, pkg.name), (RPM_TAGS["VERSION"], _STRING, pkg.version),
        (RPM_TAGS["RELEASE"], _STRING, pkg.release), (RPM_TAGS["SUMMARY"], _I18N, pkg.summary),
        (RPM_TAGS["DESCRIPTION"], _I18N, pkg.description.strip() or pkg.summary),
        (RPM_TAGS["BUILDTIME"], _INT32, mtime), (RPM_TAGS["SIZE"], _INT32, sum(len(f.data) for f in files)),
        (RPM_TAGS["LICENSE"], _STRING, pkg.license), (RPM_TAGS["GROUP"], _I18N, "Applications/System"),
        (RPM_TAGS["URL"], _STRING, pkg.url or "https://example.invalid"),
        (RPM_TAGS["OS"], _STRING, "linux"), (RPM_TAGS["ARCH"], _STRING, arch),
        (RPM_TAGS["FILESIZES"], _INT32, [len(f.data) for f in files]),
        (RPM_TAGS["FILEMODES"], _INT16, [stat.S_IFREG | f.mode for f in files]),
        (RPM_TAGS["FILERDEVS"], _INT16, [0] * n), (RPM_TAGS["FILEMTIMES"], _INT32, [mtime] * n),
        (RPM_TAGS["FILEDIGESTS"], _STRING_ARRAY, [hashlib.sha256(f.data).hexdigest() for f in files]),
        (RPM_TAGS["FILELINKTOS"], _STRING_ARRAY, [""] * n), (RPM_TAGS["FILEFLAGS"], _INT32, [0] * n),
        (RPM_TAGS["FILEUSERNAME"], _STRING_ARRAY, ["root"] * n),
        (RPM_TAGS["FILEGROUPNAME"], _STRING_ARRAY, ["root"] * n),
    ]
    if reqs:
        main += [(RPM_TAGS["REQUIREFLAGS"], _INT32, [0] * len(reqs)),
                 (RPM_TAGS["REQUIRENAME"], _STRING_ARRAY, reqs),
                 (RPM_TAGS["REQUIREVERSION"], _STRING_ARRAY, [""] * len(reqs))]
    main += [
        (RPM_TAGS["FILEINODES"], _INT32, list(range(1, n + 1))), (RPM_TAGS["FILELANGS"], _STRING_ARRAY, [""] * n),
        (RPM_TAGS["DIRINDEXES"], _INT32, dirindex), (RPM_TAGS["BASENAMES"], _STRING_ARRAY, basenames),
        (RPM_TAGS["DIRNAMES"], _STRING_ARRAY, dirs), (RPM_TAGS["PAYLOADFORMAT"], _STRING, "cpio"),
        (RPM_TAGS["PAYLOADCOMPRESSOR"], _STRING, "gzip"), (RPM_TAGS["PAYLOADFLAGS"], _STRING, "9"),
        (RPM_TAGS["FILEDIGESTALGO"], _INT32, 8),  # PGPHASHALGO_SHA256
    ]
    header = _header(sorted(main, key=lambda e: e[0]))
    sig = _header(sorted([(SIG_SIZE, _INT32, len(header) + len(payload)),
                          (SIG_SHA256, _STRING, hashlib.sha256(header).hexdigest()),
                          (SIG_MD5, _BIN, hashlib.md5(header + payload).digest()),
                          (SIG_PAYLOADSIZE, _INT32, len(gzip.decompress(payload)))], key=lambda e: e[0]),
                  region_tag=62)
    sig += b"\0" * ((8 - len(sig) % 8) % 8)
    name = f"{pkg.name}-{pkg.version}-{pkg.release}".encode()[:65]
    lead = struct.pack(">4sBBhh66shh16s", b"\xed\xab\xee\xdb", 3, 0, 0, 1, name.ljust(66, b"\0"), 1, 5, b"\0" * 16)
    return lead + sig + header + payload


def _parse_header(buf: bytes, pos: int) -> Tuple[Dict[int, object], int]:
    if buf[pos:pos + 8] != _HEADER_MAGIC:
        raise ValueError(f"bad header magic at {pos}")
    n, size = struct.unpack_from(">ii", buf, pos + 8)
    idx_at, store_at = pos + 16, pos + 16 + 16 * n
    tags: Dict[int, object] = {}
    for i in range(n):
        tag, typ, off, count = struct.unpack_from(">iiii", buf, idx_at + 16 * i)
        at = store_at + off
        if typ == _INT32:
            v: object = list(struct.unpack_from(f">{count}i", buf, at))
        elif typ == _INT16:
            v = list(struct.unpack_from(f">{count}H", buf, at))
        elif typ in (_STRING, _I18N):
            v = buf[at:buf.index(b"\0", at)].decode()
        elif typ == _STRING_ARRAY:
            vals, p = [], at
            for _ in range(count):
                e = buf.index(b"\0", p)
                vals.append(buf[p:e].decode())
                p = e + 1
            v = vals
        else:
            v = bytes(buf[at:at + count])
        tags[tag] = v
    return tags, store_at + size


def read_rpm(data: bytes) -> Dict[str, object]:
    """Parse a package written by :func:`build_rpm` (lead, signature, header, payload)."""
    if data[:4] != b"\xed\xab\xee\xdb":
        raise ValueError("not an rpm")
    sig, end = _parse_header(data, 96)
    end += (8 - end % 8) % 8
    hdr, hend = _parse_header(data, end)
    payload = gzip.decompress(data[hend:])
    files, p = {}, 0
    while True:
        h = payload[p:p + 110].decode()
        namesize, filesize = int(h[94:102], 16), int(h[54:62], 16)
        name = payload[p + 110:p + 110 + namesize - 1].decode()
        p += 110 + namesize
        p += (4 - p % 4) % 4
        if name == "TRAILER!!!":
            break
        files[name.lstrip(".")] = (payload[p:p + filesize], int(h[14:22], 16))
        p += filesize
        p += (4 - p % 4) % 4
    inv = {v: k for k, v in RPM_TAGS.items()}
    return {"signature": sig, "header": {inv.get(k, k): v for k, v in hdr.items()}, "files": files,
            "header_bytes": data[end:hend], "payload": data[hend:]}


def write_checksums(paths: Sequence[str], out: str) -> str:
    lines = []
    for p in sorted(paths):
        with open(p, "rb") as fh:
            lines.append(f"{hashlib.sha256(fh.read()).hexdigest()}  {os.path.basename(p)}\n")
    with open(out, "w", encoding="utf-8") as fh:
        fh.writelines(lines)
    return out


def tree_files(src_dir: str, dest: str, mode_for=None) -> List[PkgFile]:
    out = []
    for root, dirs, names in os.walk(src_dir):
        dirs[:] = sorted(d for d in dirs if d != "__pycache__")
        for n in sorted(names):
            if n.endswith((".pyc", ".so.part")):
                continue
            full = os.path.join(root, n)
            if os.path.islink(full) and not os.path.exists(full):
                continue
            with open(full, "rb") as fh:
                data = fh.read()
            rel = os.path.relpath(full, src_dir)
            mode = mode_for(rel) if mode_for else (0o755 if os.access(full, os.X_OK) else 0o644)
            out.append(PkgFile(os.path.join(dest, rel), data, mode))
    return out


__all__ = ["Package", "PkgFile", "build_deb", "build_rpm", "read_rpm", "write_checksums", "tree_files"]
