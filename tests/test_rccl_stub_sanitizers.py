"""The libtk_rccl ABI stub (``ops/csrc/tk_rccl_stub.cpp``) under ASan/UBSan and TSan.

The stub is threaded host C++ (gate table, sweeping set, cancel flag, file rendezvous),
and the CPU dry runs of the 8-GPU gate rest on it (``tests/test_gate_stub.py``,
``bench.py --sim-gpu``).  Here a small driver links the stub's source and drives the C ABI
from eight threads -- one world of eight ranks, a cancel while a sweep waits for peers, a
world mismatch and a double claim -- built once with AddressSanitizer + UBSan and once
with ThreadSanitizer.  Either build must run clean (sanitizers on host code).
"""

import os
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "triton_kubernetes_amd", "ops",
                    "csrc")

DRIVER = r"""
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

extern "C" {
int tkr_unique_id(unsigned char* out128);
const char* tkr_last_error();
int tkr_gate_begin_ex(const unsigned char*, int, int, int, const int*, int, size_t);
int tkr_gate_cancel(int);
int tkr_gate_pending();
int tkr_gate_sweep(int, const size_t*, int, int, int, int, double, double*, double*, double*, double*, double*);
int tkr_elf_kernel_symbol(const char* path, char* out, int cap);
int tkr_gate_poll(int);
}

static int sweep(int h, double timeout_ms, double* err_out) {
  const size_t sizes[2] = {1 << 10, 1 << 20};
  double t[2], a[2], b[2], e[2], ph[5] = {0, 0, 0, 0, 0};
  const int rc = tkr_gate_sweep(h, sizes, 2, 5, 1, /*f32*/ 0, timeout_ms, t, a, b, e, ph);
  *err_out = e[0] + e[1];
  return rc;
}

int main(int argc, char** argv) {
  int failures = 0;
  // 0. the preload's ELF scan (tk_elf_scan.h) over every file given: librccl builds, other
  //    ELF files, truncated and corrupted ones -- bounds-checked, never a read past the map
  for (int i = 1; i < argc; ++i) {
    char name[512];
    const int n = tkr_elf_kernel_symbol(argv[i], name, sizeof(name));
    std::printf("scan %s -> %d %s\n", argv[i], n, n ? name : "-");
  }
  // 1. one world of eight ranks, one thread each (the node agent's shape, ndev = 1 per thread)
  unsigned char uid[128];
  if (tkr_unique_id(uid)) return 10;
  std::vector<int> rcs(8, -99);
  std::vector<double> errs(8, -1);
  std::vector<std::thread> ts;
  for (int r = 0; r < 8; ++r)
    ts.emplace_back([&, r] {
      const int dev = r;
      const int h = tkr_gate_begin_ex(uid, 8, r, 1, &dev, 0, 0);
      rcs[r] = h < 0 ? h : sweep(h, 30000.0, &errs[r]);
    });
  for (auto& t : ts) t.join();
  for (int r = 0; r < 8; ++r)
    if (rcs[r] != 0 || errs[r] != 0.0) { std::printf("rank %d rc %d errs %g\n", r, rcs[r], errs[r]); ++failures; }

  // 2. a sweep waiting for an absent peer is canceled from another thread
  unsigned char uid2[128];
  if (tkr_unique_id(uid2)) return 11;
  const int dev0 = 0;
  const int h = tkr_gate_begin_ex(uid2, 2, 0, 1, &dev0, 0, 0);
  double e2 = 0;
  int rc2 = -99;
  std::thread waiter([&] { rc2 = sweep(h, 60000.0, &e2); });
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  while (tkr_gate_cancel(h) != 0) std::this_thread::sleep_for(std::chrono::milliseconds(5));
  waiter.join();
  if (rc2 != -4) { std::printf("cancel rc %d\n", rc2); ++failures; }

  // 3. one world size per unique id, no rank claimed twice
  unsigned char uid3[128];
  if (tkr_unique_id(uid3)) return 12;
  const int d1 = 1, d2 = 2;
  const int a = tkr_gate_begin_ex(uid3, 4, 0, 1, &d1, 0, 0);
  const int mismatch = tkr_gate_begin_ex(uid3, 8, 1, 1, &d2, 0, 0);
  const int twice = tkr_gate_begin_ex(uid3, 4, 0, 1, &d2, 0, 0);
  if (a <= 0 || mismatch != -2 || twice != -2) { std::printf("a %d mismatch %d twice %d\n", a, mismatch, twice); ++failures; }
  if (std::strstr(tkr_last_error(), "claimed twice") == nullptr) { std::printf("err %s\n", tkr_last_error()); ++failures; }
  tkr_gate_cancel(a);  // not sweeping: aborts it
  if (tkr_gate_pending() != 0) { std::printf("pending %d\n", tkr_gate_pending()); ++failures; }

  // 4. the HBM model (TK_RCCL_STUB_HBM_FREE): a non-blocking init that does not fit fails
  //    at poll and at sweep, with RCCL's out-of-memory text, and leaves nothing pending
  if (const char* hbm = std::getenv("TEST_HBM_FREE_FILE")) {
    setenv("TK_RCCL_STUB_HBM_FREE", hbm, 1);  // (the gates above had all the memory they wanted)
    setenv("TK_RCCL_STUB_FOOTPRINT_MIB", "1024", 1);
    unsigned char uid4[128];
    if (tkr_unique_id(uid4)) return 13;
    const int h4 = tkr_gate_begin_ex(uid4, 1, 0, 1, &dev0, 0, 0);
    double e4 = 0;
    const int p4 = tkr_gate_poll(h4);
    const int s4 = sweep(h4, 1000.0, &e4);
    if (h4 <= 0 || p4 != -2 || s4 != -2 || std::strstr(tkr_last_error(), "out of memory") == nullptr) {
      std::printf("oom h %d poll %d sweep %d err %s\n", h4, p4, s4, tkr_last_error());
      ++failures;
    }
    if (tkr_gate_pending() != 0) { std::printf("pending after oom %d\n", tkr_gate_pending()); ++failures; }
    unsetenv("TK_RCCL_STUB_HBM_FREE");
  }
  std::printf("stub driver: %d failure(s)\n", failures);
  return failures ? 1 : 0;
}
"""


def _build_and_run(tmp_path, flags, name):
    cxx = shutil.which("g++") or shutil.which("c++")
    if not cxx:
        pytest.skip("no host C++ compiler")
    (tmp_path / "driver.cpp").write_text(DRIVER)
    exe = tmp_path / name
    build = subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, "-I", CSRC,
                            str(tmp_path / "driver.cpp"), os.path.join(CSRC, "tk_rccl_stub.cpp"), "-o", str(exe),
                            "-pthread"], capture_output=True, text=True, timeout=240)
    if build.returncode != 0 and "sanitize" in build.stderr and "not supported" in build.stderr:
        pytest.skip(f"{flags[0]} unavailable: {build.stderr[-200:]}")
    assert build.returncode == 0, build.stderr[-3000:]
    free = tmp_path / "hbm-free"
    free.write_text(str(100 << 20))  # 100 MiB free, 1 GiB needed
    env = dict(os.environ, TK_RCCL_STUB_DIR=str(tmp_path / "rendezvous"), ASAN_OPTIONS="detect_leaks=1",
               TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1", UBSAN_OPTIONS="print_stacktrace=1",
               TEST_HBM_FREE_FILE=str(free))
    run = subprocess.run([str(exe), *_scan_inputs(tmp_path)], capture_output=True, text=True, timeout=240,
                         env=env)
    return run


def _scan_inputs(tmp_path):
    """Files for the ELF scan: the librccl builds of this image, another ELF, and broken
    copies (cut short of its section headers; section header offset pointing past the end;
    a string-table index out of range)."""
    import struct

    import torch

    libs = [p for p in (os.path.realpath("/opt/rocm/lib/librccl.so.1"),
                        os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")) if os.path.exists(p)]
    out = list(libs) + [shutil.which("ls") or "/bin/ls", str(tmp_path / "missing.so")]
    src = open(shutil.which("ls") or "/bin/ls", "rb").read()
    (tmp_path / "short.so").write_bytes(src[: len(src) // 2])
    bad = bytearray(src)
    struct.pack_into("<Q", bad, 0x28, len(src) + 4096)  # e_shoff past the end
    (tmp_path / "shoff.so").write_bytes(bytes(bad))
    bad = bytearray(src)
    struct.pack_into("<H", bad, 0x3E, 0xFFF0)  # e_shstrndx / links out of range: sections still bounded
    (tmp_path / "strndx.so").write_bytes(bytes(bad))
    out += [str(tmp_path / n) for n in ("short.so", "shoff.so", "strndx.so")]
    return out


def test_stub_clean_under_asan_ubsan(tmp_path):
    run = _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"], "stub-asan")
    assert run.returncode == 0, run.stdout[-2000:] + run.stderr[-4000:]
    assert "stub driver: 0 failure(s)" in run.stdout
    assert "ERROR: AddressSanitizer" not in run.stderr and "runtime error" not in run.stderr
    scans = [ln.split() for ln in run.stdout.splitlines() if ln.startswith("scan ")]
    found = {os.path.basename(ln[1]): ln[4] for ln in scans}  # scan <path> -> <n> <symbol>
    assert all(found[n] == "-" for n in ("short.so", "shoff.so", "missing.so", os.path.basename(shutil.which("ls")))), found
    assert any("ncclDevKernelArgsStorage" in v for v in found.values())  # a librccl of the image


def test_stub_clean_under_tsan(tmp_path):
    run = _build_and_run(tmp_path, ["-fsanitize=thread"], "stub-tsan")
    if run.returncode != 0 and "FATAL: ThreadSanitizer: unexpected memory mapping" in run.stderr:
        pytest.skip("TSan cannot map its shadow memory in this environment")
    assert run.returncode == 0, run.stdout[-2000:] + run.stderr[-4000:]
    assert "stub driver: 0 failure(s)" in run.stdout
    assert "WARNING: ThreadSanitizer" not in run.stderr
