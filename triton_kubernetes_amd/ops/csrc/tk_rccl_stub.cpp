// libtk_rccl_stub.so: the C ABI of libtk_rccl.so (tk_rccl_probe.hip) without GPUs or RCCL.
//
// A dry run of the whole cluster gate on CPU -- node agents, readiness/gate.py's
// ClusterGate, bench.py --sim-gpu -- loads this instead of the real library
// (TK_RCCL_LIB, ops/native.py).  It keeps RCCL's semantics where the callers depend on them
// and refuses what RCCL would refuse:
//
//  * a communicator exists once every rank of its world has joined under one unique id;
//    a rank waits (blocking begin, sweep) until then, or until its timeout / a cancel;
//  * geometry (tk_rccl_group.h): ranks inside the world, no GPU twice in one process;
//  * one world size per unique id, and no rank claimed twice -- across processes;
//  * the sweep is a collective: it completes when every rank has called it;
//  * bf16 verification limits (tk_rccl_verify.h).
//
// The rendezvous ("bootstrap") is a directory per unique id under $TK_RCCL_STUB_DIR
// (default /tmp/tk-rccl-stub), so ranks in different agent processes meet the way they
// would over RCCL's socket bootstrap; claims are O_EXCL files, so a double claim is seen
// whichever process makes it.  Every call is appended to $TK_RCCL_STUB_LOG as a JSON line.

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "tk_elf_scan.h"
#include "tk_rccl_group.h"
#include "tk_rccl_verify.h"

namespace {
thread_local char g_err[512];
thread_local double g_phase[4] = {0, 0, 0, 0};
thread_local double g_init_ms = 0.0;
std::mutex g_mu;
std::atomic<int> g_next{1};

struct StubGate {
  std::string dir;
  int world = 0, rank_base = 0, ndev = 0;
  std::vector<int> devices;
  std::chrono::steady_clock::time_point t0;
  double init_ms = -1.0;
  std::atomic<bool> cancel{false};
  std::string init_err;  // the init failed (the HBM model below): poll and sweep report it
};
thread_local double g_last_footprint[3] = {0, 0, 0};

// An HBM model for the gate's allocations, for tests of the agent's out-of-memory retry
// (node/agent_gate.py): TK_RCCL_STUB_HBM_FREE names a file holding the bytes each GPU has
// free (a test's burn-in child rewrites it as it holds and releases its span), and every GPU
// of an init needs TK_RCCL_STUB_FOOTPRINT_MIB.  Short of that, the init fails with the
// text libtk_rccl gives for RCCL's failed allocation.  Unset: every init fits.
size_t stub_footprint() {
  const char* f = getenv("TK_RCCL_STUB_FOOTPRINT_MIB");
  return f && *f ? (size_t)strtoull(f, nullptr, 10) << 20 : 0;
}

bool stub_hbm_short(char* err, size_t errlen) {
  const char* path = getenv("TK_RCCL_STUB_HBM_FREE");
  if (!path || !*path) return false;
  char buf[64] = {0};
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return false;
  const ssize_t n = read(fd, buf, sizeof(buf) - 1);
  close(fd);
  if (n <= 0) return false;
  const size_t free_b = (size_t)strtoull(buf, nullptr, 10);
  if (free_b >= stub_footprint()) return false;
  snprintf(err, errlen,
           "ncclCommInitRank: unhandled cuda error (run with NCCL_DEBUG=INFO for details) "
           "[rccl: Cuda failure 'out of memory'] (device 0: %zu MiB free)", free_b >> 20);
  return true;
}
std::map<int, StubGate*> g_gates;
std::map<int, StubGate*> g_sweeping;  // gates inside tkr_gate_sweep (tkr_gate_cancel reaches them)

std::string base_dir() {
  const char* d = getenv("TK_RCCL_STUB_DIR");
  return d && *d ? d : "/tmp/tk-rccl-stub";
}

std::string hex(const unsigned char* p, int n) {
  static const char* k = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < n; ++i) {
    s += k[p[i] >> 4];
    s += k[p[i] & 15];
  }
  return s;
}

void log_call(const char* op, const StubGate* g, int rc) {
  const char* path = getenv("TK_RCCL_STUB_LOG");
  if (!path || !*path) return;
  std::string devs;
  if (g)
    for (size_t i = 0; i < g->devices.size(); ++i) devs += (i ? "," : "") + std::to_string(g->devices[i]);
  char line[1024];
  snprintf(line, sizeof(line),
           "{\"op\":\"%s\",\"pid\":%d,\"uid\":\"%s\",\"world\":%d,\"rank_base\":%d,\"devices\":[%s],\"rc\":%d}\n", op,
           (int)getpid(), g ? g->dir.substr(g->dir.rfind('/') + 1).c_str() : "", g ? g->world : 0,
           g ? g->rank_base : 0, devs.c_str(), rc);
  const int fd = open(path, O_WRONLY | O_CREAT | O_APPEND, 0644);
  if (fd >= 0) {
    (void)!write(fd, line, strlen(line));
    close(fd);
  }
}

int count_prefix(const std::string& dir, const char* prefix) {
  DIR* d = opendir(dir.c_str());
  if (!d) return 0;
  int n = 0;
  const size_t len = strlen(prefix);
  while (dirent* e = readdir(d))
    if (!strncmp(e->d_name, prefix, len)) ++n;
  closedir(d);
  return n;
}

bool touch_excl(const std::string& path, const std::string& body = "") {
  const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_EXCL, 0644);
  if (fd < 0) return false;
  if (!body.empty()) (void)!write(fd, body.data(), body.size());
  close(fd);
  return true;
}

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

// Waits until `count` files named `prefix`* exist in the gate's directory: 0, -3 timeout,
// -4 canceled.
int wait_for(StubGate* g, const char* prefix, int count, double timeout_ms) {
  const auto t = std::chrono::steady_clock::now();
  while (count_prefix(g->dir, prefix) < count) {
    if (g->cancel.load()) {
      snprintf(g_err, sizeof(g_err), "gate canceled while its communicator waited for peers");
      return -4;
    }
    if (ms_since(t) > timeout_ms) {
      snprintf(g_err, sizeof(g_err), "communicator not ready after %.0f ms (%d of %d ranks)", timeout_ms,
               count_prefix(g->dir, prefix), count);
      return -3;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
  return 0;
}

void unclaim(StubGate* g) {
  for (int d = 0; d < g->ndev; ++d) unlink((g->dir + "/rank-" + std::to_string(g->rank_base + d)).c_str());
}

StubGate* take(int h) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_gates.find(h);
  if (it == g_gates.end()) return nullptr;
  StubGate* g = it->second;
  g_gates.erase(it);
  return g;
}
}  // namespace

extern "C" {
const char* tkr_last_error() { return g_err; }
int tkr_version() { return 0; }  // no RCCL behind this library
int tkr_unique_id(unsigned char* out128) {
  const int fd = open("/dev/urandom", O_RDONLY);
  const bool ok = fd >= 0 && read(fd, out128, 128) == 128;
  if (fd >= 0) close(fd);
  if (!ok) {
    snprintf(g_err, sizeof(g_err), "no /dev/urandom");
    return -1;
  }
  return 0;
}
double tkr_last_init_ms() { return g_init_ms; }
double tkr_last_phase_ms(int i) { return i >= 0 && i < 4 ? g_phase[i] : 0.0; }
void tkr_set_async_teardown(int) {}
void tkr_set_teardown_abort(int) {}
void tkr_set_teardown_quiet_ms(double) {}
int tkr_teardowns_pending() { return 0; }
int tkr_drain() { return 0; }
int tkr_gate_abandoned() { return 0; }
int tkr_inits_running() { return 0; }  // no device code to load: nothing a release could hold up
int tkr_preloads_running() { return 0; }
int tkr_preload_device_code(int, const int*) { return 1; }  // no RCCL device code behind the stub
const char* tkr_preload_symbol() { return "none"; }
const char* tkr_preload_how() { return "none"; }
int tkr_elf_kernel_symbol(const char* path, char* out, int cap) {  // the probe's scanner, on the CPU
  const std::string name = tk_elf_find_symbol(path, kTkRcclKernelNeedle, kTkRcclKernelReject);
  if (cap > 0) snprintf(out, (size_t)cap, "%s", name.c_str());
  return (int)name.size();
}
int tkr_gate_pending() {
  std::lock_guard<std::mutex> lk(g_mu);
  return (int)g_gates.size();
}
double tkr_last_footprint(int which) { return which >= 0 && which < 3 ? g_last_footprint[which] : 0.0; }

int tkr_gate_begin_ex(const unsigned char* uid128, int world, int rank_base, int ndev, const int* devices,
                      int blocking, size_t /*prealloc_bytes*/) {
  if (tk_check_geometry(world, rank_base, ndev, devices, g_err, sizeof(g_err))) {
    log_call("begin", nullptr, -1);
    return -1;
  }
  auto* g = new StubGate();
  g->dir = base_dir() + "/" + hex(uid128, 16);
  g->world = world;
  g->rank_base = rank_base;
  g->ndev = ndev;
  g->devices.assign(devices, devices + ndev);
  g->t0 = std::chrono::steady_clock::now();
  char oom[512];
  if (stub_hbm_short(oom, sizeof(oom))) {
    if (blocking) {
      snprintf(g_err, sizeof(g_err), "%s", oom);
      log_call("begin", g, -2);
      delete g;
      return -2;
    }
    g->init_err = oom;  // a non-blocking init fails on its own thread: poll / sweep see it
    int h;
    {
      std::lock_guard<std::mutex> lk(g_mu);
      h = g_next++;
      g_gates[h] = g;
    }
    log_call("begin-oom", g, h);
    return h;
  }
  mkdir(base_dir().c_str(), 0755);
  mkdir(g->dir.c_str(), 0755);
  // one world size per unique id (the first rank to arrive records it)
  const std::string wpath = g->dir + "/world";
  if (!touch_excl(wpath, std::to_string(world))) {
    char buf[32] = {0};
    const int fd = open(wpath.c_str(), O_RDONLY);
    for (int i = 0; i < 200 && fd >= 0 && read(fd, buf, sizeof(buf) - 1) <= 0; ++i)  // being written
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    if (fd >= 0) close(fd);
    if (atoi(buf) != world) {
      snprintf(g_err, sizeof(g_err), "ncclCommInitRank: unique id used with world %d and %d", atoi(buf), world);
      log_call("begin", g, -2);
      delete g;
      return -2;
    }
  }
  for (int d = 0; d < ndev; ++d)
    if (!touch_excl(g->dir + "/rank-" + std::to_string(rank_base + d), std::to_string(getpid()))) {
      snprintf(g_err, sizeof(g_err), "ncclCommInitRank: rank %d of this unique id claimed twice", rank_base + d);
      for (int u = 0; u < d; ++u) unlink((g->dir + "/rank-" + std::to_string(rank_base + u)).c_str());
      log_call("begin", g, -2);
      delete g;
      return -2;
    }
  if (blocking) {
    const int rc = wait_for(g, "rank-", world, 120000.0);
    if (rc) {
      unclaim(g);
      log_call("begin", g, rc);
      delete g;
      return rc;
    }
    g->init_ms = ms_since(g->t0);
  }
  int h;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    h = g_next++;
    g_gates[h] = g;
  }
  log_call("begin", g, h);
  return h;
}

int tkr_gate_begin(const unsigned char* uid128, int world, int rank_base, int ndev, const int* devices,
                   int blocking) {
  return tkr_gate_begin_ex(uid128, world, rank_base, ndev, devices, blocking, 0);
}

int tkr_gate_poll(int h) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_gates.find(h);
  if (it == g_gates.end()) {
    snprintf(g_err, sizeof(g_err), "unknown gate %d", h);
    return -1;
  }
  if (!it->second->init_err.empty()) {
    snprintf(g_err, sizeof(g_err), "%s", it->second->init_err.c_str());
    return -2;
  }
  return count_prefix(it->second->dir, "rank-") >= it->second->world ? 0 : 1;
}

int tkr_gate_abort(int h) {
  StubGate* g = take(h);
  if (!g) return -1;
  const int pending = g->init_err.empty() && count_prefix(g->dir, "rank-") < g->world ? 1 : 0;
  if (g->init_err.empty()) unclaim(g);  // a failed init claimed nothing
  log_call("abort", g, pending);
  delete g;
  return pending;
}

int tkr_gate_cancel(int h) {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_sweeping.find(h);
    if (it != g_sweeping.end()) {
      it->second->cancel.store(true);
      log_call("cancel", it->second, 0);
      return 0;
    }
  }
  return tkr_gate_abort(h) < 0 ? -1 : 0;
}

int tkr_gate_sweep(int h, const size_t* sizes, int nsizes, int /*iters*/, int /*warmup*/, int dtype, double timeout_ms,
                   double* time_us, double* algbw, double* busbw, double* errors, double* phase_ms) {
  StubGate* g = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_gates.find(h);
    if (it != g_gates.end()) {
      g = it->second;
      g_gates.erase(it);
      g_sweeping[h] = g;
    }
  }
  if (!g) {
    snprintf(g_err, sizeof(g_err), "unknown gate %d", h);
    return -1;
  }
  const auto t = std::chrono::steady_clock::now();
  if (!g->init_err.empty()) {
    snprintf(g_err, sizeof(g_err), "%s", g->init_err.c_str());
    {
      std::lock_guard<std::mutex> lk(g_mu);
      g_sweeping.erase(h);
    }
    log_call("sweep", g, -2);
    delete g;
    return -2;
  }
  int rc = wait_for(g, "rank-", g->world, timeout_ms);  // the communicator's init
  if (g->init_ms < 0 && rc == 0) g->init_ms = ms_since(g->t0);
  phase_ms[0] = ms_since(t);
  phase_ms[4] = g->init_ms;
  if (rc == 0 && !tk_verifiable(dtype, g->world)) {
    snprintf(g_err, sizeof(g_err), "bf16 all-reduce sums of %d ranks are not exact in bf16", g->world);
    rc = -1;
  }
  if (rc == 0) {
    // the collective: every rank calls it, none finishes before all have
    for (int d = 0; d < g->ndev; ++d) touch_excl(g->dir + "/swept-" + std::to_string(g->rank_base + d));
    rc = wait_for(g, "swept-", g->world, timeout_ms);
  }
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_sweeping.erase(h);
  }
  if (rc == 0) {
    float sum = 0.f;  // what every rank would hold: the verification rule, exercised
    for (int r = 0; r < g->world; ++r) sum += tk_verify_value(dtype, g->world, r);
    for (int s = 0; s < nsizes; ++s) {
      const double us = 5.0 + (double)sizes[s] / 100e3;  // a nominal ~100 GB/s: not a measurement
      time_us[s] = us;
      algbw[s] = (double)sizes[s] / (us * 1e-6) / 1e9;
      busbw[s] = algbw[s] * (g->world > 1 ? 2.0 * (g->world - 1) / g->world : 1.0);
      errors[s] = sum == tk_verify_sum(dtype, g->world) ? 0.0 : 1.0;
    }
    phase_ms[1] = 0.0;
    phase_ms[2] = ms_since(t) - phase_ms[0];
    g_last_footprint[0] = g_last_footprint[1] = (double)stub_footprint();
    // 1: as if this process's own accounting; TK_RCCL_STUB_FOOTPRINT_KIND=2: a device-wide number
    const char* kind = getenv("TK_RCCL_STUB_FOOTPRINT_KIND");
    g_last_footprint[2] = kind && *kind ? atof(kind) : 1.0;
    phase_ms[3] = 0.0;
    // the last rank to leave removes the rendezvous
    for (int d = 0; d < g->ndev; ++d) touch_excl(g->dir + "/done-" + std::to_string(g->rank_base + d));
    if (count_prefix(g->dir, "done-") >= g->world) {
      DIR* dd = opendir(g->dir.c_str());
      while (dd) {
        dirent* e = readdir(dd);
        if (!e) break;
        if (e->d_name[0] != '.') unlink((g->dir + "/" + e->d_name).c_str());
      }
      if (dd) closedir(dd);
      rmdir(g->dir.c_str());
    }
  } else {
    unclaim(g);
  }
  g_init_ms = phase_ms[4];
  g_phase[0] = phase_ms[4];
  g_phase[1] = phase_ms[1];
  g_phase[2] = phase_ms[2];
  g_phase[3] = phase_ms[3];
  log_call("sweep", g, rc);
  delete g;
  return rc;
}

int tkr_sweep_rank(int rank, int world, const unsigned char* uid128, int device, const size_t* sizes, int nsizes,
                   int iters, int warmup, int dtype, double* time_us, double* algbw, double* busbw, double* errors) {
  const int h = tkr_gate_begin(uid128, world, rank, 1, &device, 1);
  if (h < 0) return h;
  double ph[5] = {0, 0, 0, 0, 0};
  return tkr_gate_sweep(h, sizes, nsizes, iters, warmup, dtype, 600000.0, time_us, algbw, busbw, errors, ph);
}

int tkr_sweep_local(int ndev, const size_t* sizes, int nsizes, int iters, int warmup, int dtype, double* time_us,
                    double* algbw, double* busbw, double* errors) {
  unsigned char uid[128];
  if (tkr_unique_id(uid)) return -1;
  std::vector<int> devs(ndev);
  for (int d = 0; d < ndev; ++d) devs[d] = d;
  const int h = tkr_gate_begin(uid, ndev, 0, ndev, devs.data(), 1);
  if (h < 0) return h;
  double ph[5] = {0, 0, 0, 0, 0};
  return tkr_gate_sweep(h, sizes, nsizes, iters, warmup, dtype, 600000.0, time_us, algbw, busbw, errors, ph);
}
}
