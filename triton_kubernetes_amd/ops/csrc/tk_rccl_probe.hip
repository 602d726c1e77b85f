// rccl-ready (N2): RCCL all-reduce readiness / bandwidth probe.
//
// The "GPU-ready" gate of the readiness waiter.  Two entry points:
//
//  * tkr_sweep_rank  — one rank of a multi-process (multi-node) communicator,
//    bootstrapped from a ncclUniqueId the caller distributes (the cluster-wide
//    gate across MI355X workers, one process per GPU);
//  * tkr_sweep_local — one process driving every local GPU with
//    ncclCommInitAll + grouped calls (the node-level gate on an 8xMI355X node,
//    where all traffic is point-to-point xGMI).
//
// For each message size: ncclAllReduce(sum) of a buffer holding a per-rank value,
// verified on device against the exact sum (tk_rccl_verify.h: rank + 1
// in f32, and in bf16 up to 15 ranks; 1 per rank in bf16 beyond, exact up to 256
// ranks, and bf16 refused above that), timed with HIP events over `iters` launches after
// `warmup`.  Reported as algbw = bytes / t and busbw = algbw * 2(n-1)/n (the
// ring all-reduce bus bandwidth, comparable with the per-link xGMI rate).
//
// C ABI for ctypes; the stand-alone `rccl-ready` executable (-DTK_RCCL_MAIN)
// runs the local sweep and exits non-zero when verification fails or the
// largest message's busbw is below the --min-busbw threshold.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "tk_elf_scan.h"
#include "tk_rccl_group.h"
#include "tk_rccl_verify.h"

#include <dlfcn.h>
#include <unistd.h>

#include <cctype>
#include <cerrno>
#include <climits>
#include <cmath>
#include <string>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

static thread_local char g_err[512];
static inline double ms_since(std::chrono::steady_clock::time_point t);
static thread_local double g_last_init_ms = 0.0;
extern "C" const char* tkr_last_error() { return g_err; }
// Wall time of the calling thread's last communicator init (ms).
extern "C" double tkr_last_init_ms() { return g_last_init_ms; }

#define HIPCHECK(call)                                                                            \
  do {                                                                                            \
    hipError_t _e = (call);                                                                       \
    if (_e != hipSuccess) {                                                                       \
      snprintf(g_err, sizeof(g_err), "%s: %s", #call, hipGetErrorString(_e));                     \
      return -1;                                                                                  \
    }                                                                                             \
  } while (0)

#define NCCLCHECK(call)                                                                           \
  do {                                                                                            \
    ncclResult_t _r = (call);                                                                     \
    if (_r != ncclSuccess) {                                                                      \
      snprintf(g_err, sizeof(g_err), "%s: %s", #call, ncclGetErrorString(_r));                    \
      return -2;                                                                                  \
    }                                                                                             \
  } while (0)

__global__ void k_fill_f32(float* p, size_t n, float v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void k_fill_bf16(__bf16* p, size_t n, float v) {
  const __bf16 b = (__bf16)v;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = b;
}
__global__ void k_check_f32(const float* p, size_t n, float want, unsigned long long* bad) {
  unsigned int c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    c += (p[i] != want);
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(bad, (unsigned long long)c);
}
__global__ void k_check_bf16(const __bf16* p, size_t n, float want, unsigned long long* bad) {
  unsigned int c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    c += ((float)p[i] != want);
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(bad, (unsigned long long)c);
}

extern "C" int tkr_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

extern "C" int tkr_unique_id(unsigned char* out128) {
  ncclUniqueId id;
  NCCLCHECK(ncclGetUniqueId(&id));
  memcpy(out128, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

struct RankBufs {
  void* send = nullptr;
  void* recv = nullptr;
  unsigned long long* bad = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t t0 = nullptr, t1 = nullptr;
};

static int alloc_bufs(RankBufs& b, size_t max_bytes) {
  HIPCHECK(hipMalloc(&b.send, max_bytes));
  HIPCHECK(hipMalloc(&b.recv, max_bytes));
  HIPCHECK(hipMalloc(&b.bad, sizeof(unsigned long long)));
  HIPCHECK(hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking));
  HIPCHECK(hipEventCreate(&b.t0));
  HIPCHECK(hipEventCreate(&b.t1));
  return 0;
}

static void free_bufs(RankBufs& b) {
  if (b.t0) (void)hipEventDestroy(b.t0);
  if (b.t1) (void)hipEventDestroy(b.t1);
  if (b.stream) (void)hipStreamDestroy(b.stream);
  if (b.send) (void)hipFree(b.send);
  if (b.recv) (void)hipFree(b.recv);
  if (b.bad) (void)hipFree(b.bad);
  b = RankBufs{};
}

static int check_verifiable(int dtype, int world) {
  if (!tk_verifiable(dtype, world)) {
    snprintf(g_err, sizeof(g_err),
             "bf16 all-reduce sums of %d ranks are not exact in bf16 (8 significant bits, at most %d ranks); "
             "gate in f32",
             world, kBf16MaxWorld);
    return -1;
  }
  return 0;
}
static int fill(RankBufs& b, size_t count, int dtype, float v) {
  if (dtype == 1) k_fill_bf16<<<512, 256, 0, b.stream>>>((__bf16*)b.send, count, v);
  else k_fill_f32<<<512, 256, 0, b.stream>>>((float*)b.send, count, v);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipMemsetAsync(b.bad, 0, sizeof(unsigned long long), b.stream));
  return 0;
}

static int check(RankBufs& b, size_t count, int dtype, float want) {
  if (dtype == 1) k_check_bf16<<<512, 256, 0, b.stream>>>((const __bf16*)b.recv, count, want, b.bad);
  else k_check_f32<<<512, 256, 0, b.stream>>>((const float*)b.recv, count, want, b.bad);
  HIPCHECK(hipGetLastError());
  return 0;
}

static inline double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

// Per-thread phase timings of the last tkr_sweep_rank: init, alloc, sweep, teardown (ms).
static thread_local double g_phase_ms[4] = {0, 0, 0, 0};
extern "C" double tkr_last_phase_ms(int phase) { return (phase >= 0 && phase < 4) ? g_phase_ms[phase] : -1.0; }

// Communicator teardown (ncclCommDestroy joins RCCL's proxy threads and frees
// its device resources; ~0.5 s measured on MI355X, longer than init) is not
// part of the readiness answer.  With async teardown on, it runs on a
// background thread after the verified result is returned; tkr_drain() waits for
// every pending teardown and should run before process exit.
// One background worker owns every asynchronous teardown, in submission order: destroys
// never run concurrently with each other (a thread per communicator piled up ~10 concurrent
// ncclCommDestroy calls behind back-to-back gates and stalled the next bring-up), and the
// worker is started once, not per gate.
//
// Teardowns can also wait for a quiet period (tkr_set_teardown_quiet_ms): a destroy
// frees pinned host and device memory, and doing that while another bring-up allocates
// stalled that bring-up (≈120 ms once per run, measured); with a quiet period the queue
// runs only after `quiet_ms` without gate activity (begin / sweep) in the process.
struct TeardownQueue {
  std::mutex mu;
  std::condition_variable cv, idle_cv;
  std::vector<std::function<void()>> q;
  bool busy = false, stop = false, flush = false;
  std::thread worker;
  double quiet_ms = 0.0;
  std::chrono::steady_clock::time_point last_activity = std::chrono::steady_clock::now();

  void touch() {
    std::lock_guard<std::mutex> lk(mu);
    last_activity = std::chrono::steady_clock::now();
  }

  void submit(std::function<void()> fn) {
    std::unique_lock<std::mutex> lk(mu);
    q.push_back(std::move(fn));
    if (!worker.joinable()) worker = std::thread([this] { run(); });
    cv.notify_one();
  }
  void run() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [this] { return stop || !q.empty(); });
      if (q.empty()) return;  // stop requested and nothing left
      // hold off while bring-ups are active (unless draining / exiting)
      while (!stop && !flush && quiet_ms > 0) {
        const double since = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() -
                                                                        last_activity).count();
        if (since >= quiet_ms) break;
        cv.wait_for(lk, std::chrono::duration<double, std::milli>(quiet_ms - since));
      }
      auto fn = std::move(q.front());
      q.erase(q.begin());
      busy = true;
      lk.unlock();
      fn();
      lk.lock();
      busy = false;
      if (q.empty()) idle_cv.notify_all();
    }
  }
  // Waits until every submitted teardown has run; returns how many were waited for.
  int drain() {
    std::unique_lock<std::mutex> lk(mu);
    const int n = (int)q.size() + (busy ? 1 : 0);
    flush = true;
    cv.notify_all();
    idle_cv.wait(lk, [this] { return q.empty() && !busy; });
    flush = false;
    return n;
  }
  ~TeardownQueue() {  // process exit: finish queued work, then join the worker
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    if (worker.joinable()) worker.join();
  }
};
static TeardownQueue g_teardowns;

// Per calling thread: a gate served on one agent thread never changes the
// teardown mode of probes running on other threads.
static thread_local int g_async_teardown = 0;
extern "C" void tkr_set_async_teardown(int on) { g_async_teardown = on; }

// ncclCommAbort instead of ncclCommDestroy for the teardown (no in-flight work remains
// after a verified sweep, so nothing is lost; it skips the graceful finalize).
static std::atomic<int> g_teardown_abort{0};
extern "C" void tkr_set_teardown_abort(int on) { g_teardown_abort = on; }

// split of the last teardown (ms): buffer frees, communicator destroy/abort
static std::atomic<double> g_teardown_free_ms{0.0}, g_teardown_comm_ms{0.0};
extern "C" double tkr_last_teardown_ms(int which) {
  return which == 0 ? g_teardown_free_ms.load() : which == 1 ? g_teardown_comm_ms.load() : -1.0;
}

static void teardown(ncclComm_t comm, RankBufs b, int device) {
  const bool abort = g_teardown_abort.load() != 0;
  auto work = [comm, b, device, abort]() mutable {
    (void)hipSetDevice(device);
    auto t0 = std::chrono::steady_clock::now();
    free_bufs(b);
    g_teardown_free_ms.store(ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    if (abort) ncclCommAbort(comm);
    else ncclCommDestroy(comm);
    g_teardown_comm_ms.store(ms_since(t0));
  };
  if (g_async_teardown) {
    g_teardowns.submit(work);
    g_phase_ms[3] = 0.0;
  } else {
    const auto t = std::chrono::steady_clock::now();
    work();
    g_phase_ms[3] = ms_since(t);
  }
}

extern "C" int tkr_drain() { return g_teardowns.drain(); }
extern "C" void tkr_set_teardown_quiet_ms(double ms) {
  std::lock_guard<std::mutex> lk(g_teardowns.mu);
  g_teardowns.quiet_ms = ms > 0 ? ms : 0.0;
}
extern "C" int tkr_teardowns_pending() {
  std::lock_guard<std::mutex> lk(g_teardowns.mu);
  return (int)g_teardowns.q.size() + (g_teardowns.busy ? 1 : 0);
}

static inline size_t elem_size(int dtype) { return dtype == 1 ? 2 : 4; }
static inline ncclDataType_t nccl_type(int dtype) { return dtype == 1 ? ncclBfloat16 : ncclFloat32; }

// ---------------------------------------------------------------------------------------------
// Cluster gate communicators.  One process (a node agent) owns `ndev` local GPUs and joins the
// cluster-wide communicator as ranks rank_base .. rank_base+ndev-1 (one ncclCommInitRank per
// device inside one group).  With blocking=0 the init runs on a thread of its own: begin
// returns at once, so an agent can start it as soon as cluster membership is known and overlap
// the bootstrap / topology / connection setup with the rest of the node bring-up; the gate
// request later only waits for the remainder and runs the verified sweep.
//
// Only the long-stable RCCL API is used (ncclCommInitRank, groups, ncclAllReduce,
// ncclCommDestroy/Abort): inside a PyTorch process this library binds to the RCCL that torch
// already loaded (same SONAME), which can be older than the headers it was compiled with, so
// the versioned ncclConfig_t of ncclCommInitRankConfig is avoided.
//
// A gate that will never run (a node failed) is released with tkr_gate_abort.  If its init is
// still waiting for peers that will not come, RCCL cannot be interrupted there (there is no
// bootstrap timeout); the init thread is detached and cleans up after itself should the init
// ever complete.  tkr_gate_abandoned() counts such threads: a process holding one cannot run
// the HIP/RCCL exit teardown safely and should leave with _exit (ops/rccl.py:exit_now).
struct Gate {
  std::vector<int> devices;
  std::vector<ncclComm_t> comms;
  int rank_base = 0, world = 0;
  std::chrono::steady_clock::time_point t_begin;
  double init_ms = -1.0;  // begin -> every comm ready
  std::mutex mu;
  std::condition_variable cv;
  int init_state = 0;  // 0 running, 1 ready, -2 failed
  bool abandoned = false;
  bool cancel = false;  // tkr_gate_cancel: stop waiting for peers that will not come
  char err[512] = {0};
  std::thread init_thread;
  size_t prealloc_bytes = 0;     // sweep buffers allocated by the init thread after the comms
  std::vector<RankBufs> bufs;    // (filled when prealloc_bytes > 0 and the init succeeded)
  // device memory the init took, max over this gate's GPUs (this process's VRAM before and
  // after, proc_vram): the communicators (RCCL's per-channel, per-peer buffers, its device
  // code) and then the preallocated sweep buffers
  long long footprint_comm = 0, footprint_total = 0;  // -1: not measurable here
  int footprint_kind = 0;                             // 1: this process's VRAM, 2: the device's
};
// the footprint of the gate the calling thread last swept (tkr_last_footprint; -1: unknown)
static thread_local double g_last_footprint[3] = {0, 0, 0};  // comm, with the sweep buffers, kind
extern "C" double tkr_last_footprint(int which) { return which >= 0 && which < 3 ? g_last_footprint[which] : 0.0; }

static size_t device_free(int dev) {
  size_t free_b = 0, total_b = 0;
  if (hipSetDevice(dev) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) return 0;
  return free_b;
}

// VRAM this process holds on HIP device `dev` (bytes), from the amdgpu KFD's per-process
// accounting (/sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>); -1 when it cannot be read.  The
// gate's footprint is measured with it, not with hipMemGetInfo: the device's free memory
// also moves with the burn-in child allocating its ~280 GB span at the same moment (a
// device-wide delta read 290 GB on MI355X, profiles/round6/README.md).
static long long proc_vram(int dev) {
  static std::mutex mu;
  static std::vector<long long> gpu_id;  // HIP device -> KFD gpu_id (0: not found yet, -1: none)
  unsigned long long gid = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    if ((int)gpu_id.size() <= dev) gpu_id.resize((size_t)dev + 1, 0);
    if (gpu_id[dev] == 0) {
      gpu_id[dev] = -1;
      char bus[64] = {0};
      unsigned dom = 0, b = 0, d = 0, f = 0;
      if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) == hipSuccess &&
          sscanf(bus, "%x:%x:%x.%x", &dom, &b, &d, &f) == 4) {
        const unsigned long long loc = ((unsigned long long)b << 8) | (d << 3) | f;
        for (int n = 0; n < 1024; ++n) {
          char path[128];
          snprintf(path, sizeof(path), "/sys/class/kfd/kfd/topology/nodes/%d/properties", n);
          FILE* fp = fopen(path, "r");
          if (!fp) {
            if (errno == ENOENT) break;  // past the last node
            continue;                    // a node this process may not read (another tenant's GPU)
          }
          char key[64];
          unsigned long long v = 0, nloc = ~0ull, ndom = ~0ull;
          while (fscanf(fp, "%63s %llu", key, &v) == 2) {
            if (!strcmp(key, "location_id")) nloc = v;
            else if (!strcmp(key, "domain")) ndom = v;
          }
          fclose(fp);
          if (nloc != loc || ndom != dom) continue;
          snprintf(path, sizeof(path), "/sys/class/kfd/kfd/topology/nodes/%d/gpu_id", n);
          if ((fp = fopen(path, "r")) != nullptr) {
            if (fscanf(fp, "%llu", &v) == 1 && v) gpu_id[dev] = (long long)v;
            fclose(fp);
          }
          break;
        }
      }
    }
    if (gpu_id[dev] <= 0) return -1;
    gid = (unsigned long long)gpu_id[dev];
  }
  char path[128];
  snprintf(path, sizeof(path), "/sys/class/kfd/kfd/proc/%d/vram_%llu", (int)getpid(), gid);
  FILE* fp = fopen(path, "r");
  if (!fp) return -1;
  unsigned long long v = 0;
  const int got = fscanf(fp, "%llu", &v);
  fclose(fp);
  return got == 1 ? (long long)v : -1;
}
static std::mutex g_gate_mu;
static std::vector<std::pair<int, Gate*>> g_gates;
// gates a tkr_gate_sweep is waiting on (taken out of g_gates): reachable by tkr_gate_cancel
static std::vector<std::pair<int, Gate*>> g_sweeping;
static int g_next_gate = 1;
// inits released while still waiting for peers (their threads are detached)
static std::atomic<int> g_abandoned{0};
extern "C" int tkr_gate_abandoned() { return g_abandoned.load(); }
// communicator inits still running (begun, not yet ready or failed): a burn-in child that
// is about to release its HBM waits for these -- the driver's clearing of the release holds
// up the init's copies and allocations (ops/probe.py:set_release_hold)
static std::atomic<int> g_inits_running{0};
extern "C" int tkr_inits_running() { return g_inits_running.load(); }

// RCCL's device code for `devs`, loaded on background threads now (one per device), before
// any communicator: a node agent calls this as it starts, so the load -- most of a fresh
// process's first ncclCommInitRank, which finds the code resident afterwards
// (profiles/round2/cold_rccl_init.md) -- overlaps the rest of its start-up instead of
// following the gate's first request.  The load is triggered by the attributes query of
// one kernel librccl exports; the runtime loads the library's whole code object for the
// device then.  The handle is looked up by name first (the names /opt/rocm's librccl
// exports), then found by scanning the loaded librccl's dynamic symbols for any exported
// device kernel (tk_elf_scan.h) -- torch's librccl names its kernels differently, and a
// ROCm update may rename them.  Returns 0 when started, 1 when no kernel handle was found
// (nothing started), -1 when librccl is not loaded.  tkr_preload_symbol names the handle
// used and how it was found ("none" before a successful call).
static std::atomic<int> g_preloads_running{0};
extern "C" int tkr_preloads_running() { return g_preloads_running.load(); }
static char g_preload_symbol[512] = "none";
static char g_preload_how[16] = "none";
extern "C" const char* tkr_preload_symbol() { return g_preload_symbol; }
extern "C" const char* tkr_preload_how() { return g_preload_how; }

// The kernel symbol tk_elf_scan.h finds in the ELF file at `path` ("" -> returns 0); for
// tests and for the agent's start-up report.
extern "C" int tkr_elf_kernel_symbol(const char* path, char* out, int cap) {
  const std::string name = tk_elf_find_symbol(path, kTkRcclKernelNeedle, kTkRcclKernelReject);
  if (cap > 0) snprintf(out, (size_t)cap, "%s", name.c_str());
  return (int)name.size();
}

extern "C" int tkr_preload_device_code(int ndev, const int* devs) {
  void* lib = dlopen("librccl.so.1", RTLD_LAZY | RTLD_NOLOAD);
  if (!lib) {
    snprintf(g_err, sizeof(g_err), "librccl.so.1 is not loaded");
    return -1;
  }
  static const char* kHandles[] = {"_Z23ncclDevKernel_Generic_124ncclDevKernelArgsStorageILm4096EE",
                                   "_Z23ncclDevKernel_Generic_224ncclDevKernelArgsStorageILm4096EE"};
  const void* handle = nullptr;
  for (const char* name : kHandles)
    if ((handle = dlsym(lib, name)) != nullptr) {
      snprintf(g_preload_symbol, sizeof(g_preload_symbol), "%s", name);
      snprintf(g_preload_how, sizeof(g_preload_how), "known");
      break;
    }
  if (!handle) {
    // the file the loaded librccl came from: an exported function's dladdr
    Dl_info info;
    void* anchor = dlsym(lib, "ncclGetVersion");
    if (anchor && dladdr(anchor, &info) && info.dli_fname) {
      const std::string name = tk_elf_find_symbol(info.dli_fname, kTkRcclKernelNeedle, kTkRcclKernelReject);
      if (!name.empty() && (handle = dlsym(lib, name.c_str())) != nullptr) {
        snprintf(g_preload_symbol, sizeof(g_preload_symbol), "%s", name.c_str());
        snprintf(g_preload_how, sizeof(g_preload_how), "scan");
      }
    }
  }
  dlclose(lib);  // RTLD_NOLOAD took a reference of its own; the library stays loaded
  if (!handle) {
    snprintf(g_err, sizeof(g_err), "librccl exports no device-kernel handle (%s)", kTkRcclKernelNeedle);
    return 1;
  }
  for (int i = 0; i < ndev; ++i) {
    const int dev = devs[i];
    g_preloads_running.fetch_add(1);
    std::thread([dev, handle] {
      if (hipSetDevice(dev) == hipSuccess) {
        hipFuncAttributes a;
        (void)hipFuncGetAttributes(&a, handle);
        (void)hipGetLastError();
      }
      g_preloads_running.fetch_sub(1);
    }).detach();
  }
  return 0;
}

static Gate* take_gate(int h) {
  std::lock_guard<std::mutex> lk(g_gate_mu);
  for (size_t i = 0; i < g_gates.size(); ++i)
    if (g_gates[i].first == h) {
      Gate* g = g_gates[i].second;
      g_gates.erase(g_gates.begin() + (long)i);
      return g;
    }
  return nullptr;
}

static Gate* peek_gate(int h) {
  std::lock_guard<std::mutex> lk(g_gate_mu);
  for (auto& e : g_gates)
    if (e.first == h) return e.second;
  return nullptr;
}

static void destroy_comms(Gate* g, bool abort) {
  for (size_t d = 0; d < g->comms.size(); ++d) {
    if (!g->comms[d]) continue;
    (void)hipSetDevice(g->devices[d]);
    if (abort) ncclCommAbort(g->comms[d]);
    else ncclCommDestroy(g->comms[d]);
    g->comms[d] = nullptr;
  }
}

// RCCL and HIP behind tk_rccl_group.h's Api (the grouped-init sequence lives there, where a
// CPU test checks it against a mock that enforces RCCL's contract).
struct HipNcclApi {
  using Comm = ncclComm_t;
  static constexpr int kInvalidArgument = (int)ncclInvalidArgument;
  ncclUniqueId id;
  int group_start() { return (int)ncclGroupStart(); }
  int group_end() { return (int)ncclGroupEnd(); }
  int set_device(int dev) { return hipSetDevice(dev) == hipSuccess ? 0 : 1; }
  int init_rank(Comm* c, int world, int rank) { return (int)ncclCommInitRank(c, world, id, rank); }
  const char* error_string(int r) { return ncclGetErrorString((ncclResult_t)r); }
};

// An init that failed says what the devices had left: RCCL reports an allocation failure as
// "unhandled cuda error" (or "unhandled system error"), and its own last-error text -- when
// this librccl has ncclGetLastError -- names the failing call.  ops/rccl.py:is_oom_error reads
// both (the agent releases held burn-in spans and retries once, node/agent_gate.py).
static void annotate_init_error(Gate* g) {
  using LastError = const char* (*)(ncclComm_t);
  static LastError last = (LastError)dlsym(RTLD_DEFAULT, "ncclGetLastError");
  size_t len = strnlen(g->err, sizeof(g->err));
  if (last) {
    const char* why = last(nullptr);
    if (why && *why && len + 8 < sizeof(g->err)) {
      snprintf(g->err + len, sizeof(g->err) - len, " [rccl: %s]", why);
      len = strnlen(g->err, sizeof(g->err));
    }
  }
  size_t low = SIZE_MAX;
  int low_dev = -1;
  for (int d : g->devices) {
    const size_t f = device_free(d);
    if (f < low) { low = f; low_dev = d; }
  }
  if (low_dev >= 0 && len + 8 < sizeof(g->err))
    snprintf(g->err + len, sizeof(g->err) - len, " (device %d: %zu MiB free)", low_dev, low >> 20);
}

static void init_body(Gate* g, ncclUniqueId id) {
  HipNcclApi api{id};
  const size_t nd = g->devices.size();
  // this process's VRAM when the KFD accounting is reachable (not from inside a PID
  // namespace: its per-process entries are keyed by the host's pids), else the device's
  // used memory -- which counts whatever else allocates meanwhile: the agent keeps such a
  // number only for a window in which none of its burn-ins ran (node/agent_gate.py)
  auto used = [](int dev, bool per_process) -> long long {
    if (per_process) return proc_vram(dev);
    size_t free_b = 0, total_b = 0;
    if (hipSetDevice(dev) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) return -1;
    return (long long)(total_b - free_b);
  };
  bool per_process = true;
  std::vector<long long> before(nd);
  for (size_t d = 0; d < nd && per_process; ++d) per_process = (before[d] = proc_vram(g->devices[d])) >= 0;
  if (!per_process)
    for (size_t d = 0; d < nd; ++d) before[d] = used(g->devices[d], false);
  g->footprint_kind = per_process ? 1 : 2;
  const int r = tk_group_init(api, g->world, g->rank_base, (int)g->devices.size(), g->devices.data(),
                              g->comms.data(), g->err, sizeof(g->err));
  if (r != 0) annotate_init_error(g);
  auto taken = [&]() -> long long {  // growth on the most-grown GPU; -1 unknown
    long long most = 0;
    for (size_t d = 0; d < nd; ++d) {
      const long long now = used(g->devices[d], per_process);
      if (before[d] < 0 || now < 0) return -1;
      if (now - before[d] > most) most = now - before[d];
    }
    return most;
  };
  if (r == 0) g->footprint_comm = g->footprint_total = taken();
  if (r == 0 && g->prealloc_bytes) {
    // the sweep's buffers too, so the gate request only runs collectives
    g->bufs.resize(g->devices.size());
    for (size_t d = 0; d < g->devices.size(); ++d) {
      (void)hipSetDevice(g->devices[d]);
      if (alloc_bufs(g->bufs[d], g->prealloc_bytes) != 0) {
        for (auto& b : g->bufs) free_bufs(b);
        g->bufs.clear();
        break;
      }
    }
    g->footprint_total = taken();
  }
  bool orphan;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    g->init_ms = ms_since(g->t_begin);
    g->init_state = r == 0 ? 1 : -2;
    orphan = g->abandoned;
  }
  g_inits_running.fetch_sub(1);
  g->cv.notify_all();
  if (orphan) {  // released while initialising: nobody else will touch it
    for (size_t d = 0; d < g->bufs.size(); ++d) { (void)hipSetDevice(g->devices[d]); free_bufs(g->bufs[d]); }
    destroy_comms(g, /*abort=*/true);
    delete g;
    g_abandoned.fetch_sub(1);
  }
}

// 0 ready, -2 init failed, -3 timeout, -4 canceled.
static int gate_wait(Gate* g, double timeout_ms) {
  std::unique_lock<std::mutex> lk(g->mu);
  const bool done = g->cv.wait_for(lk, std::chrono::duration<double, std::milli>(timeout_ms),
                                   [g] { return g->init_state != 0 || g->cancel; });
  if (g->init_state == 0 && g->cancel) {
    snprintf(g_err, sizeof(g_err), "gate canceled while its communicator waited for peers");
    return -4;
  }
  if (!done) {
    snprintf(g_err, sizeof(g_err), "communicator not ready after %.0f ms", timeout_ms);
    return -3;
  }
  if (g->init_state < 0) {
    snprintf(g_err, sizeof(g_err), "%s", g->err);
    return -2;
  }
  return 0;
}

// Frees a gate taken out of the table: joins and destroys when its init is over, otherwise
// hands it to the (detached) init thread.
static void release_gate(Gate* g, bool abort) {
  {
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->init_state == 0) {
      g->abandoned = true;
      g->init_thread.detach();
      g_abandoned.fetch_add(1);
      return;
    }
  }
  if (g->init_thread.joinable()) g->init_thread.join();
  for (size_t d = 0; d < g->bufs.size(); ++d) { (void)hipSetDevice(g->devices[d]); free_bufs(g->bufs[d]); }
  destroy_comms(g, abort);
  delete g;
}

// Returns a handle > 0, or < 0 on error (tkr_last_error()).  prealloc_bytes > 0: the init
// thread also allocates the sweep buffers (largest message size) once the comms are up.
extern "C" int tkr_gate_begin_ex(const unsigned char* uid128, int world, int rank_base, int ndev,
                                 const int* devices, int blocking, size_t prealloc_bytes) {
  if (tk_check_geometry(world, rank_base, ndev, devices, g_err, sizeof(g_err))) return -1;
  ncclUniqueId id;
  memcpy(id.internal, uid128, NCCL_UNIQUE_ID_BYTES);
  Gate* g = new Gate();
  g->devices.assign(devices, devices + ndev);
  g->comms.assign(ndev, nullptr);
  g->rank_base = rank_base;
  g->world = world;
  g->prealloc_bytes = prealloc_bytes;
  g->t_begin = std::chrono::steady_clock::now();
  g_teardowns.touch();
  g_inits_running.fetch_add(1);
  if (blocking) {
    init_body(g, id);
    if (g->init_state < 0) {
      snprintf(g_err, sizeof(g_err), "%s", g->err);
      destroy_comms(g, true);
      delete g;
      return -2;
    }
  } else {
    g->init_thread = std::thread(init_body, g, id);
  }
  std::lock_guard<std::mutex> lk(g_gate_mu);
  const int h = g_next_gate++;
  g_gates.emplace_back(h, g);
  return h;
}

extern "C" int tkr_gate_begin(const unsigned char* uid128, int world, int rank_base, int ndev, const int* devices,
                              int blocking) {
  return tkr_gate_begin_ex(uid128, world, rank_base, ndev, devices, blocking, 0);
}

// 0 ready, 1 still initialising, < 0 error.
extern "C" int tkr_gate_poll(int h) {
  Gate* g = peek_gate(h);
  if (!g) { snprintf(g_err, sizeof(g_err), "unknown gate %d", h); return -1; }
  std::lock_guard<std::mutex> lk(g->mu);
  if (g->init_state < 0) { snprintf(g_err, sizeof(g_err), "%s", g->err); return -2; }
  return g->init_state == 1 ? 0 : 1;
}

// 0 released, 1 released while still initialising (init thread detached), -1 unknown handle.
extern "C" int tkr_gate_abort(int h) {
  Gate* g = take_gate(h);
  if (!g) return -1;
  int pending;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    pending = g->init_state == 0;
  }
  release_gate(g, /*abort=*/true);
  return pending;
}

// Stops a gate: a pending one is aborted (as tkr_gate_abort); one whose tkr_gate_sweep is
// waiting for its communicator's peers makes that sweep return -4 at once (a cluster gate
// whose other member failed must not wait out its timeout).  0 done, -1 unknown handle.
extern "C" int tkr_gate_cancel(int h) {
  {
    std::lock_guard<std::mutex> lk(g_gate_mu);
    for (auto& e : g_sweeping)
      if (e.first == h) {
        Gate* g = e.second;
        {
          std::lock_guard<std::mutex> glk(g->mu);
          g->cancel = true;
        }
        g->cv.notify_all();
        return 0;
      }
  }
  return tkr_gate_abort(h) < 0 ? -1 : 0;
}

extern "C" int tkr_gate_pending() {
  std::lock_guard<std::mutex> lk(g_gate_mu);
  return (int)g_gates.size();
}

// Completes the handle's init (waiting at most timeout_ms), runs the verified all-reduce sweep
// over its devices and tears the communicators down (async per tkr_set_async_teardown).  The
// handle is consumed.  phase_ms[0..4]: init wait in this call, alloc, sweep, teardown, and the
// total init time since begin.  Per-size outputs as for tkr_sweep_local (slowest device).
extern "C" int tkr_gate_sweep(int h, const size_t* sizes, int nsizes, int iters, int warmup, int dtype,
                              double timeout_ms, double* time_us, double* algbw, double* busbw, double* errors,
                              double* phase_ms) {
  Gate* g = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_gate_mu);
    for (size_t i = 0; i < g_gates.size(); ++i)
      if (g_gates[i].first == h) {
        g = g_gates[i].second;
        g_gates.erase(g_gates.begin() + (long)i);
        g_sweeping.emplace_back(h, g);  // cancelable while it waits for peers
        break;
      }
  }
  if (!g) { snprintf(g_err, sizeof(g_err), "unknown gate %d", h); return -1; }
  const int ndev = (int)g->devices.size();
  auto t_phase = std::chrono::steady_clock::now();
  int rc = gate_wait(g, timeout_ms);
  {
    std::lock_guard<std::mutex> lk(g_gate_mu);
    for (size_t i = 0; i < g_sweeping.size(); ++i)
      if (g_sweeping[i].second == g) {
        g_sweeping.erase(g_sweeping.begin() + (long)i);
        break;
      }
  }
  phase_ms[0] = ms_since(t_phase);
  phase_ms[4] = g->init_ms;
  if (rc) {
    release_gate(g, /*abort=*/true);
    return rc;
  }
  g_last_footprint[0] = (double)g->footprint_comm;
  g_last_footprint[1] = (double)g->footprint_total;
  g_last_footprint[2] = (double)g->footprint_kind;
  if (g->init_thread.joinable()) g->init_thread.join();
  size_t max_bytes = 0;
  for (int s = 0; s < nsizes; ++s) max_bytes = sizes[s] > max_bytes ? sizes[s] : max_bytes;
  std::vector<RankBufs> bufs;
  t_phase = std::chrono::steady_clock::now();
  if (!g->bufs.empty() && g->prealloc_bytes >= max_bytes) {
    bufs.swap(g->bufs);  // allocated by the init thread
  } else {
    for (size_t d = 0; d < g->bufs.size(); ++d) { (void)hipSetDevice(g->devices[d]); free_bufs(g->bufs[d]); }
    g->bufs.clear();
    bufs.resize(ndev);
    for (int d = 0; d < ndev && rc == 0; ++d) {
      if (hipSetDevice(g->devices[d]) != hipSuccess) { rc = -1; break; }
      rc = alloc_bufs(bufs[d], max_bytes);
    }
  }
  phase_ms[1] = ms_since(t_phase);
  t_phase = std::chrono::steady_clock::now();
  if (rc == 0) rc = check_verifiable(dtype, g->world);
  const float want = tk_verify_sum(dtype, g->world);
  auto run = [&](size_t count, int n) -> int {
    for (int it = 0; it < n; ++it) {
      ncclResult_t r = ncclGroupStart();
      for (int d = 0; d < ndev && r == ncclSuccess; ++d)
        r = ncclAllReduce(bufs[d].send, bufs[d].recv, count, nccl_type(dtype), ncclSum, g->comms[d],
                          bufs[d].stream);
      ncclResult_t re = ncclGroupEnd();
      if (r == ncclSuccess) r = re;
      if (r != ncclSuccess) {
        snprintf(g_err, sizeof(g_err), "ncclAllReduce: %s", ncclGetErrorString(r));
        return -2;
      }
    }
    return 0;
  };
  for (int s = 0; rc == 0 && s < nsizes; ++s) {
    const size_t count = sizes[s] / elem_size(dtype);
    for (int d = 0; d < ndev && rc == 0; ++d) {
      (void)hipSetDevice(g->devices[d]);
      rc = fill(bufs[d], count, dtype, tk_verify_value(dtype, g->world, g->rank_base + d));
    }
    if (rc || (rc = run(count, warmup)) != 0) break;
    for (int d = 0; d < ndev; ++d) { (void)hipSetDevice(g->devices[d]); (void)hipEventRecord(bufs[d].t0, bufs[d].stream); }
    if ((rc = run(count, iters)) != 0) break;
    double worst = 0.0;
    unsigned long long bad_total = 0;
    for (int d = 0; d < ndev && rc == 0; ++d) {
      (void)hipSetDevice(g->devices[d]);
      (void)hipEventRecord(bufs[d].t1, bufs[d].stream);
      rc = check(bufs[d], count, dtype, want);
    }
    for (int d = 0; d < ndev && rc == 0; ++d) {
      (void)hipSetDevice(g->devices[d]);
      if (hipStreamSynchronize(bufs[d].stream) != hipSuccess) { snprintf(g_err, sizeof(g_err), "stream sync failed"); rc = -1; break; }
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, bufs[d].t0, bufs[d].t1);
      if (ms > worst) worst = ms;
      unsigned long long bad = 0;
      (void)hipMemcpy(&bad, bufs[d].bad, sizeof(bad), hipMemcpyDeviceToHost);
      bad_total += bad;
    }
    if (rc) break;
    const double t = worst * 1e-3 / (iters > 0 ? iters : 1);
    time_us[s] = t * 1e6;
    algbw[s] = (double)sizes[s] / t / 1e9;
    busbw[s] = algbw[s] * (g->world > 1 ? 2.0 * (g->world - 1) / g->world : 1.0);
    errors[s] = (double)bad_total;
  }
  phase_ms[2] = ms_since(t_phase);
  t_phase = std::chrono::steady_clock::now();
  g_teardowns.touch();
  for (int d = 0; d < ndev; ++d) {
    teardown(g->comms[d], bufs[d], g->devices[d]);
    g->comms[d] = nullptr;
  }
  phase_ms[3] = ms_since(t_phase);
  delete g;
  return rc;
}

// Multi-process: one rank on one device (blocking init + sweep + teardown).  Kept as the
// single-call form of the gate; per-size outputs as above.
extern "C" int tkr_sweep_rank(int rank, int world, const unsigned char* uid128, int device, const size_t* sizes,
                              int nsizes, int iters, int warmup, int dtype, double* time_us, double* algbw,
                              double* busbw, double* errors) {
  const int h = tkr_gate_begin(uid128, world, rank, 1, &device, 1);
  if (h < 0) return h;
  double ph[5] = {0, 0, 0, 0, 0};
  const int rc = tkr_gate_sweep(h, sizes, nsizes, iters, warmup, dtype, 600000.0, time_us, algbw, busbw, errors, ph);
  g_last_init_ms = ph[4];
  g_phase_ms[0] = ph[4];
  g_phase_ms[1] = ph[1];
  g_phase_ms[2] = ph[2];
  g_phase_ms[3] = ph[3];
  return rc;
}

// Single process, all `ndev` local GPUs (ncclCommInitAll).  Same outputs; the
// error count is summed over devices, the time is the slowest device's.
extern "C" int tkr_sweep_local(int ndev, const size_t* sizes, int nsizes, int iters, int warmup, int dtype,
                               double* time_us, double* algbw, double* busbw, double* errors) {
  if (ndev < 1) { snprintf(g_err, sizeof(g_err), "ndev must be >= 1"); return -1; }
  std::vector<int> devs(ndev);
  for (int d = 0; d < ndev; ++d) devs[d] = d;
  std::vector<ncclComm_t> comms(ndev);
  const auto t_init = std::chrono::steady_clock::now();
  NCCLCHECK(ncclCommInitAll(comms.data(), ndev, devs.data()));
  g_last_init_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_init).count();
  size_t max_bytes = 0;
  for (int s = 0; s < nsizes; ++s) max_bytes = sizes[s] > max_bytes ? sizes[s] : max_bytes;
  std::vector<RankBufs> bufs(ndev);
  int rc = 0;
  for (int d = 0; d < ndev && rc == 0; ++d) {
    if (hipSetDevice(d) != hipSuccess) { rc = -1; break; }
    rc = alloc_bufs(bufs[d], max_bytes);
  }
  const float want = tk_verify_sum(dtype, ndev);
  for (int s = 0; rc == 0 && s < nsizes; ++s) {
    const size_t count = sizes[s] / elem_size(dtype);
    for (int d = 0; d < ndev && rc == 0; ++d) {
      (void)hipSetDevice(d);
      rc = fill(bufs[d], count, dtype, tk_verify_value(dtype, ndev, d));
    }
    if (rc) break;
    auto run = [&](int n) -> int {
      for (int it = 0; it < n; ++it) {
        NCCLCHECK(ncclGroupStart());
        ncclResult_t r = ncclSuccess;
        for (int d = 0; d < ndev && r == ncclSuccess; ++d)
          r = ncclAllReduce(bufs[d].send, bufs[d].recv, count, nccl_type(dtype), ncclSum, comms[d], bufs[d].stream);
        const ncclResult_t re = ncclGroupEnd();  // balanced even after a failed call inside the group
        if (r == ncclSuccess) r = re;
        if (r != ncclSuccess) {
          snprintf(g_err, sizeof(g_err), "ncclAllReduce: %s", ncclGetErrorString(r));
          return -2;
        }
      }
      return 0;
    };
    if ((rc = run(warmup)) != 0) break;
    for (int d = 0; d < ndev; ++d) { (void)hipSetDevice(d); (void)hipEventRecord(bufs[d].t0, bufs[d].stream); }
    if ((rc = run(iters)) != 0) break;
    double worst = 0.0;
    unsigned long long bad_total = 0;
    for (int d = 0; d < ndev && rc == 0; ++d) {
      (void)hipSetDevice(d);
      (void)hipEventRecord(bufs[d].t1, bufs[d].stream);
      rc = check(bufs[d], count, dtype, want);
    }
    for (int d = 0; d < ndev && rc == 0; ++d) {
      (void)hipSetDevice(d);
      if (hipStreamSynchronize(bufs[d].stream) != hipSuccess) { rc = -1; break; }
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, bufs[d].t0, bufs[d].t1);
      if (ms > worst) worst = ms;
      unsigned long long bad = 0;
      (void)hipMemcpy(&bad, bufs[d].bad, sizeof(bad), hipMemcpyDeviceToHost);
      bad_total += bad;
    }
    if (rc) break;
    const double t = worst * 1e-3 / (iters > 0 ? iters : 1);
    time_us[s] = t * 1e6;
    algbw[s] = (double)sizes[s] / t / 1e9;
    busbw[s] = algbw[s] * (ndev > 1 ? 2.0 * (ndev - 1) / ndev : 1.0);
    errors[s] = (double)bad_total;
  }
  for (int d = 0; d < ndev; ++d) {
    (void)hipSetDevice(d);
    free_bufs(bufs[d]);
    ncclCommDestroy(comms[d]);
  }
  return rc;
}

#ifdef TK_RCCL_MAIN
// {"error":"<msg>"} on stderr, the message escaped (RCCL's own error text can hold quotes)
static void print_error_json(const char* msg) {
  std::string o;
  for (const char* p = msg; *p; ++p) {
    const unsigned char c = static_cast<unsigned char>(*p);
    if (c == '"' || c == '\\') { o += '\\'; o += *p; }
    else if (c < 0x20) { char b[8]; snprintf(b, sizeof(b), "\\u%04x", c); o += b; }
    else o += *p;
  }
  fprintf(stderr, "{\"error\":\"%s\"}\n", o.c_str());
}

// Cluster mode (one process per node, all its GPUs): the cluster-wide gate for nodes that
// have no node agent (SSH / Terraform delivery; readiness/ssh_gate.py fans it out).
//   rank-0 node:  rccl-ready --cluster --world W --rank-base 0 --ngpus n --uid-out
//                 prints {"uid":"<256 hex>"} at once, then joins as ranks 0..n-1;
//   other nodes:  rccl-ready --cluster --world W --rank-base B --ngpus n --uid <hex>.
// Every process then runs the same verified all-reduce sweep (the agents' gate schedule:
// 1 MiB and --max-mib, warmup 2) and prints one JSON result line.
static int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

static int cluster_main(int world, int rank_base, int ndev, const char* uid_hex, bool uid_out, int max_mib,
                        int iters, int dtype, double min_busbw, double timeout_s) {
  unsigned char uid[NCCL_UNIQUE_ID_BYTES];
  if (uid_out) {
    if (tkr_unique_id(uid) != 0) {
      fprintf(stderr, "{\"error\":\"ncclGetUniqueId: %s\"}\n", g_err);
      return 2;
    }
    printf("{\"uid\":\"");
    for (int i = 0; i < NCCL_UNIQUE_ID_BYTES; ++i) printf("%02x", uid[i]);
    printf("\"}\n");
    fflush(stdout);
  } else {
    if (!uid_hex || strlen(uid_hex) != 2 * NCCL_UNIQUE_ID_BYTES) {
      fprintf(stderr, "{\"error\":\"--uid needs %d hex digits\"}\n", 2 * NCCL_UNIQUE_ID_BYTES);
      return 2;
    }
    for (int i = 0; i < NCCL_UNIQUE_ID_BYTES; ++i) {
      const int hi = hexval(uid_hex[2 * i]), lo = hexval(uid_hex[2 * i + 1]);
      if (hi < 0 || lo < 0) { fprintf(stderr, "{\"error\":\"bad --uid\"}\n"); return 2; }
      uid[i] = (unsigned char)(hi * 16 + lo);
    }
  }
  std::vector<int> devs(ndev);
  for (int d = 0; d < ndev; ++d) devs[d] = d;
  std::vector<size_t> sizes{1u << 20};
  if ((size_t)max_mib << 20 > sizes[0]) sizes.push_back((size_t)max_mib << 20);
  const int n = (int)sizes.size();
  const size_t max_bytes = sizes[n - 1];
  const int h = tkr_gate_begin_ex(uid, world, rank_base, ndev, devs.data(), /*blocking=*/0, max_bytes);
  if (h < 0) {
    print_error_json(g_err);
    return 2;
  }
  std::vector<double> t(n), alg(n), bus(n), err(n);
  double ph[5] = {0, 0, 0, 0, 0};
  const int rc = tkr_gate_sweep(h, sizes.data(), n, iters, 2, dtype, timeout_s * 1e3, t.data(), alg.data(),
                                bus.data(), err.data(), ph);
  if (rc) {
    print_error_json(g_err);
    printf("{\"ok\":false,\"world\":%d,\"rank_base\":%d,\"ngpus\":%d,\"error\":\"sweep failed\"}\n", world,
           rank_base, ndev);
    return 2;
  }
  double errs = 0;
  printf("{\"world\":%d,\"rank_base\":%d,\"ngpus\":%d,\"dtype\":\"%s\",\"init_ms\":%.1f,\"results\":[", world,
         rank_base, ndev, dtype ? "bf16" : "f32", ph[4]);
  for (int i = 0; i < n; ++i) {
    errs += err[i];
    printf("%s{\"bytes\":%zu,\"time_us\":%.2f,\"algbw_gbps\":%.2f,\"busbw_gbps\":%.2f,\"errors\":%.0f}", i ? "," : "",
           sizes[i], t[i], alg[i], bus[i], err[i]);
  }
  const bool ok = errs == 0 && bus[n - 1] >= min_busbw;
  // the communicator's device memory per GPU (node/agent_gate.py span_headroom; -1: unknown;
  // kind 1: this process's own VRAM, 2: the device's used memory)
  printf("],\"footprint_mib\":%.1f,\"footprint_total_mib\":%.1f,\"footprint_kind\":%.0f,\"ok\":%s}\n",
         tkr_last_footprint(0) < 0 ? -1.0 : tkr_last_footprint(0) / 1048576.0,
         tkr_last_footprint(1) < 0 ? -1.0 : tkr_last_footprint(1) / 1048576.0, tkr_last_footprint(2),
         ok ? "true" : "false");
  fflush(stdout);
  tkr_drain();
  return ok ? 0 : 1;
}

// True when /proc/self/maps has a librccl mapping whose real path is `want`'s.
static bool rccl_mapped(const char* want) {
  char want_real[PATH_MAX];
  if (!realpath(want, want_real)) return false;
  FILE* f = fopen("/proc/self/maps", "r");
  if (!f) return false;
  char line[PATH_MAX + 256];
  bool found = false;
  while (!found && fgets(line, sizeof line, f)) {
    const char* p = strchr(line, '/');
    if (!p || !strstr(p, "librccl")) continue;
    std::string path(p);
    while (!path.empty() && (path.back() == '\n' || path.back() == ' ')) path.pop_back();
    char real[PATH_MAX];
    found = realpath(path.c_str(), real) && !strcmp(real, want_real);
  }
  fclose(f);
  return found;
}

int main(int argc, char** argv) {
  double min_busbw = 0.0, timeout_s = 600.0;
  int iters = 20, warmup = 5, dtype = 0, world = 0, rank_base = 0, max_mib = 64, ngpus = 0;
  bool cluster = false, uid_out = false, max_set = false, preload = false;
  const char* uid_hex = nullptr;
  const char* expect_rccl = nullptr;  // --expect-rccl: the librccl this process must have mapped
  // The command line is read before the GPU is touched: a value that does not parse
  // (atof("abc") == 0 turned the bandwidth floor off) or an unknown option is a usage error.
  const char* bad = nullptr;
  const auto want = [&](int& i) -> const char* {
    if (i + 1 >= argc) { bad = argv[i]; return nullptr; }
    return argv[++i];
  };
  const auto real = [&](int& i, double* out, bool positive) {
    const char* opt = argv[i];
    const char* v = want(i);
    if (!v) return;
    char* end = nullptr;
    const double x = strtod(v, &end);
    if (!*v || *end || !std::isfinite(x) || x < 0 || (positive && x == 0)) bad = opt;
    else *out = x;
  };
  const auto whole = [&](int& i, int* out, long lo) {
    const char* opt = argv[i];
    const char* v = want(i);
    if (!v) return;
    char* end = nullptr;
    errno = 0;
    const long x = strtol(v, &end, 10);
    if (!*v || *end || errno == ERANGE || x < lo || x > INT_MAX || isspace((unsigned char)*v)) bad = opt;
    else *out = (int)x;
  };
  for (int i = 1; i < argc && !bad; ++i) {
    const char* a = argv[i];
    if (!strcmp(a, "--min-busbw")) real(i, &min_busbw, false);
    else if (!strcmp(a, "--iters")) whole(i, &iters, 1);
    else if (!strcmp(a, "--ngpus")) whole(i, &ngpus, 1);
    else if (!strcmp(a, "--bf16")) dtype = 1;
    else if (!strcmp(a, "--cluster")) cluster = true;
    else if (!strcmp(a, "--world")) whole(i, &world, 1);
    else if (!strcmp(a, "--rank-base")) whole(i, &rank_base, 0);
    else if (!strcmp(a, "--uid")) uid_hex = want(i);
    else if (!strcmp(a, "--uid-out")) uid_out = true;
    else if (!strcmp(a, "--max-mib")) { whole(i, &max_mib, 1); max_set = true; }
    else if (!strcmp(a, "--timeout-s")) real(i, &timeout_s, true);
    else if (!strcmp(a, "--expect-rccl")) expect_rccl = want(i);
    else if (!strcmp(a, "--preload")) preload = true;  // tkr_preload_device_code first
    else bad = a;
  }
  if (bad) {
    print_error_json(("usage: unknown option, or a bad or missing value, at '" + std::string(bad) + "'").c_str());
    return 64;
  }
  int visible = 0;
  if (hipGetDeviceCount(&visible) != hipSuccess || visible < 1) {
    fprintf(stderr, "{\"error\":\"no HIP devices\"}\n");
    return 3;
  }
  const int ndev = ngpus ? ngpus : visible;
  if (ndev < 1 || ndev > visible) {
    fprintf(stderr, "{\"error\":\"--ngpus %d but %d visible\"}\n", ndev, visible);
    return 3;
  }
  if (preload) {  // what a node agent does at start (the communicator then finds the code loaded)
    std::vector<int> devs(ndev);
    for (int d = 0; d < ndev; ++d) devs[d] = d;
    if (tkr_preload_device_code(ndev, devs.data()) < 0) fprintf(stderr, "preload: %s\n", g_err);
  }
  struct PreloadJoin {  // no preload thread outlives main
    ~PreloadJoin() {
      while (tkr_preloads_running() > 0) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
  } preload_join;
  if (cluster) {
    if (world < ndev || rank_base < 0 || rank_base + ndev > world || (!uid_out && !uid_hex) || max_mib < 1) {
      fprintf(stderr, "{\"error\":\"cluster mode needs --world >= --rank-base + --ngpus and --uid or --uid-out\"}\n");
      return 2;
    }
    if (check_verifiable(dtype, world)) {  // refused before any communicator exists
      print_error_json(g_err);
      return 2;
    }
    return cluster_main(world, rank_base, ndev, uid_hex, uid_out, max_mib, iters, dtype, min_busbw, timeout_s);
  }
  std::vector<size_t> sizes;
  const size_t top = max_set ? ((size_t)(max_mib < 1 ? 1 : max_mib) << 20) : (1ull << 30);
  for (size_t b = 1u << 20; b <= top; b <<= 2) sizes.push_back(b);
  const int n = (int)sizes.size();
  std::vector<double> t(n), alg(n), bus(n), err(n);
  int rc = tkr_sweep_local(ndev, sizes.data(), n, iters, warmup, dtype, t.data(), alg.data(), bus.data(), err.data());
  if (rc) {
    print_error_json(g_err);
    return 2;
  }
  double errs = 0;
  printf("{\"ngpus\":%d,\"dtype\":\"%s\",\"results\":[", ndev, dtype ? "bf16" : "f32");
  for (int i = 0; i < n; ++i) {
    errs += err[i];
    printf("%s{\"bytes\":%zu,\"time_us\":%.2f,\"algbw_gbps\":%.2f,\"busbw_gbps\":%.2f,\"errors\":%.0f}", i ? "," : "",
           sizes[i], t[i], alg[i], bus[i], err[i]);
  }
  bool ok = errs == 0 && bus[n - 1] >= min_busbw;
  printf("]");
  if (expect_rccl) {
    // the opt-in single-target RCCL is verified by a run that provably loaded it
    const bool mapped = rccl_mapped(expect_rccl);
    printf(",\"expect_rccl\":\"%s\",\"rccl_mapped\":%s", expect_rccl, mapped ? "true" : "false");
    ok = ok && mapped;
  }
  printf(",\"ok\":%s}\n", ok ? "true" : "false");
  return ok ? 0 : 1;
}
#endif
