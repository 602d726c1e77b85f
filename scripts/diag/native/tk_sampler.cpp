// In-process native stack sampler (diagnostic tool, not part of the product).
//
// Samples one thread (or, with tid <= 0, every thread) of the calling process: a sampler
// thread sends SIGPROF to the target(s) every `interval_us`, the handler records its native backtrace, and tks_stop()
// resolves the frames (dladdr: shared object + nearest exported symbol + offset) and writes
// one line per sample ("obj!sym+0xoff;..." leaf first) to a file.  Used to find where an
// RCCL communicator init spends its ~45 ms (scripts/rccl_init_sampler.py): the HIP, HSA
// and libc entry points on the stack are exported symbols, so the leaf and the first
// HIP API frame name the cost even in stripped libraries.
//
// Build: g++ -O2 -shared -fPIC -o tk_sampler.so tk_sampler.cpp -ldl -lpthread

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <dirent.h>

#include <cerrno>
#include <cstdlib>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

namespace {
constexpr int kMaxFrames = 40;
constexpr int kMaxSamples = 100000;
struct Sample {
  int tid;
  int n;
  void* pc[kMaxFrames];
};
Sample* g_samples = nullptr;
std::atomic<int> g_count{0};
std::atomic<bool> g_run{false};
std::thread g_thread;
struct sigaction g_old;

void on_prof(int, siginfo_t*, void*) {
  const int saved = errno;
  const int i = g_count.fetch_add(1, std::memory_order_relaxed);
  if (i < kMaxSamples) {
    g_samples[i].tid = (int)syscall(SYS_gettid);
    g_samples[i].n = backtrace(g_samples[i].pc, kMaxFrames);
  }
  errno = saved;
}

std::string frame(void* pc) {
  Dl_info info;
  char buf[512];
  if (dladdr(pc, &info) && info.dli_fname) {
    const char* base = strrchr(info.dli_fname, '/');
    base = base ? base + 1 : info.dli_fname;
    if (info.dli_sname)
      snprintf(buf, sizeof(buf), "%s!%s+0x%lx", base, info.dli_sname,
               (unsigned long)((char*)pc - (char*)info.dli_saddr));
    else
      snprintf(buf, sizeof(buf), "%s!?+0x%lx", base, (unsigned long)((char*)pc - (char*)info.dli_fbase));
    return buf;
  }
  snprintf(buf, sizeof(buf), "?!%p", pc);
  return buf;
}
}  // namespace

extern "C" int tks_start(int tid, int interval_us) {
  if (g_run.load()) return -1;
  if (!g_samples) g_samples = new Sample[kMaxSamples];
  g_count = 0;
  void* warm[4];
  backtrace(warm, 4);  // loads the unwinder before any signal arrives
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, &g_old) != 0) return -2;
  g_run = true;
  const pid_t pid = getpid();
  g_thread = std::thread([=] {
    const pid_t self = (pid_t)syscall(SYS_gettid);
    while (g_run.load()) {
      if (tid > 0) {
        syscall(SYS_tgkill, pid, tid, SIGPROF);
      } else if (DIR* d = opendir("/proc/self/task")) {  // tid <= 0: every thread but this one
        while (struct dirent* e = readdir(d)) {
          const int t = atoi(e->d_name);
          if (t > 0 && t != self) syscall(SYS_tgkill, pid, t, SIGPROF);
        }
        closedir(d);
      }
      usleep(interval_us);
    }
  });
  return 0;
}

// Stops sampling and writes the samples to `path`; returns how many were written.
extern "C" int tks_stop(const char* path) {
  if (!g_run.exchange(false)) return -1;
  g_thread.join();
  usleep(2000);  // a signal in flight lands before the handler is restored
  sigaction(SIGPROF, &g_old, nullptr);
  const int n = g_count.load() < kMaxSamples ? g_count.load() : kMaxSamples;
  FILE* f = fopen(path, "w");
  if (!f) return -3;
  for (int i = 0; i < n; ++i) {
    // frame 0 is the handler, 1 the signal trampoline
    fprintf(f, "%d ", g_samples[i].tid);
    for (int k = 2; k < g_samples[i].n; ++k) fprintf(f, "%s%s", k > 2 ? ";" : "", frame(g_samples[i].pc[k]).c_str());
    fputc('\n', f);
  }
  fclose(f);
  return n;
}
