// Where the full burn-in's allocation time goes: one scenario per process run.
//   alloc_probe <scenario> [chunk_gib]
//   fresh     : the span's chunks allocated in a fresh process
//   prefree   : 2 x 16 GiB allocated, touched and freed first (the stream bench's buffers)
//   presync   : as prefree, then hipDeviceSynchronize before the span
//   untouched : 2 x 16 GiB allocated and freed without a kernel touching them
// Prints one JSON line: per-chunk hipMalloc ms, total alloc/free ms.  Leaves 8 GiB free.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

__global__ void k_touch(float4* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

#define OK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  const char* scenario = argc > 1 ? argv[1] : "fresh";
  const size_t chunk = (size_t)(argc > 2 ? atoi(argv[2]) : 16) << 30;
  const auto t_init = std::chrono::steady_clock::now();
  OK(hipSetDevice(0));
  OK(hipFree(nullptr));
  const double init_ms = ms_since(t_init);
  double pre_ms = 0.0;
  if (strcmp(scenario, "fresh") != 0) {
    const auto t = std::chrono::steady_clock::now();
    void* a = nullptr;
    void* b = nullptr;
    OK(hipMalloc(&a, 16ull << 30));
    OK(hipMalloc(&b, 16ull << 30));
    if (strcmp(scenario, "untouched") != 0) {
      k_touch<<<4096, 256>>>(static_cast<float4*>(a), (16ull << 30) / sizeof(float4));
      k_touch<<<4096, 256>>>(static_cast<float4*>(b), (16ull << 30) / sizeof(float4));
      OK(hipGetLastError());
      OK(hipDeviceSynchronize());
    }
    OK(hipFree(a));
    OK(hipFree(b));
    if (strcmp(scenario, "presync") == 0) OK(hipDeviceSynchronize());
    pre_ms = ms_since(t);
  }
  size_t free_b = 0, total_b = 0;
  OK(hipMemGetInfo(&free_b, &total_b));
  const size_t want = free_b > (8ull << 30) ? free_b - (8ull << 30) : 0;
  std::vector<void*> chunks;
  std::vector<double> per;
  const auto t_alloc = std::chrono::steady_clock::now();
  for (size_t done = 0; done < want;) {
    const size_t n = want - done < chunk ? want - done : chunk;
    void* p = nullptr;
    const auto t = std::chrono::steady_clock::now();
    if (hipMalloc(&p, n) != hipSuccess) {
      (void)hipGetLastError();
      break;
    }
    per.push_back(ms_since(t));
    chunks.push_back(p);
    done += n;
  }
  const double alloc_ms = ms_since(t_alloc);
  const auto t_touch = std::chrono::steady_clock::now();
  for (size_t i = 0; i < chunks.size(); ++i) {
    const size_t n = (i + 1 < chunks.size() ? chunk : want - chunk * (chunks.size() - 1)) / sizeof(float4);
    k_touch<<<4096, 256>>>(static_cast<float4*>(chunks[i]), n);
  }
  OK(hipGetLastError());
  OK(hipDeviceSynchronize());
  const double touch_ms = ms_since(t_touch);
  const auto t_free = std::chrono::steady_clock::now();
  for (void* p : chunks) OK(hipFree(p));
  const double free_ms = ms_since(t_free);
  const auto t_sync = std::chrono::steady_clock::now();
  OK(hipDeviceSynchronize());
  size_t free_after = 0;
  OK(hipMemGetInfo(&free_after, &total_b));
  const double post_ms = ms_since(t_sync);
  printf("{\"scenario\": \"%s\", \"chunk_gib\": %zu, \"init_ms\": %.1f, \"pre_ms\": %.1f, \"free_gib\": %.1f, "
         "\"chunks\": %zu, \"alloc_ms\": %.1f, \"touch_ms\": %.1f, \"free_ms\": %.1f, \"post_ms\": %.1f, "
         "\"free_after_gib\": %.1f, \"per_chunk_ms\": [",
         scenario, chunk >> 30, init_ms, pre_ms, free_b / 1073741824.0, chunks.size(), alloc_ms, touch_ms, free_ms,
         post_ms, free_after / 1073741824.0);
  for (size_t i = 0; i < per.size(); ++i) printf("%s%.2f", i ? ", " : "", per[i]);
  printf("]}\n");
  fflush(stdout);
  return 0;
}
