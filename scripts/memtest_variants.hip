// GPU box: the span memtest's fill/check kernels (ops/csrc/tk_gpu_probe.hip k_mem_fill /
// k_mem_check) against variants, on one 1 GiB chunk (what the agent's span uses) and on
// 16 GiB.  Prints one JSON line per (kernel, variant, size): GB/s (best of 5) and errors.
//   variants: plain (as shipped), nt (non-temporal loads/stores, as the stream kernels)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int THREADS = 256;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int UNROLL = 8;

#define OK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

struct Slice {
  size_t begin, end;
};
__device__ __forceinline__ Slice block_slice(size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t b = (size_t)blockIdx.x * per;
  return {b < n ? b : n, b + per < n ? b + per : n};
}
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint4 pattern(size_t i, uint32_t seed) {
  const uint32_t h = hash32((uint32_t)i ^ seed ^ (uint32_t)(i >> 32) * 0x9e3779b9U);
  return make_uint4(h, ~h, h ^ 0xa5a5a5a5U, h * 0x01000193U);
}

template <bool NT>
__global__ __launch_bounds__(THREADS) void k_fill(uint4* __restrict__ p, size_t n, uint32_t seed) {
  const Slice sl = block_slice(n);
  size_t i = sl.begin + threadIdx.x;
  for (; i + (UNROLL - 1) * THREADS < sl.end; i += UNROLL * THREADS) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint4 w = pattern(i + u * THREADS, seed);
      if (NT) {
        const u32x4 x = {w.x, w.y, w.z, w.w};
        __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p) + i + u * THREADS);
      } else {
        p[i + u * THREADS] = w;
      }
    }
  }
  for (; i < sl.end; i += THREADS) p[i] = pattern(i, seed);
}

template <bool NT>
__global__ __launch_bounds__(THREADS) void k_check(const uint4* __restrict__ p, size_t n, uint32_t seed,
                                                   unsigned long long* __restrict__ errors) {
  const Slice sl = block_slice(n);
  uint32_t bad = 0;
  auto cmp = [&](const uint4 v, size_t j) {
    const uint4 w = pattern(j, seed);
    bad += (v.x != w.x) + (v.y != w.y) + (v.z != w.z) + (v.w != w.w);
  };
  size_t i = sl.begin + threadIdx.x;
  for (; i + (UNROLL - 1) * THREADS < sl.end; i += UNROLL * THREADS) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (NT) {
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p) + i + u * THREADS);
        v[u] = make_uint4(x.x, x.y, x.z, x.w);
      } else {
        v[u] = p[i + u * THREADS];
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) cmp(v[u], i + u * THREADS);
  }
  for (; i < sl.end; i += THREADS) cmp(p[i], i);
  for (int off = 32; off > 0; off >>= 1) bad += __shfl_down(bad, off, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(errors, (unsigned long long)bad);
}

int main() {
  hipDeviceProp_t prop;
  OK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount * 16;
  const size_t big = 16ull << 30;
  uint4* p = nullptr;
  unsigned long long* err = nullptr;
  OK(hipMalloc(&p, big));
  OK(hipMalloc(&err, sizeof(unsigned long long)));
  hipEvent_t a, b;
  OK(hipEventCreate(&a));
  OK(hipEventCreate(&b));
  for (size_t bytes : {(size_t)1 << 30, big}) {
    const size_t n = bytes / sizeof(uint4);
    for (int nt = 0; nt < 2; ++nt) {
      float best_fill = 1e30f, best_check = 1e30f;
      unsigned long long h = 0;
      for (int rep = 0; rep < 5; ++rep) {
        const uint32_t seed = 0x1234567u + 977u * (uint32_t)rep;
        float ms = 0.f;
        OK(hipEventRecord(a));
        if (nt) k_fill<true><<<grid, THREADS>>>(p, n, seed);
        else k_fill<false><<<grid, THREADS>>>(p, n, seed);
        OK(hipEventRecord(b));
        OK(hipEventSynchronize(b));
        OK(hipEventElapsedTime(&ms, a, b));
        best_fill = std::min(best_fill, ms);
        OK(hipMemset(err, 0, sizeof(unsigned long long)));
        OK(hipEventRecord(a));
        if (nt) k_check<true><<<grid, THREADS>>>(p, n, seed, err);
        else k_check<false><<<grid, THREADS>>>(p, n, seed, err);
        OK(hipEventRecord(b));
        OK(hipEventSynchronize(b));
        OK(hipEventElapsedTime(&ms, a, b));
        best_check = std::min(best_check, ms);
        unsigned long long e = 0;
        OK(hipMemcpy(&e, err, sizeof(e), hipMemcpyDeviceToHost));
        h += e;
      }
      printf("{\"variant\": \"%s\", \"gib\": %zu, \"fill_gbps\": %.1f, \"check_gbps\": %.1f, \"fill_us\": %.1f, "
             "\"check_us\": %.1f, \"errors\": %llu}\n",
             nt ? "nt" : "plain", bytes >> 30, bytes / (best_fill * 1e-3) / 1e9, bytes / (best_check * 1e-3) / 1e9,
             best_fill * 1e3, best_check * 1e3, h);
      fflush(stdout);
    }
  }
  OK(hipFree(p));
  OK(hipFree(err));
  return 0;
}
