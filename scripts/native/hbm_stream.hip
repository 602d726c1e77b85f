// HBM streaming microbenchmark (diagnostic): read / write / copy kernel variants and grid
// sizes on 1 and 4 GiB buffers, best of 5 timed launches after warm-up.  Used to tune the
// k_stream_* kernels of triton_kubernetes_amd/ops/csrc/tk_gpu_probe.hip.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_stream hbm_stream.hip

#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((ext_vector_type(4))) float f32x4;
constexpr int T = 256;

// grid-stride, U independent 16-B accesses in flight per lane (the production shape)
template <int U, bool NT_LOAD>
__global__ __launch_bounds__(T) void rd_stride(const f32x4* __restrict__ src, size_t n4, float* sink) {
  const size_t stride = (size_t)gridDim.x * T;
  size_t i = (size_t)blockIdx.x * T + threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT_LOAD ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  for (; i < n4; i += stride) acc += src[i];
  const float s = acc[0] + acc[1] + acc[2] + acc[3];
  if (s == 1.2345678e-30f) sink[threadIdx.x] = s;
}

// each block owns one contiguous chunk, U accesses in flight per lane
template <int U>
__global__ __launch_bounds__(T) void rd_chunk(const f32x4* __restrict__ src, size_t n4, float* sink) {
  const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const size_t b = (size_t)blockIdx.x * per, e = b + per < n4 ? b + per : n4;
  f32x4 acc = {0, 0, 0, 0};
  size_t i = b + threadIdx.x;
  for (; i + (U - 1) * T < e; i += U * T) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + i + u * T);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  for (; i < e; i += T) acc += src[i];
  const float s = acc[0] + acc[1] + acc[2] + acc[3];
  if (s == 1.2345678e-30f) sink[threadIdx.x] = s;
}

template <int U, bool NT_STORE>
__global__ __launch_bounds__(T) void wr_stride(f32x4* __restrict__ dst, size_t n4, float v) {
  const size_t stride = (size_t)gridDim.x * T;
  const f32x4 x = {v, v + 1.f, v + 2.f, v + 3.f};
  size_t i = (size_t)blockIdx.x * T + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (NT_STORE) __builtin_nontemporal_store(x, dst + i + u * stride);
      else dst[i + u * stride] = x;
    }
  }
  for (; i < n4; i += stride) dst[i] = x;
}

template <int U>
__global__ __launch_bounds__(T) void wr_chunk(f32x4* __restrict__ dst, size_t n4, float v) {
  const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const size_t b = (size_t)blockIdx.x * per, e = b + per < n4 ? b + per : n4;
  const f32x4 x = {v, v + 1.f, v + 2.f, v + 3.f};
  size_t i = b + threadIdx.x;
  for (; i + (U - 1) * T < e; i += U * T) {
#pragma unroll
    for (int u = 0; u < U; ++u) dst[i + u * T] = x;
  }
  for (; i < e; i += T) dst[i] = x;
}

template <int U, bool NT_LOAD>
__global__ __launch_bounds__(T) void cp_stride(const f32x4* __restrict__ src, f32x4* __restrict__ dst, size_t n4) {
  const size_t stride = (size_t)gridDim.x * T;
  size_t i = (size_t)blockIdx.x * T + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT_LOAD ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) dst[i + u * stride] = v[u];
  }
  for (; i < n4; i += stride) dst[i] = src[i];
}

template <int U>
__global__ __launch_bounds__(T) void cp_chunk(const f32x4* __restrict__ src, f32x4* __restrict__ dst, size_t n4) {
  const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const size_t b = (size_t)blockIdx.x * per, e = b + per < n4 ? b + per : n4;
  size_t i = b + threadIdx.x;
  for (; i + (U - 1) * T < e; i += U * T) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + i + u * T);
#pragma unroll
    for (int u = 0; u < U; ++u) dst[i + u * T] = v[u];
  }
  for (; i < e; i += T) dst[i] = src[i];
}

template <typename F>
static double best_ms(F launch) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch();
  launch();
  (void)hipDeviceSynchronize();
  double best = 1e30;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(a);
    launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return best;
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  f32x4 *a, *b;
  float* sink;
  const size_t maxb = 4ull << 30;
  (void)hipMalloc(&a, maxb);
  (void)hipMalloc(&b, maxb);
  (void)hipMalloc(&sink, 4096);
  (void)hipMemset(a, 0, maxb);
  (void)hipMemset(b, 0, maxb);
  for (size_t bytes : {1ull << 30, 4ull << 30}) {
    const size_t n4 = bytes / 16;
    for (int bpcu : {4, 8, 16, 32}) {
      const int g = cus * bpcu;
#define R(name, expr, moved)                                                                              \
  do {                                                                                                    \
    const double ms = best_ms([&] { expr; });                                                             \
    printf("{\"kernel\": \"%s\", \"gib\": %zu, \"blocks_per_cu\": %d, \"ms\": %.4f, \"tbps\": %.3f}\n", name, \
           bytes >> 30, bpcu, ms, (double)(moved) / (ms * 1e-3) / 1e12);                                  \
  } while (0)
      R("rd_stride_u8_nt", (rd_stride<8, true><<<g, T>>>(a, n4, sink)), bytes);
      R("rd_stride_u8", (rd_stride<8, false><<<g, T>>>(a, n4, sink)), bytes);
      R("rd_stride_u4_nt", (rd_stride<4, true><<<g, T>>>(a, n4, sink)), bytes);
      R("rd_chunk_u8", (rd_chunk<8><<<g, T>>>(a, n4, sink)), bytes);
      R("wr_stride_u8", (wr_stride<8, false><<<g, T>>>(b, n4, 1.f)), bytes);
      R("wr_stride_u4", (wr_stride<4, false><<<g, T>>>(b, n4, 1.f)), bytes);
      R("wr_stride_u8_nt", (wr_stride<8, true><<<g, T>>>(b, n4, 1.f)), bytes);
      R("wr_chunk_u8", (wr_chunk<8><<<g, T>>>(b, n4, 1.f)), bytes);
      R("cp_stride_u8_nt", (cp_stride<8, true><<<g, T>>>(a, b, n4)), 2 * bytes);
      R("cp_stride_u8", (cp_stride<8, false><<<g, T>>>(a, b, n4)), 2 * bytes);
      R("cp_stride_u4_nt", (cp_stride<4, true><<<g, T>>>(a, b, n4)), 2 * bytes);
      R("cp_chunk_u8", (cp_chunk<8><<<g, T>>>(a, b, n4)), 2 * bytes);
    }
  }
  return 0;
}
