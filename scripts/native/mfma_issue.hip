// MFMA issue-rate microbenchmark (diagnostic): FLOP per clock per SIMD of register-resident
// MFMA loops under loop-unroll / accumulator-count / waves-per-SIMD variants, with the
// in-kernel clock from s_memtime / s_memrealtime after ~1 s of back-to-back launches.
// Used to tune k_mfma_* in triton_kubernetes_amd/ops/csrc/tk_gpu_probe.hip.
//
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form -o mfma_issue mfma_issue.hip

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float rnd_unit(uint32_t seed) {
  return ((hash32(seed) >> 8) * (1.0f / 8388608.0f)) - 1.0f + (1.0f / 16777216.0f);
}

template <int ACC, int UNROLL, bool FP8>
__global__ __launch_bounds__(256) void k_loop(float* out, int iters, unsigned long long* stamps) {
  const uint32_t lane = blockIdx.x * 256 + threadIdx.x;
  bf16x8 a, b;
  i32x8 a8, b8;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)rnd_unit(lane * 16 + j);
    b[j] = (__bf16)rnd_unit(lane * 16 + 8 + j);
    a8[j] = (int)(hash32(lane * 16 + j) & 0x3e3e3e3eU);
    b8[j] = (int)(hash32(lane * 16 + 8 + j) & 0x3e3e3e3eU);
  }
  f32x4 acc[ACC];
#pragma unroll
  for (int c = 0; c < ACC; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i += UNROLL) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
      for (int c = 0; c < ACC; ++c) {
        if constexpr (FP8)
          acc[c] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8, b8, acc[c], 0, 0, 0, 127, 0, 127);
        else
          acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[c], 0, 0, 0);
      }
    }
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < ACC; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  if (s == 1.2345678e-30f) out[lane] = s;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = c1 - c0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int ACC, int UNROLL, bool FP8>
static void run(const char* name, int bpcu, int cus) {
  const int grid = cus * bpcu;
  const int iters = FP8 ? 8192 : 16384;  // multiple of every UNROLL
  float* sink;
  unsigned long long* st;
  (void)hipMalloc(&sink, (size_t)grid * 256 * 4);
  (void)hipMalloc(&st, (size_t)grid * 16);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const auto w0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count() < 1.0) {
    for (int k = 0; k < 4; ++k) k_loop<ACC, UNROLL, FP8><<<grid, 256>>>(sink, iters, st);
    (void)hipDeviceSynchronize();
  }
  (void)hipEventRecord(e0);
  k_loop<ACC, UNROLL, FP8><<<grid, 256>>>(sink, iters, st);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h((size_t)grid * 2);
  (void)hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> mhz, cyc;
  for (int i = 0; i < grid; ++i) {
    mhz.push_back((double)h[2 * i] / h[2 * i + 1] * 100.0);
    cyc.push_back((double)h[2 * i]);
  }
  std::sort(mhz.begin(), mhz.end());
  std::sort(cyc.begin(), cyc.end());
  const double flop_inst = FP8 ? 2.0 * 16 * 16 * 128 : 2.0 * 16 * 16 * 32;
  const double flops = (double)grid * 4 * iters * ACC * flop_inst;
  const double clk = mhz[mhz.size() / 2];
  // cycles per MFMA per SIMD from the median workgroup's own stamps (waves per SIMD = bpcu)
  const double mfma_per_simd = (double)iters * ACC * bpcu;
  printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"acc\": %d, \"unroll\": %d, \"mhz\": %.0f, "
         "\"tflops\": %.1f, \"flop_per_clk_per_simd\": %.1f, \"cyc_per_mfma\": %.2f}\n",
         name, bpcu, ACC, UNROLL, clk, flops / (ms * 1e-3) / 1e12, flops / (ms * 1e-3) / (clk * 1e6) / (cus * 4.0),
         cyc[cyc.size() / 2] / mfma_per_simd);
  (void)hipFree(sink);
  (void)hipFree(st);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  for (int bpcu : {1, 2}) {
    run<4, 1, false>("bf16", bpcu, cus);
    run<4, 4, false>("bf16", bpcu, cus);
    run<8, 2, false>("bf16", bpcu, cus);
    run<16, 1, false>("bf16", bpcu, cus);
    run<4, 1, true>("fp8", bpcu, cus);
    run<4, 4, true>("fp8", bpcu, cus);
    run<8, 2, true>("fp8", bpcu, cus);
  }
  return 0;
}
