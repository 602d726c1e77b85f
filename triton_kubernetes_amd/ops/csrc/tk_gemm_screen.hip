// MI355X GEMM silent-data-corruption screen (burn-in step `gemm`).
//
// The MFMA peak loops in tk_gpu_probe.hip prove the matrix cores ISSUE at rate, but they
// never check a result.  This screen runs a real LDS-tiled bf16 GEMM — HBM -> LDS (async
// global_load_lds) -> VGPR fragments -> v_mfma_f32_16x16x32_bf16 — and verifies it with
// algorithm-based fault tolerance (Huang & Abraham): for C = A * B^T,
//
//     sum_m C[m][n] = sum_k (sum_m A[m][k]) * B[n][k]      (column checksums)
//     sum_n C[m][n] = sum_k A[m][k] * (sum_n B[n][k])      (row checksums)
//
// The GEMM epilogue reduces its accumulator tile to per-wave column/row partial sums in
// registers (no C store in screen mode), and independent fp32 SIMT kernels compute the
// right-hand sides from A and B.  A corrupted product — a bad MFMA, LDS or VGPR bit, a
// wrong staged tile — shows up as a column AND a row mismatch, which also locates it.
//
// Kernel structure (gfx950, one 256x256 output tile per 512-thread workgroup, 8 waves,
// 128 KiB of LDS, K in steps of 64, 16-byte buffer_load ... lds copies HBM -> LDS):
//  * default, k_gemm8 (schedule 1, "staggered"): the LDS holds half-tiles ([128][64] bf16
//    of A or B, two K-tiles deep); each wave owns four 64x32 quadrants and a K-tile is two
//    phases of 32 MFMAs; the two wave groups run one barrier apart, so on every SIMD one
//    wave issues MFMAs while the other reads LDS and issues copies (details at the kernel).
//    1.41 / 1.54 PF at 4096^3 / 8192^3 on random data, MFMA pipe 77 % busy;
//  * k_gemm_bt (schedule 0, "single-barrier", kept for A/B): whole [256][64] tiles in two
//    buffers, one barrier per K-step, every wave reads then issues 64 MFMAs in lockstep —
//    1.20 / 1.27 PF, MFMA pipe 61.5 % busy (profiles/round1/round1_gemm_pmc.md);
//  * the LDS image is XOR-swizzled by 16-byte chunk (chunk ^ ((row >> 1) & 7)): the
//    swizzle is applied to the per-lane GLOBAL source address (the LDS-DMA destination
//    is lane-linear), so the 16 lanes of a ds_read_b128 group read 16 distinct bank
//    slots (row stride 128 B would otherwise give an 8-way conflict; 0 conflicts measured);
//  * blocks are remapped so the tiles one XCD works on share A rows / B columns in its
//    own L2 (blocks are dispatched round-robin over the 8 XCDs);
//  * shapes: M, N multiples of 256, K a multiple of 64 — checked on the host before any
//    launch (no bounds checks inside the tile loops).
//
// C ABI for ctypes: triton_kubernetes_amd/ops/gemm.py.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;

static thread_local char g_err[512];

static int set_err(const char* what, hipError_t e) {
  snprintf(g_err, sizeof(g_err), "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
  return (int)e == 0 ? -1 : (int)e;
}

#define CHECK(call)                                  \
  do {                                               \
    hipError_t _e = (call);                          \
    if (_e != hipSuccess) return set_err(#call, _e); \
  } while (0)

extern "C" const char* tkg_last_error() { return g_err; }

namespace {
#ifndef TKG_BK
#define TKG_BK 64
#endif
#ifndef TKG_DEFAULT_SCHED
#define TKG_DEFAULT_SCHED 1
#endif
#ifndef TKG8_STAGGER  // staggered schedule: wave group 1 one barrier behind group 0 (0: lockstep, for A/B)
#define TKG8_STAGGER 1
#endif
#ifndef TKG8_PRIO  // staggered schedule: s_setprio 1 around the MFMA clusters
#define TKG8_PRIO 1
#endif
#ifndef TKG_GROUP_M  // tile-rows per L2 group in the XCD-aware block map
#define TKG_GROUP_M 8
#endif
constexpr int BM = 256, BN = 256, BK = TKG_BK;                            // K-step 64 (default) or 32
constexpr int WAVES_M = 2, WAVES_N = 4, THREADS = 64 * WAVES_M * WAVES_N;  // 512
constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;                       // 128 x 64 per wave
constexpr int FM = WM / 16, FN = WN / 16;                                 // 8 x 4 fragments
constexpr int KSUB = BK / 32;                                             // MFMA K-steps per stage
constexpr int TILE_BYTES = BM * BK * 2;                                   // per operand tile
constexpr int STAGE_BYTES = 2 * TILE_BYTES;                               // A + B
constexpr int NSTAGE = (128 * 1024) / STAGE_BYTES;                        // 128 KiB: 4 stages (BK 32) / 2 (BK 64)
constexpr int LDS_BYTES = NSTAGE * STAGE_BYTES;
constexpr int GLDS_PER_TILE = TILE_BYTES / (THREADS * 16);                // copies per thread per operand
constexpr int CHUNKS = BK / 8;                                            // 16-byte chunks per row
constexpr int ROWS_PER_BANKROW = 256 / (BK * 2);                          // rows sharing one 256-B bank row
constexpr int ROWS_PER_COPY = THREADS / CHUNKS;                           // rows one copy instruction covers

// physical 16-byte chunk of logical chunk `c` in row `r`: the 16 lanes of a ds_read_b128
// group (16 consecutive rows, one chunk) land in 16 distinct 16-byte bank slots
__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r / ROWS_PER_BANKROW) & (CHUNKS - 1)); }

// Stage one [256][BK] bf16 tile (k0..k0+BK-1 of a 256-row panel of a K-contiguous matrix)
// into LDS at `lds`.  Buffer loads straight to LDS: the panel is one SRSRC descriptor
// (wave-uniform), every lane keeps ONE 32-bit byte offset `voff` for all its copies (the
// per-copy row step and k0 go in the scalar offset), and the LDS destination is the
// wave-uniform base + lane*16.  The swizzle lives in `voff` (see panel_voffset).
__device__ __forceinline__ void stage_tile(__amdgpu_buffer_rsrc_t panel, int ld, int voff, int k0, char* lds,
                                           int tid) {
#pragma unroll
  for (int i = 0; i < GLDS_PER_TILE; ++i) {
    char* dst = lds + (size_t)(i * THREADS + (tid & ~63)) * 16;
    const int soff = (i * ROWS_PER_COPY * ld + k0) * 2;  // copy i covers the next ROWS_PER_COPY rows
    __builtin_amdgcn_raw_ptr_buffer_load_lds(panel, reinterpret_cast<__shared__ void*>(dst), 16, voff, soff, 0, 0);
  }
}

// Byte offset of this thread's 16-byte chunk: slot tid of the lane-linear LDS image is row
// r = tid / CHUNKS (+ ROWS_PER_COPY per copy), physical chunk tid % CHUNKS, which holds
// logical chunk swz(r, tid % CHUNKS) — the same for every copy (the row step is a multiple
// of the swizzle period).
__device__ __forceinline__ int panel_voffset(int ld, int tid) {
  const int r = tid / CHUNKS, c = swz(r, tid % CHUNKS);
  return (r * ld + c * 8) * 2;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_panel(const __bf16* base, int row0, int ld) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(base + (size_t)row0 * ld), 0, BM * ld * 2, 0x00020000);
}

__device__ __forceinline__ bf16x8 lds_frag(const char* img, int r, int c) {
  return *reinterpret_cast<const bf16x8*>(img + r * (BK * 2) + swz(r, c) * 16);
}

// s_waitcnt vmcnt(n * copies per stage) for a runtime n in [0, NSTAGE): the count must be
// an immediate
__device__ __forceinline__ void wait_copies_but(int n) {
  static_assert(2 * GLDS_PER_TILE == 4 || 2 * GLDS_PER_TILE == 8, "copies per stage");
  if (n <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if TKG_BK == 32
  else if (n == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
#else
  else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
#endif
}

// XCD-aware, bijective block -> tile map: blocks b, b+8, b+16.. run on one XCD; give each
// XCD a contiguous range of tiles, walked in groups of GROUP_M tile-rows so neighbouring
// blocks on an XCD share A rows and B columns in that XCD's L2.
__device__ __forceinline__ void tile_of(int b, int nwg, int tiles_m, int tiles_n, int* tm, int* tn) {
  const int xcd = b & 7, q = nwg >> 3, rem = nwg & 7;
  const int w = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  constexpr int GROUP_M = TKG_GROUP_M;
  const int per_group = GROUP_M * tiles_n;
  const int g = w / per_group, first_m = g * GROUP_M;
  const int rows = min(tiles_m - first_m, GROUP_M);
  const int in = w - g * per_group;
  *tm = first_m + in % rows;
  *tn = in / rows;
}
}  // namespace

// mode 0: write C (fp32, row-major [M][N]); mode 1: screen — per-wave checksums only:
// colpart[(tm*WAVES_M + wr)][n] = sum over the wave's 128 rows, rowpart[(tn*WAVES_N + wc)][m]
// = sum over the wave's 64 columns.  inject >= 0 adds 1024.0 to the element C[inject/N][inject%N]
// before the reduction (fault-injection self-test of the screen).
template <int MODE>
__global__ __launch_bounds__(THREADS) void k_gemm_bt(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                     float* __restrict__ C, float* __restrict__ colpart,
                                                     float* __restrict__ rowpart, int M, int N, int K,
                                                     long long inject) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WAVES_N, wc = wid % WAVES_N;
  const int tiles_m = M / BM, tiles_n = N / BN;
  int tm, tn;
  tile_of(blockIdx.x, gridDim.x, tiles_m, tiles_n, &tm, &tn);
  const int row0 = tm * BM, col0 = tn * BN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  const __amdgpu_buffer_rsrc_t pa = make_panel(A, row0, K), pb = make_panel(B, col0, K);
  const int voff = panel_voffset(K, tid);
  auto stage = [&](int t) {  // K-step t into buffer t % NSTAGE
    char* dst = smem + (t % NSTAGE) * STAGE_BYTES;
    stage_tile(pa, K, voff, t * BK, dst, tid);
    stage_tile(pb, K, voff, t * BK, dst + TILE_BYTES, tid);
  };
  // prologue: the first NSTAGE steps in flight; wait for step 0 only
  for (int t = 0; t < NSTAGE && t < nk; ++t) stage(t);
  wait_copies_but(min(nk, NSTAGE) - 1);
  __builtin_amdgcn_s_barrier();

  const int fr = lane & 15, fq = lane >> 4;  // fragment row/col within 16, k-chunk group
  bf16x8 bf[KSUB][FN], af[KSUB][FM];
  auto read_frags = [&](int t) {
    const char* a_img = smem + (t % NSTAGE) * STAGE_BYTES;
    const char* b_img = a_img + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < KSUB; ++kk) {
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[kk][j] = lds_frag(b_img, wc * WN + j * 16 + fr, kk * 4 + fq);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[kk][i] = lds_frag(a_img, wr * WM + i * 16 + fr, kk * 4 + fq);
    }
  };
  auto mfmas = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < KSUB; ++kk)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bf[kk][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // Every fragment of step t is read into VGPRs before its MFMAs, so buffer t % NSTAGE is
  // free once the barrier after those reads has passed: step t + NSTAGE is copied into it
  // right there, and the MFMAs run while the NSTAGE - 1 later steps are in flight.  Before
  // the barrier each thread waits for its copy of step t+1 only (later ones keep flying),
  // so the barrier also publishes step t+1 to every wave.
  // (A variant with two wave groups staggered by one barrier slot measured the same at
  // BK 64: 1162 / 1224 vs 1155 / 1238 TF at 4096^3 / 8192^3 — profiles/round1/round1_gemm_pmc.md.)
  for (int t = 0; t < nk; ++t) {
    read_frags(t);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wait_copies_but(min(nk - 1, t + NSTAGE - 1) - (t + 1));
    __builtin_amdgcn_s_barrier();
    if (t + NSTAGE < nk) stage(t + NSTAGE);
    mfmas();
  }

  // accumulator element (i, j, e): row = wr*WM + i*16 + fq*4 + e, col = wc*WN + j*16 + fr
  if constexpr (MODE == 0) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = row0 + wr * WM + i * 16 + fq * 4 + e, c = col0 + wc * WN + j * 16 + fr;
          C[(size_t)r * N + c] = acc[i][j][e];
        }
  } else {
    if (inject >= 0) {
      const long long ir = inject / N, ic = inject % N;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (row0 + wr * WM + i * 16 + fq * 4 + e == ir && col0 + wc * WN + j * 16 + fr == ic) acc[i][j][e] += 1024.f;
    }
    // column sums over the wave's 128 rows: per lane over (i, e), then across the 4 lanes
    // sharing a column (fq = 0..3 -> lanes fr, fr+16, fr+32, fr+48)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (fq == 0) colpart[(size_t)(tm * WAVES_M + wr) * N + col0 + wc * WN + j * 16 + fr] = s;
    }
    // row sums over the wave's 64 columns: per lane over j, then across the 16 lanes of a row group
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < FN; ++j) s += acc[i][j][e];
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        if (fr == 0) rowpart[(size_t)(tn * WAVES_N + wc) * M + row0 + wr * WM + i * 16 + fq * 4 + e] = s;
      }
    }
  }
}

// --- staggered schedule (k_gemm8: bf16 and fp8) ------------------------------------------
// Same 256x256 output tile, 8 waves and 128 KiB of LDS as k_gemm_bt; a K-tile is 128 bytes
// of every row (64 bf16 or 128 fp8 e4m3), so one code path serves both element types.
// The LDS holds half-tiles: slot (t & 1, h) for h = A0 | A1 | B0 | B1 = rows 0-127 /
// 128-255 of the A or B panel of K-tile t, [128][128 B] each (16 KiB, same XOR swizzle).
// Wave (wr, wc) owns four 64x32 quadrants (mh, nh): rows mh*128 + wr*64 .. +63, columns
// nh*128 + wc*32 .. +31, so quadrant (mh, nh) reads only half-tiles A{mh} and B{nh}.  A
// K-tile is two phases of 32 MFMAs (bf16: 16x16x32 x2 per fragment pair; fp8: one
// block-scaled 16x16x128 at twice the cycles and four times the K):
//   Pa(t): read A0, B0, B1 -> quadrants (0,0), (0,1); refill B1, A1 of t+1
//   Pb(t): read A1         -> quadrants (1,1), (1,0); refill A0, B0 of t+2
// each  [ds_reads][copies][s_waitcnt vmcnt(..) lgkmcnt(..)] s_barrier [32 MFMAs] s_barrier.
// Group wr = 1 runs one barrier behind group wr = 0 (an extra s_barrier at the start, the
// other group's at the end), so on every SIMD — which holds one wave of each group — one
// wave issues MFMAs while the other reads LDS and issues copies.
// WAR: A0/B0(t) are refilled one phase after their reads, so Pa retires those 12 reads
// (lgkmcnt(4): the 4 B1 reads, issued last, may stay in flight) before its first barrier;
// with the stagger that orders them before the other group's refill.  B1(t) is refilled two
// phases on; A1(t) one phase on (Pb retires all its reads).
// RAW: a half-tile is waited for before the first barrier of the phase BEFORE the one that
// reads it (one barrier of margin for the stagger): Pa(t) retires A1(t) (4 younger stages
// = 8 copies may stay in flight), Pb(t) retires A0/B0/B1 of t+1 (3 younger: vmcnt(6)); the
// last K-tiles wait with vmcnt(0), where fewer younger copies exist.
// (Variants measured on the way — four phases of 16 MFMAs, other wait placements, B1 refilled
// early, no stagger — and their counters: profiles/round1/round1_gemm_pmc.md.)
namespace p8 {
constexpr int KT_BYTES = 128, HROWS = 128;       // bytes of a row per K-tile; rows per half-tile
constexpr int HBYTES = HROWS * KT_BYTES;         // 16 KiB
constexpr int HCOPIES = HBYTES / (THREADS * 16);  // 2 copies per thread per half-tile
constexpr int LDS = 8 * HBYTES;                  // 128 KiB
constexpr int ROWS_PER_COPY8 = THREADS / 8;       // 64
static_assert(HCOPIES == 2, "copies per half-tile");

__device__ __forceinline__ int swz8(int r, int c) { return c ^ ((r >> 1) & 7); }
__device__ __forceinline__ u32x4 chunk(const char* img, int r, int c) {
  return *reinterpret_cast<const u32x4*>(img + r * KT_BYTES + swz8(r, c) * 16);
}
__device__ __forceinline__ char* slot(char* smem, int t, int h) { return smem + ((t & 1) * 4 + h) * HBYTES; }
// this thread's byte offset in a panel of rows `ldb` bytes long (see panel_voffset)
__device__ __forceinline__ int voffset(int ldb, int tid) {
  const int r = tid >> 3, c = swz8(r, tid & 7);
  return r * ldb + c * 16;
}
__device__ __forceinline__ void stage_half(__amdgpu_buffer_rsrc_t panel, int ldb, int voff, int row_off, int kb0,
                                           char* dst, int tid) {
#pragma unroll
  for (int i = 0; i < HCOPIES; ++i) {
    char* d = dst + (size_t)(i * THREADS + (tid & ~63)) * 16;
    const int soff = (row_off + i * ROWS_PER_COPY8) * ldb + kb0;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(panel, reinterpret_cast<__shared__ void*>(d), 16, voff, soff, 0, 0);
  }
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t panel(const void* base, int row0, int ldb) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(static_cast<const char*>(base) + (size_t)row0 * ldb), 0,
                                           BM * ldb, 0x00020000);
}
__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}
}  // namespace p8

// ESIZE 2: bf16, ESIZE 1: fp8 e4m3 (OCP).  K counts elements.
template <int MODE, int ESIZE>
__global__ __launch_bounds__(THREADS) void k_gemm8(const void* __restrict__ A, const void* __restrict__ B,
                                                   float* __restrict__ C, float* __restrict__ colpart,
                                                   float* __restrict__ rowpart, int M, int N, int K,
                                                   long long inject) {
  using namespace p8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int tiles_m = M / BM, tiles_n = N / BN;
  int tm, tn;
  tile_of(blockIdx.x, gridDim.x, tiles_m, tiles_n, &tm, &tn);
  const int row0 = tm * BM, col0 = tn * BN;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mh][nh][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ldb = K * ESIZE, nk = ldb / KT_BYTES;
  const __amdgpu_buffer_rsrc_t pa = panel(A, row0, ldb), pb = panel(B, col0, ldb);
  const int voff = voffset(ldb, tid);
  auto stage = [&](int t, int h) {  // h: 0 A0, 1 A1, 2 B0, 3 B1
    stage_half(h < 2 ? pa : pb, ldb, voff, (h & 1) * HROWS, t * KT_BYTES, slot(smem, t, h), tid);
  };
  // A fragment of one 16-row group for the whole K-tile: 16-byte chunks fq and 4 + fq of
  // the row (bf16: one per 16x16x32 k-step, lane holds k = 8 fq .. +7 of each; fp8: both
  // feed one 16x16x128 step).  A and B use the same map, so every product pairs equal k —
  // for fp8 the MFMA's k positions are a permutation of the row's bytes, which leaves the
  // dot product unchanged.  The natural fp8 map (chunks 2 fq, 2 fq + 1) would put the two
  // lane quarters of a ds_read_b128 group on the same banks: 50 M conflict cycles per
  // 8192^3 (profiles/round1/round1_gemm_pmc.md); this one is conflict-free, as for bf16.
  u32x4 a[4][2], b[2][2][2];
  auto ld_frag = [&](const char* img, int r, u32x4* f) {
    f[0] = chunk(img, r, fq);
    f[1] = chunk(img, r, 4 + fq);
  };
  auto read_a = [&](int t, int mh) {
    const char* img = slot(smem, t, mh);
#pragma unroll
    for (int i = 0; i < 4; ++i) ld_frag(img, wr * 64 + i * 16 + fr, a[i]);
  };
  auto read_b = [&](int t, int nh) {
    const char* img = slot(smem, t, 2 + nh);
#pragma unroll
    for (int j = 0; j < 2; ++j) ld_frag(img, wc * 32 + j * 16 + fr, b[nh][j]);
  };
  auto quad = [&](int mh, int nh) {
    if (TKG8_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (ESIZE == 2) {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            acc[mh][nh][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, a[i][kk]), __builtin_bit_cast(bf16x8, b[nh][j][kk]), acc[mh][nh][i][j], 0,
                0, 0);
        } else {
          const i32x8 av = __builtin_shufflevector(__builtin_bit_cast(i32x4, a[i][0]), __builtin_bit_cast(i32x4, a[i][1]),
                                                   0, 1, 2, 3, 4, 5, 6, 7);
          const i32x8 bv = __builtin_shufflevector(__builtin_bit_cast(i32x4, b[nh][j][0]),
                                                   __builtin_bit_cast(i32x4, b[nh][j][1]), 0, 1, 2, 3, 4, 5, 6, 7);
          // FMT 0 = fp8 e4m3 for A and B; E8M0 scales 127 = 2^0
          acc[mh][nh][i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc[mh][nh][i][j], 0, 0, 0,
                                                                               127, 0, 127);
        }
      }
    if (TKG8_PRIO) __builtin_amdgcn_s_setprio(0);
  };

  // prologue: K-tile 0 whole plus A0/B0 of K-tile 1; wait for A0, B0, B1 of K-tile 0
  stage(0, 0);
  stage(0, 2);
  stage(0, 3);
  stage(0, 1);
  if (nk > 1) {
    stage(1, 0);
    stage(1, 2);
  }
  if (nk > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  barrier();
  if (TKG8_STAGGER && wr == 1) barrier();  // the stagger

  // The MFMAs are pure register ops: without pins the compiler may move them across the
  // s_barriers (it sank Pb's MFMAs into the next iteration of the fp8 loop).  An empty
  // volatile asm that "rewrites" the fragments right after a phase's first barrier, and one
  // that "reads" the accumulators before its second, keeps every MFMA in its slot.
  auto pin_frags = [&](bool with_b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(a[i][0]), "+v"(a[i][1]));
    if (with_b) {
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(b[nh][j][0]), "+v"(b[nh][j][1]));
    }
  };
  auto pin_acc = [&](int mh) {
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[mh][nh][i][j]));
  };
  for (int t = 0; t < nk; ++t) {
    const bool more1 = t + 1 < nk, more2 = t + 2 < nk;
    read_a(t, 0);
    read_b(t, 0);
    __builtin_amdgcn_sched_barrier(0);  // the B1 reads last: lgkmcnt(4) below leaves only them
    read_b(t, 1);
    if (more1) {
      stage(t + 1, 3);
      stage(t + 1, 1);
      asm volatile("s_waitcnt vmcnt(8) lgkmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(4)" ::: "memory");
    }
    barrier();
    pin_frags(true);
    quad(0, 0);
    quad(0, 1);
    pin_acc(0);
    barrier();
    read_a(t, 1);
    if (more2) {
      stage(t + 2, 0);
      stage(t + 2, 2);
      asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    barrier();
    pin_frags(false);
    quad(1, 1);
    quad(1, 0);
    pin_acc(1);
    barrier();
  }
  if (TKG8_STAGGER && wr == 0) barrier();  // match the stagger's extra barrier

  // accumulator element (mh, nh, i, j, e): row = mh*128 + wr*64 + i*16 + fq*4 + e,
  //                                         col = nh*128 + wc*32 + j*16 + fr
  if constexpr (MODE == 2) {
    // bf16 C (the vendor GEMM's output type) through a wave-private 16 KiB LDS image, so
    // the global stores are 16 bytes per lane (a store tail of 4-byte stores is issue-bound).
    // A lane holds rows fq*4 + e of column fr; it swaps two values with its neighbour fr ^ 1
    // (DPP quad_perm [1,0,3,2]) so each lane has two bf16 pairs: even lanes rows e = 0, 1 at
    // columns fr, fr + 1, odd lanes rows e = 2, 3 at fr - 1, fr.  The image is 4 blocks (mh,
    // nh) of [64 rows][64 B]; dword column bit 3 is XORed with row bit 1, which leaves the
    // ds_write_b32s 2-way (free) and the ds_read_b128s conflict-free.
    barrier();  // every wave is past its last fragment read of the main loop
    char* img = smem + wid * (4 * 64 * 64);
    const int odd = fr & 1;
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const f32x4 v = acc[mh][nh][i][j];
            const float s0 = odd ? v[0] : v[2], s1 = odd ? v[1] : v[3];
            const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s0),
                                                                                   0xB1, 0xF, 0xF, false));
            const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s1),
                                                                                   0xB1, 0xF, 0xF, false));
            typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
            const bf16x2 p0 = {(__bf16)(odd ? r0 : v[0]), (__bf16)(odd ? v[2] : r0)};
            const bf16x2 p1 = {(__bf16)(odd ? r1 : v[1]), (__bf16)(odd ? v[3] : r1)};
            const int row = i * 16 + fq * 4 + odd * 2, cdw = j * 8 + (fr >> 1);
            uint32_t* blk = reinterpret_cast<uint32_t*>(img + (mh * 2 + nh) * 4096);
            blk[row * 16 + (cdw ^ (((row >> 1) & 1) << 3))] = __builtin_bit_cast(uint32_t, p0);
            blk[(row + 1) * 16 + (cdw ^ ((((row + 1) >> 1) & 1) << 3))] = __builtin_bit_cast(uint32_t, p1);
          }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    char* cb = reinterpret_cast<char*>(C);
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = q * 16 + (lane >> 2), c = lane & 3;
          const u32x4 d =
              *reinterpret_cast<const u32x4*>(img + (mh * 2 + nh) * 4096 + r * 64 + ((c ^ (((r >> 1) & 1) << 1)) * 16));
          const size_t grow = (size_t)row0 + mh * 128 + wr * 64 + r;
          const int gcol = col0 + nh * 128 + wc * 32 + c * 8;
          *reinterpret_cast<u32x4*>(cb + (grow * N + gcol) * 2) = d;
        }
  } else if constexpr (MODE == 0) {
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = row0 + mh * 128 + wr * 64 + i * 16 + fq * 4 + e;
              const int c = col0 + nh * 128 + wc * 32 + j * 16 + fr;
              C[(size_t)r * N + c] = acc[mh][nh][i][j][e];
            }
  } else {
    if (inject >= 0) {
      const long long ir = inject / N, ic = inject % N;
#pragma unroll
      for (int mh = 0; mh < 2; ++mh)
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (row0 + mh * 128 + wr * 64 + i * 16 + fq * 4 + e == ir &&
                    col0 + nh * 128 + wc * 32 + j * 16 + fr == ic)
                  acc[mh][nh][i][j][e] += 1024.f;
    }
    // column sums over the wave's 128 rows (both row halves)
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float s = 0.f;
#pragma unroll
        for (int mh = 0; mh < 2; ++mh)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            s += acc[mh][nh][i][j][0] + acc[mh][nh][i][j][1] + acc[mh][nh][i][j][2] + acc[mh][nh][i][j][3];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        if (fq == 0) colpart[(size_t)(tm * WAVES_M + wr) * N + col0 + nh * 128 + wc * 32 + j * 16 + fr] = s;
      }
    // row sums over the wave's 64 columns (both column halves)
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float s = 0.f;
#pragma unroll
          for (int nh = 0; nh < 2; ++nh)
#pragma unroll
            for (int j = 0; j < 2; ++j) s += acc[mh][nh][i][j][e];
          s += __shfl_xor(s, 1, 64);
          s += __shfl_xor(s, 2, 64);
          s += __shfl_xor(s, 4, 64);
          s += __shfl_xor(s, 8, 64);
          if (fr == 0)
            rowpart[(size_t)(tn * WAVES_N + wc) * M + row0 + mh * 128 + wr * 64 + i * 16 + fq * 4 + e] = s;
        }
  }
}

// --- checksum right-hand sides and comparison (fp32 SIMT, independent of the MFMA path) ----
// out[k] += sum over this block's chunk of rows of X[r][k] (X is [rows][K] bf16); grid.y
// splits the rows, partial sums meet in fp32 atomics (out / out_abs zeroed beforehand)
constexpr int COLSUM_CHUNKS = 64;

// OCP fp8 e4m3 (e4m3fn: bias 7, no infinities, S.1111.111 = NaN) -> float
__device__ __forceinline__ float e4m3_to_f(uint8_t v) {
  const int e = (v >> 3) & 15, m = v & 7;
  float x = e ? ldexpf(1.0f + m * 0.125f, e - 7) : ldexpf(m * 0.125f, -6);
  if (e == 15 && m == 7) x = __builtin_nanf("");
  return (v & 0x80) ? -x : x;
}
__device__ __forceinline__ float elem(const __bf16* p, size_t i) { return (float)p[i]; }
__device__ __forceinline__ float elem(const uint8_t* p, size_t i) { return e4m3_to_f(p[i]); }

template <typename T>
__global__ __launch_bounds__(256) void k_colsum(const T* __restrict__ X, int rows, int K, float* __restrict__ out,
                                                float* __restrict__ out_abs) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  const int per = (rows + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
  float s = 0.f, a = 0.f;
  for (int r = r0; r < r1; ++r) {
    const float v = elem(X, (size_t)r * K + k);
    s += v;
    a += fabsf(v);
  }
  atomicAdd(out + k, s);
  atomicAdd(out_abs + k, a);
}

// expected[r] = sum_k X[r][k] * v[k]; bound[r] = sum_k |X[r][k]| * vabs[k]  (one wave per row)
template <typename T>
__global__ __launch_bounds__(256) void k_rowdot(const T* __restrict__ X, int rows, int K, const float* __restrict__ v,
                                                const float* __restrict__ vabs, float* __restrict__ expected,
                                                float* __restrict__ bound) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  float s = 0.f, b = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float x = elem(X, (size_t)r * K + k);
    s += x * v[k];
    b += fabsf(x) * vabs[k];
  }
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_down(s, off, 64);
    b += __shfl_down(b, off, 64);
  }
  if (lane == 0) {
    expected[r] = s;
    bound[r] = b;
  }
}

// actual[x] = sum over `parts` partial rows; count |actual - expected| > rtol * bound + atol,
// record the worst index and the largest normalised error
__global__ __launch_bounds__(256) void k_compare(const float* __restrict__ part, int parts, int n,
                                                 const float* __restrict__ expected, const float* __restrict__ bound,
                                                 float rtol, float atol, unsigned int* __restrict__ bad,
                                                 unsigned int* __restrict__ first_bad, float* __restrict__ max_err) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= n) return;
  float s = 0.f;
  for (int p = 0; p < parts; ++p) s += part[(size_t)p * n + x];
  const float tol = rtol * bound[x] + atol;
  const float err = fabsf(s - expected[x]);
  if (!(err <= tol)) {  // NaN counts as bad
    atomicAdd(bad, 1u);
    atomicMin(first_bad, (unsigned int)x);
  }
  const float norm = err / tol;
  // float max via int ordering (non-negative values)
  atomicMax(reinterpret_cast<unsigned int*>(max_err), __float_as_uint(isnan(norm) ? 3.0e38f : norm));
}

// deterministic pseudo-random bf16 in [-1, 1)
__global__ __launch_bounds__(256) void k_fill_bf16(__bf16* __restrict__ p, size_t n, uint32_t seed) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint32_t x = (uint32_t)i * 0x9e3779b9u ^ seed ^ (uint32_t)(i >> 32);
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    p[i] = (__bf16)(((x >> 8) * (1.0f / 8388608.0f)) - 1.0f);
  }
}

// deterministic pseudo-random finite fp8 e4m3 with |v| in [2^-4, 2): random sign, exponent
// field 3..7, random mantissa (so products and sums stay well inside fp32)
__global__ __launch_bounds__(256) void k_fill_fp8(uint8_t* __restrict__ p, size_t n, uint32_t seed) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint32_t x = (uint32_t)i * 0x9e3779b9u ^ seed ^ (uint32_t)(i >> 32);
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    p[i] = (uint8_t)(((x >> 31) << 7) | ((3 + (x >> 8) % 5) << 3) | (x & 7));
  }
}

// elements per K-tile: 64 bf16 / 128 fp8 (schedule 1); BK for the single-barrier loop
static int k_granule(int esize) { return esize == 1 ? 128 : BK; }

static int check_shape(int M, int N, int K, int esize = 2) {
  const int kg = k_granule(esize);
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % kg) {
    snprintf(g_err, sizeof(g_err), "shape %dx%dx%d: M and N must be multiples of %d, K of %d", M, N, K, BM, kg);
    return -1;
  }
  return 0;
}

// schedule: 0 = one barrier per K-step (k_gemm_bt), 1 = 8-phase staggered (k_gemm8, BK 64);
// env TKG_SCHED or tkg_set_schedule() selects it (A/B in one process: scripts/gemm_ab.py)
static int g_sched = -1;

static int schedule() {
  if (g_sched < 0) {
    const char* e = getenv("TKG_SCHED");  // "0" or "1"; anything else (atoi's 0) keeps the default
    g_sched = e && (!strcmp(e, "0") || !strcmp(e, "1")) ? e[0] - '0' : TKG_DEFAULT_SCHED;
  }
  return (g_sched == 1 && BK * 2 == p8::KT_BYTES) ? 1 : 0;
}

extern "C" int tkg_set_schedule(int s) {
  g_sched = s;
  return schedule();
}

// mode 0: fp32 C, 1: screen (checksums only), 2: bf16 C (staggered schedule only)
static hipError_t launch_gemm(int mode, int esize, const void* A, const void* B, float* C, float* colpart,
                              float* rowpart, int M, int N, int K, long long inject, hipStream_t s) {
  const int grid = (M / BM) * (N / BN);
  if (esize == 1) {  // fp8: staggered schedule only
    if (mode == 0) k_gemm8<0, 1><<<grid, THREADS, p8::LDS, s>>>(A, B, C, colpart, rowpart, M, N, K, inject);
    else if (mode == 2) k_gemm8<2, 1><<<grid, THREADS, p8::LDS, s>>>(A, B, C, colpart, rowpart, M, N, K, inject);
    else k_gemm8<1, 1><<<grid, THREADS, p8::LDS, s>>>(A, B, C, colpart, rowpart, M, N, K, inject);
  } else if (schedule() == 1) {
    if (mode == 0) k_gemm8<0, 2><<<grid, THREADS, p8::LDS, s>>>(A, B, C, colpart, rowpart, M, N, K, inject);
    else if (mode == 2) k_gemm8<2, 2><<<grid, THREADS, p8::LDS, s>>>(A, B, C, colpart, rowpart, M, N, K, inject);
    else k_gemm8<1, 2><<<grid, THREADS, p8::LDS, s>>>(A, B, C, colpart, rowpart, M, N, K, inject);
  } else {
    if (mode == 2) return hipErrorInvalidValue;  // the single-barrier loop (A/B only) writes fp32
    const __bf16 *a = static_cast<const __bf16*>(A), *b = static_cast<const __bf16*>(B);
    if (mode == 0) k_gemm_bt<0><<<grid, THREADS, LDS_BYTES, s>>>(a, b, C, colpart, rowpart, M, N, K, inject);
    else k_gemm_bt<1><<<grid, THREADS, LDS_BYTES, s>>>(a, b, C, colpart, rowpart, M, N, K, inject);
  }
  return hipGetLastError();
}

static hipError_t set_lds_limit() {
  static hipError_t once = [] {
    const void* fns[] = {reinterpret_cast<const void*>(&k_gemm_bt<0>), reinterpret_cast<const void*>(&k_gemm_bt<1>),
                         reinterpret_cast<const void*>(&k_gemm8<0, 2>), reinterpret_cast<const void*>(&k_gemm8<1, 2>),
                         reinterpret_cast<const void*>(&k_gemm8<0, 1>), reinterpret_cast<const void*>(&k_gemm8<1, 1>),
                         reinterpret_cast<const void*>(&k_gemm8<2, 2>), reinterpret_cast<const void*>(&k_gemm8<2, 1>)};
    for (const void* f : fns) {
      hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }();
  return once;
}

// Stream-ordered C = A * B^T, no host synchronisation (torch tensors on torch's stream: one
// HIP runtime, see ops/native.py:require_torch_first).  esize 2: bf16 operands, 1: fp8
// e4m3; out_bf16: C is bf16 (the vendor GEMM's output type), else fp32.  C must be 16-byte
// aligned for bf16 output.  Returns 0, or -1 / a HIP error with tkg_last_error() set.
extern "C" int tkg_gemm(int dev, int esize, const void* A, const void* B, void* C, int M, int N, int K, int out_bf16,
                        void* stream) {
  if (esize != 1 && esize != 2) {
    snprintf(g_err, sizeof(g_err), "element size %d (1: fp8 e4m3, 2: bf16)", esize);
    return -1;
  }
  if (check_shape(M, N, K, esize)) return -1;
  if (out_bf16 && (reinterpret_cast<uintptr_t>(C) & 15)) {
    snprintf(g_err, sizeof(g_err), "bf16 C must be 16-byte aligned");
    return -1;
  }
  if (out_bf16 && esize == 2 && schedule() != 1) {
    snprintf(g_err, sizeof(g_err), "bf16 output needs the staggered schedule");
    return -1;
  }
  int prev = 0;
  CHECK(hipGetDevice(&prev));
  CHECK(hipSetDevice(dev));
  CHECK(set_lds_limit());
  const hipError_t e = launch_gemm(out_bf16 ? 2 : 0, esize, A, B, static_cast<float*>(C), nullptr, nullptr, M, N, K,
                                   -1, static_cast<hipStream_t>(stream));
  CHECK(hipSetDevice(prev));
  CHECK(e);
  return 0;
}

// The screen: random A[M][K], B[N][K]; `reps` timed checksum-mode GEMMs (best time), then the
// ABFT comparison of the last one.  inject >= 0 corrupts C[inject/N][inject%N] (self-test).
// out[0] TFLOP/s (best rep), out[1] ms of that rep, out[2] bad columns, out[3] bad rows,
// out[4] first bad column (-1: none), out[5] first bad row, out[6] max normalised error
// (err / tolerance over every checksum; < 1 passes).
static int screen(int dev, int esize, int M, int N, int K, int reps, long long inject, double* out) {
  if (check_shape(M, N, K, esize)) return -1;
  CHECK(hipSetDevice(dev));
  CHECK(set_lds_limit());
  void *A = nullptr, *B = nullptr;
  float *colpart = nullptr, *rowpart = nullptr, *work = nullptr;
  unsigned int* flags = nullptr;
  const size_t parts_c = (size_t)(M / BM) * WAVES_M, parts_r = (size_t)(N / BN) * WAVES_N;
  CHECK(hipMalloc(&A, (size_t)M * K * esize));
  CHECK(hipMalloc(&B, (size_t)N * K * esize));
  CHECK(hipMalloc(&colpart, parts_c * N * 4));
  CHECK(hipMalloc(&rowpart, parts_r * M * 4));
  // sA, |sA|, sB, |sB| (K each), colexp/colbound (N), rowexp/rowbound (M)
  CHECK(hipMalloc(&work, ((size_t)4 * K + 2 * N + 2 * M) * 4));
  CHECK(hipMalloc(&flags, 6 * 4));
  float *sA = work, *sAabs = sA + K, *sB = sAabs + K, *sBabs = sB + K, *colexp = sBabs + K, *colbd = colexp + N,
        *rowexp = colbd + N, *rowbd = rowexp + M;
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  if (esize == 1) {
    k_fill_fp8<<<2048, 256, 0, s>>>(static_cast<uint8_t*>(A), (size_t)M * K, 0x51f15eedu);
    k_fill_fp8<<<2048, 256, 0, s>>>(static_cast<uint8_t*>(B), (size_t)N * K, 0x0b5e55edu);
  } else {
    k_fill_bf16<<<2048, 256, 0, s>>>(static_cast<__bf16*>(A), (size_t)M * K, 0x51f15eedu);
    k_fill_bf16<<<2048, 256, 0, s>>>(static_cast<__bf16*>(B), (size_t)N * K, 0x0b5e55edu);
  }
  CHECK(hipGetLastError());
  CHECK(launch_gemm(1, esize, A, B, nullptr, colpart, rowpart, M, N, K, -1, s));  // warm-up
  double best = 1e30;
  for (int r = 0; r < (reps < 1 ? 1 : reps); ++r) {
    CHECK(hipEventRecord(e0, s));
    CHECK(launch_gemm(1, esize, A, B, nullptr, colpart, rowpart, M, N, K, inject, s));
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, (double)ms);
  }
  // right-hand sides: column sums of A and B over M / N, then the two mat-vecs
  CHECK(hipMemsetAsync(sA, 0, (size_t)4 * K * sizeof(float), s));  // sA, |sA|, sB, |sB|
  if (esize == 1) {
    const uint8_t *a = static_cast<const uint8_t*>(A), *b = static_cast<const uint8_t*>(B);
    k_colsum<<<dim3((K + 255) / 256, COLSUM_CHUNKS), 256, 0, s>>>(a, M, K, sA, sAabs);
    k_colsum<<<dim3((K + 255) / 256, COLSUM_CHUNKS), 256, 0, s>>>(b, N, K, sB, sBabs);
    k_rowdot<<<(N + 3) / 4, 256, 0, s>>>(b, N, K, sA, sAabs, colexp, colbd);
    k_rowdot<<<(M + 3) / 4, 256, 0, s>>>(a, M, K, sB, sBabs, rowexp, rowbd);
  } else {
    const __bf16 *a = static_cast<const __bf16*>(A), *b = static_cast<const __bf16*>(B);
    k_colsum<<<dim3((K + 255) / 256, COLSUM_CHUNKS), 256, 0, s>>>(a, M, K, sA, sAabs);
    k_colsum<<<dim3((K + 255) / 256, COLSUM_CHUNKS), 256, 0, s>>>(b, N, K, sB, sBabs);
    k_rowdot<<<(N + 3) / 4, 256, 0, s>>>(b, N, K, sA, sAabs, colexp, colbd);
    k_rowdot<<<(M + 3) / 4, 256, 0, s>>>(a, M, K, sB, sBabs, rowexp, rowbd);
  }
  const unsigned int init[6] = {0u, 0xffffffffu, 0u, 0u, 0xffffffffu, 0u};
  CHECK(hipMemcpyAsync(flags, init, sizeof(init), hipMemcpyHostToDevice, s));
  // fp32 reassociation error of two different summation orders over K*M (or K*N) products
  const float rtol = 1e-6f, atol = 1e-3f;  // healthy runs measure ~1e-3 of this tolerance
  k_compare<<<(N + 255) / 256, 256, 0, s>>>(colpart, (int)parts_c, N, colexp, colbd, rtol, atol, flags, flags + 1,
                                            reinterpret_cast<float*>(flags + 2));
  k_compare<<<(M + 255) / 256, 256, 0, s>>>(rowpart, (int)parts_r, M, rowexp, rowbd, rtol, atol, flags + 3, flags + 4,
                                            reinterpret_cast<float*>(flags + 5));
  CHECK(hipGetLastError());
  unsigned int h[6];
  CHECK(hipMemcpyAsync(h, flags, sizeof(h), hipMemcpyDeviceToHost, s));
  CHECK(hipStreamSynchronize(s));
  float maxc, maxr;
  memcpy(&maxc, &h[2], 4);
  memcpy(&maxr, &h[5], 4);
  out[0] = 2.0 * M * N * (double)K / (best * 1e-3) / 1e12;
  out[1] = best;
  out[2] = h[0];
  out[3] = h[3];
  out[4] = h[0] ? (double)h[1] : -1.0;
  out[5] = h[3] ? (double)h[4] : -1.0;
  out[6] = std::max(maxc, maxr);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamDestroy(s);
  (void)hipFree(flags);
  (void)hipFree(work);
  (void)hipFree(rowpart);
  (void)hipFree(colpart);
  (void)hipFree(B);
  (void)hipFree(A);
  return 0;
}

extern "C" int tkg_screen(int dev, int M, int N, int K, int reps, long long inject, double* out) {
  return screen(dev, 2, M, N, K, reps, inject, out);
}

// the same screen on fp8 e4m3 operands (block-scaled 16x16x128 MFMA, unit scales)
extern "C" int tkg_screen_fp8(int dev, int M, int N, int K, int reps, long long inject, double* out) {
  return screen(dev, 1, M, N, K, reps, inject, out);
}
