// What each rank contributes to the verified all-reduce of the RCCL gate, and the sum
// every rank must then hold (tk_rccl_probe.hip).  Host-only C++, so the rule is unit-tested
// on the CPU (tests/test_rccl_verify.py) against a simulation of the reduction's partial
// sums in bf16.
//
// The sum is compared exactly, so every partial sum the collective forms -- ring, tree,
// any order -- must be representable in the wire type:
//  * f32 holds integers to 2^24: rank r contributes r + 1 (sum world(world+1)/2), which
//    also catches a swapped or duplicated contribution;
//  * bf16 has 8 significant bits (integers exact to 256): r + 1 while the total stays
//    <= 120 (world <= 15), else 1 per rank (every partial sum <= world), exact up to 256
//    ranks.  Larger bf16 worlds cannot be verified exactly and are refused.
#pragma once

constexpr int kBf16RankValuesMaxWorld = 15;
constexpr int kBf16MaxWorld = 256;

static inline bool tk_verifiable(int dtype, int world) { return !(dtype == 1 && world > kBf16MaxWorld); }

static inline float tk_verify_value(int dtype, int world, int rank) {
  return (dtype == 1 && world > kBf16RankValuesMaxWorld) ? 1.0f : (float)(rank + 1);
}

static inline float tk_verify_sum(int dtype, int world) {
  return (dtype == 1 && world > kBf16RankValuesMaxWorld) ? (float)world
                                                           : (float)world * (float)(world + 1) / 2.0f;
}
