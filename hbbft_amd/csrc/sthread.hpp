// One-thread-per-check pairing on signed limbs (HBH_IMPL_THREAD_SIGNED): shared pieces of
// k_ts_miller.hip and k_ts_fe.hip.
//
// The pipeline mirrors the lane-cooperative one (k_lc.hip): Miller loop -> easy part -> five
// cyclotomic exponentiations by x / x-1 with two Frobenius glue steps -> verdict, one kernel per
// stage, the Fp12 state handed over through HBM between stages.  Handing over costs 2 x 672 B per
// check per stage (~90 MB for 65,536 checks, ~20 us at HBM rate, <0.1% of the pipeline) and buys
// small kernels: each compiles in its own register budget and fits the instruction cache.
//
// State layout: 42 int4 chunks per check (12 Fp x 14 limbs, tower order c0.c0 .. c1.c2), chunk q of
// check i at st[q * stride + i], stride = pad64(n): a wave's 64 lanes read 64 consecutive 16-byte
// chunks (fully coalesced).
#pragma once
#include "stower.hpp"

namespace hbs {

constexpr int ST_Q4 = 42;

__device__ __forceinline__ void st12(int4* __restrict__ st, int stride, int i, const Fp12& f) {
  const Fp* c[12] = {&f.c0.c0.c0, &f.c0.c0.c1, &f.c0.c1.c0, &f.c0.c1.c1, &f.c0.c2.c0, &f.c0.c2.c1,
                     &f.c1.c0.c0, &f.c1.c0.c1, &f.c1.c1.c0, &f.c1.c1.c1, &f.c1.c2.c0, &f.c1.c2.c1};
  int32_t w[168];
#pragma unroll
  for (int k = 0; k < 12; k++)
#pragma unroll
    for (int j = 0; j < NL; j++) w[k * NL + j] = c[k]->l[j];
#pragma unroll
  for (int q = 0; q < ST_Q4; q++) st[(size_t)q * stride + i] = make_int4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

__device__ __forceinline__ Fp12 ld12(const int4* __restrict__ st, int stride, int i) {
  int32_t w[168];
#pragma unroll
  for (int q = 0; q < ST_Q4; q++) {
    const int4 v = st[(size_t)q * stride + i];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
  Fp12 f;
  Fp* c[12] = {&f.c0.c0.c0, &f.c0.c0.c1, &f.c0.c1.c0, &f.c0.c1.c1, &f.c0.c2.c0, &f.c0.c2.c1,
               &f.c1.c0.c0, &f.c1.c0.c1, &f.c1.c1.c0, &f.c1.c1.c1, &f.c1.c2.c0, &f.c1.c2.c1};
#pragma unroll
  for (int k = 0; k < 12; k++)
#pragma unroll
    for (int j = 0; j < NL; j++) c[k]->l[j] = w[k * NL + j];
  return f;
}

}  // namespace hbs
