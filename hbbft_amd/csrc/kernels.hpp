// Batch kernels of the pairing-equality path (gfx950).
#pragma once
#include "lines.hpp"

namespace hb {

__device__ __forceinline__ Fp12 mul_line_masked(const Fp12& f, const Line& l, const Fp& xP, const Fp& yP, bool active) {
  Fp2 c0 = f2_sel(active, l.c0, f2_one());
  Fp2 c1 = f2_sel(active, f2_mul_fp(l.c1, xP), f2_zero());
  Fp2 c4 = f2_sel(active, f2_mul_fp(l.c4, yP), f2_zero());
  return f12_mul_014(f, c0, c1, c4);
}

// prod_{k=1,2} f_{|x|,Q_k}(P_k) with P2 negated: FE(f) == 1  <=>  e(P1,Q1) == e(P2,Q2).
__device__ __forceinline__ Fp12 miller_2pairs(const G1Aff& P1, const uint4* __restrict__ coef1, int stride1, int q1, bool act1,
                                              const G1Aff& P2n, const uint4* __restrict__ coef2, int stride2, int q2, bool act2) {
  Fp12 f = f12_one();
  int step = 0;
  for (int b = 62; b >= 0; b--) {
    f = f12_sqr(f);
    Line l = load_line(coef1, stride1, step, q1);
    f = mul_line_masked(f, l, P1.x, P1.y, act1);
    l = load_line(coef2, stride2, step, q2);
    f = mul_line_masked(f, l, P2n.x, P2n.y, act2);
    step++;
    if ((X_ABS >> b) & 1) {
      l = load_line(coef1, stride1, step, q1);
      f = mul_line_masked(f, l, P1.x, P1.y, act1);
      l = load_line(coef2, stride2, step, q2);
      f = mul_line_masked(f, l, P2n.x, P2n.y, act2);
      step++;
    }
  }
  return f;
}

__global__ void __launch_bounds__(256, 1) k_pairing_eq(int n,
    const uint32_t* __restrict__ p1, const uint4* __restrict__ coef1, int stride1, const uint8_t* __restrict__ inf1,
    const uint32_t* __restrict__ idx1,
    const uint32_t* __restrict__ p2, const uint4* __restrict__ coef2, int stride2, const uint8_t* __restrict__ inf2,
    const uint32_t* __restrict__ idx2, uint8_t* __restrict__ verdict) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1Aff P1 = g1_from_words(p1 + (size_t)i * G1_WORDS);
  G1Aff P2 = g1_from_words(p2 + (size_t)i * G1_WORDS);
  P2.y = fp_neg(P2.y);
  const int q1 = idx1 ? (int)idx1[i] : i;
  const int q2 = idx2 ? (int)idx2[i] : i;
  const bool act1 = !P1.inf && !inf1[q1];
  const bool act2 = !P2.inf && !inf2[q2];
  Fp12 f = miller_2pairs(P1, coef1, stride1, q1, act1, P2, coef2, stride2, q2, act2);
  Fp12 e = final_exp_x3(f);
  verdict[i] = f12_is_one(e) ? 1 : 0;
}

// Debug: e(P, Q)^3 as canonical words (12 Fp2 coefficients in storage order).
__global__ void __launch_bounds__(256, 1) k_dbg_pairing(int n, const uint32_t* __restrict__ p, const uint4* __restrict__ coef,
                                                        int stride, const uint8_t* __restrict__ inf, uint32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1Aff P = g1_from_words(p + (size_t)i * G1_WORDS);
  const bool act = !P.inf && !inf[i];
  Fp12 f = f12_one();
  int step = 0;
  for (int b = 62; b >= 0; b--) {
    f = f12_sqr(f);
    f = mul_line_masked(f, load_line(coef, stride, step++, i), P.x, P.y, act);
    if ((X_ABS >> b) & 1) f = mul_line_masked(f, load_line(coef, stride, step++, i), P.x, P.y, act);
  }
  f = f12_conj(f);  // x < 0
  Fp12 e = final_exp_x3(f);
  const Fp2* c[6] = {&e.c0.c0, &e.c0.c1, &e.c0.c2, &e.c1.c0, &e.c1.c1, &e.c1.c2};
  uint32_t* o = out + (size_t)i * 144;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    fp_to_words(c[k]->c0, o + 24 * k);
    fp_to_words(c[k]->c1, o + 24 * k + 12);
  }
}

}  // namespace hb
