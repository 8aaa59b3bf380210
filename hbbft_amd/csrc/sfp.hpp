// Signed-limb BLS12-381 Fp / Fp2 (namespace hbs): the base of the lane-pair tower (pfp.hpp) and of the
// lane-quad G1 kernels (k_g1quad.hip).
//
// Representation: 14 int32 limbs of radix 2^28, value = sum l[i] 2^(28 i) (signed), Montgomery
// form with R = 2^392.  "Normalised": l[0..12] in [0, 2^28), l[13] signed.
// Why signed limbs: a - b is 14 plain subtractions (no modulus offset, no carry pass); values stay
// centred on 0, so an Fp2 coefficient needs one cheap top-limb reduction per Fp12 operation
// instead of a carry + conditional subtraction per addition.
//
// Bounds:
//   (M) fp_mul / fp_sqr inputs: |limb| <= 2^29, |value| < 16p -> output normalised in (-p/8, 9p/8).
//       Column sums stay below 14*2^58 + 14*2^56 + 2^36 < 2^62.2: no int64 overflow.
//   (A) fp_add / fp_sub of normalised inputs: normalised output (one carry pass).
//       fp_addl / fp_subl (lazy): |limb| < 2^29 from two normalised inputs -> mul input only.
//   (R) fp_reduce: normalised |v| < 2^30 p -> normalised v in [-p, 2p).
#pragma once
#include <stdint.h>

#include "constants.hpp"

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define HS_HD __host__ __device__ __forceinline__
#else
#define HS_HD inline
#endif

// Product linkage: inlined by default; a translation unit may define HS_MULFN as a static
// non-inlined device function to keep one copy of the product hot in the instruction cache (the
// pairing kernels k_pair.hip, k_quad_g*.hip, k_oct_g*.hip and k_interp_pair.hip do).
#ifndef HS_MULFN
#define HS_MULFN HS_HD
#endif

namespace hbs {

using hb::NL;
using hb::NP0;
using hb::P_L;
constexpr int32_t MASK28 = 0x0fffffff;
constexpr int64_t QINV = 40323;  // floor(2^396 / p): quotient estimate from the top limb
// -p in normalised signed limbs
constexpr int32_t NEGP_L[NL] = {21845,     1048576,  201326662, 5354,      165405012, 99652848,  10014509,
                                13086420,  193508475, 189084297, 72894908, 26630990,  236308096, -106514};

struct Fp {
  int32_t l[NL];
};
struct Fp2 {
  Fp c0, c1;
};

// Montgomery digit m = low 28 bits of (column * -p^-1).  (v_mul_lo_u32 issues at full rate on gfx950,
// tools/ubench_mullo.hip: 30.8 T ops/s; computing it with v_mad_u64_u32 instead measured slower:
// sign 22.87 -> 23.01 ms, profiles/r03/ab_mad_digit.txt.)
HS_HD int32_t mont_digit(int64_t col) { return (int32_t)(((uint32_t)col * NP0) & (uint32_t)MASK28); }

HS_HD Fp fp_zero() {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = 0;
  return r;
}
HS_HD Fp fp_const(const uint32_t (&c)[NL]) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = (int32_t)c[i];
  return r;
}
HS_HD Fp fp_one() { return fp_const(hb::ONE_L); }

// Product scanning (FIPS): column k accumulates a_i b_{k-i} and m_i p_{k-i} in one int64; m_k
// clears the low 28 bits, the arithmetic shift then carries exactly (also for negative sums).
// The multiplier takes its operands as 28 scalar arguments: the AMDGPU calling convention passes
// scalars in VGPRs v0-v31, but an aggregate (struct Fp) beyond 16 argument registers through the
// stack -- a 56-byte scratch store + load per call when HS_MULFN is a real call.
#define HS_L14(p) p##0, p##1, p##2, p##3, p##4, p##5, p##6, p##7, p##8, p##9, p##10, p##11, p##12, p##13
#define HS_P14(p) int32_t p##0, int32_t p##1, int32_t p##2, int32_t p##3, int32_t p##4, int32_t p##5, int32_t p##6, \
                  int32_t p##7, int32_t p##8, int32_t p##9, int32_t p##10, int32_t p##11, int32_t p##12, int32_t p##13
#define HS_E14(x) x.l[0], x.l[1], x.l[2], x.l[3], x.l[4], x.l[5], x.l[6], x.l[7], x.l[8], x.l[9], x.l[10], x.l[11], x.l[12], x.l[13]

HS_MULFN Fp fp_mul_l(HS_P14(x), HS_P14(y)) {
  const Fp a = {{HS_L14(x)}};
  const Fp b = {{HS_L14(y)}};
  int32_t m[NL];
  int64_t acc = 0;
  Fp r;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc += (int64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = 0; i < k; i++) acc += (int64_t)m[i] * (int32_t)P_L[k - i];
    m[k] = mont_digit(acc);
    acc += (int64_t)m[k] * (int32_t)P_L[0];
    acc >>= 28;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int i = k - NL + 1; i < NL; i++) {
      acc += (int64_t)a.l[i] * b.l[k - i];
      acc += (int64_t)m[i] * (int32_t)P_L[k - i];
    }
    r.l[k - NL] = (int32_t)acc & MASK28;
    acc >>= 28;
  }
  r.l[NL - 1] = (int32_t)acc;
  return r;
}

HS_MULFN Fp fp_sqr_l(HS_P14(x)) {
  const Fp a = {{HS_L14(x)}};
  int32_t m[NL];
  int64_t acc = 0;
  Fp r;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    int64_t cr = 0;
#pragma unroll
    for (int i = 0; i < (k + 1) / 2; i++) cr += (int64_t)a.l[i] * a.l[k - i];
    acc += cr * 2;
    if ((k & 1) == 0) acc += (int64_t)a.l[k / 2] * a.l[k / 2];
#pragma unroll
    for (int i = 0; i < k; i++) acc += (int64_t)m[i] * (int32_t)P_L[k - i];
    m[k] = mont_digit(acc);
    acc += (int64_t)m[k] * (int32_t)P_L[0];
    acc >>= 28;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    int64_t cr = 0;
#pragma unroll
    for (int i = k - NL + 1; i < (k + 1) / 2; i++) cr += (int64_t)a.l[i] * a.l[k - i];
    acc += cr * 2;
    if ((k & 1) == 0) acc += (int64_t)a.l[k / 2] * a.l[k / 2];
#pragma unroll
    for (int i = k - NL + 1; i < NL; i++) acc += (int64_t)m[i] * (int32_t)P_L[k - i];
    r.l[k - NL] = (int32_t)acc & MASK28;
    acc >>= 28;
  }
  r.l[NL - 1] = (int32_t)acc;
  return r;
}

HS_HD Fp fp_mul(const Fp& a, const Fp& b) { return fp_mul_l(HS_E14(a), HS_E14(b)); }
HS_HD Fp fp_sqr(const Fp& a) { return fp_sqr_l(HS_E14(a)); }

HS_HD void fp_norm(Fp& a) {
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    const int32_t c = a.l[i] >> 28;
    a.l[i] &= MASK28;
    a.l[i + 1] += c;
  }
}
HS_HD Fp fp_addl(const Fp& a, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = a.l[i] + b.l[i];
  return r;
}
HS_HD Fp fp_subl(const Fp& a, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = a.l[i] - b.l[i];
  return r;
}
HS_HD Fp fp_add(const Fp& a, const Fp& b) {
  Fp r = fp_addl(a, b);
  fp_norm(r);
  return r;
}
HS_HD Fp fp_sub(const Fp& a, const Fp& b) {
  Fp r = fp_subl(a, b);
  fp_norm(r);
  return r;
}
HS_HD Fp fp_neg(const Fp& a) { return fp_sub(fp_zero(), a); }
// k1 a + k2 b for small signed k (|k1|+|k2| <= 7), normalised
HS_HD Fp fp_lin(int k1, const Fp& a, int k2, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = k1 * a.l[i] + k2 * b.l[i];
  fp_norm(r);
  return r;
}
HS_HD Fp fp_sel(bool c, const Fp& a, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}
// (R)
HS_HD Fp fp_reduce(const Fp& a) {
  const int32_t q = (int32_t)(((int64_t)a.l[NL - 1] * QINV) >> 32);
  Fp r;
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    acc += (int64_t)a.l[i] - (int64_t)q * (int32_t)P_L[i];
    r.l[i] = (int32_t)acc & MASK28;
    acc >>= 28;
  }
  r.l[NL - 1] = (int32_t)(acc + a.l[NL - 1] - (int64_t)q * (int32_t)P_L[NL - 1]);
  return r;
}
// v == 0 mod p for normalised |v| < 2^30 p: after reduction v is in {-p, 0, p} exactly then
HS_HD bool fp_is_zero(const Fp& a) {
  const Fp r = fp_reduce(a);
  uint32_t z = 0, zp = 0, zn = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    z |= (uint32_t)r.l[i];
    zp |= (uint32_t)(r.l[i] ^ (int32_t)P_L[i]);
    zn |= (uint32_t)(r.l[i] ^ NEGP_L[i]);
  }
  return z == 0 || zp == 0 || zn == 0;
}

// canonical 12-word integer (< p) -> Montgomery limbs
HS_HD Fp fp_from_words(const uint32_t* w) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const int bit = 28 * i;
    const int wi = bit >> 5, sh = bit & 31;
    uint64_t v = w[wi];
    if (wi + 1 < 12) v |= (uint64_t)w[wi + 1] << 32;
    r.l[i] = (int32_t)((uint32_t)(v >> sh) & (uint32_t)MASK28);
  }
  return fp_mul(r, fp_const(hb::R2_L));
}
// Montgomery -> canonical [0, p) words
HS_HD void fp_to_words(const Fp& a, uint32_t* w) {
  Fp one = fp_zero();
  one.l[0] = 1;
  const Fp r = fp_mul(a, one);  // in (-1, p + 1)
  Fp rp = fp_addl(r, fp_const(P_L));
  fp_norm(rp);
  Fp rm = fp_subl(r, fp_const(P_L));
  fp_norm(rm);
  const Fp c = (r.l[NL - 1] < 0) ? rp : ((rm.l[NL - 1] >= 0) ? rm : r);
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const int bit = 32 * i;
    const int li = bit / 28, sh = bit % 28;
    uint64_t v = (uint64_t)(uint32_t)c.l[li] >> sh;
    if (li + 1 < NL) v |= (uint64_t)(uint32_t)c.l[li + 1] << (28 - sh);
    if (li + 2 < NL) v |= (uint64_t)(uint32_t)c.l[li + 2] << (56 - sh);
    w[i] = (uint32_t)v;
  }
}
HS_HD Fp fp_inv(const Fp& a) {  // a^(p-2)
  Fp r = a;
  for (int i = hb::PM2_BITS - 2; i >= 0; i--) {
    r = fp_sqr(r);
    if ((hb::PM2_W[i >> 5] >> (i & 31)) & 1) r = fp_mul(r, a);
  }
  return r;
}

// ------------------------------------------------------------------ Fp2 = Fp[u]/(u^2+1)
// contracts: f2_mul / f2_sqr inputs |.| < 8p (normalised) -> outputs |.| < 2.5p
HS_HD Fp2 f2_zero() { return {fp_zero(), fp_zero()}; }
HS_HD Fp2 f2_one() { return {fp_one(), fp_zero()}; }
HS_HD Fp2 f2_add(const Fp2& a, const Fp2& b) { return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
HS_HD Fp2 f2_sub(const Fp2& a, const Fp2& b) { return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
HS_HD Fp2 f2_neg(const Fp2& a) { return {fp_neg(a.c0), fp_neg(a.c1)}; }
HS_HD Fp2 f2_conj(const Fp2& a) { return {a.c0, fp_neg(a.c1)}; }
HS_HD Fp2 f2_lin(int k1, const Fp2& a, int k2, const Fp2& b) { return {fp_lin(k1, a.c0, k2, b.c0), fp_lin(k1, a.c1, k2, b.c1)}; }
HS_HD Fp2 f2_sel(bool c, const Fp2& a, const Fp2& b) { return {fp_sel(c, a.c0, b.c0), fp_sel(c, a.c1, b.c1)}; }
HS_HD Fp2 f2_red(const Fp2& a) { return {fp_reduce(a.c0), fp_reduce(a.c1)}; }
HS_HD Fp2 f2_mul_xi(const Fp2& a) { return {fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }  // * (1 + u)
HS_HD Fp2 f2_mul(const Fp2& a, const Fp2& b) {
  const Fp t0 = fp_mul(a.c0, b.c0);
  const Fp t1 = fp_mul(a.c1, b.c1);
  const Fp t2 = fp_mul(fp_addl(a.c0, a.c1), fp_addl(b.c0, b.c1));
  Fp c1 = fp_subl(fp_subl(t2, t0), t1);
  fp_norm(c1);
  return {fp_sub(t0, t1), c1};
}
HS_HD Fp2 f2_sqr(const Fp2& a) {
  const Fp s = fp_mul(fp_addl(a.c0, a.c1), fp_subl(a.c0, a.c1));
  const Fp m = fp_mul(a.c0, a.c1);
  return {s, fp_add(m, m)};
}
HS_HD Fp2 f2_mul_fp(const Fp2& a, const Fp& s) { return {fp_mul(a.c0, s), fp_mul(a.c1, s)}; }
HS_HD Fp2 f2_inv(const Fp2& a) {
  const Fp t = fp_inv(fp_reduce(fp_add(fp_sqr(a.c0), fp_sqr(a.c1))));
  return {fp_mul(a.c0, t), fp_neg(fp_mul(a.c1, t))};
}
HS_HD bool f2_is_zero(const Fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }

}  // namespace hbs
