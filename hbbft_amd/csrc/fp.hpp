// BLS12-381 base field Fp for gfx950: radix 2^28, 14 limbs in 32-bit VGPRs, Montgomery R = 2^392.
//
// Why radix 2^28 (profiles/r01/ubench_fpmul.txt): every limb product is < 2^56, so a
// whole product-scanning column (<= 28 products + carry) accumulates in ONE 64-bit register with
// v_mad_u64_u32 and no carry-out handling.  hipcc then emits one v_mad_u64_u32 per limb product with
// no v_mov/v_addc glue, and the 11 spare bits let add/sub skip modular reduction before a multiply.
// Measured on MI355X: 69 G Fp-mul/s vs 57.6 (32-bit limbs, inline-asm FIPS) vs 40 (32-bit CIOS).
//
// Invariants ("normalised" = limbs 0..12 < 2^28, top limb holds the rest):
//   fp_mul inputs: limbs < 2^30 and value < 45p;   output: normalised, value < 2p.
//   fp_add / fp_sub / fp_neg: inputs normalised < 2p; output normalised < 2p.
//   Canonical form (< p, non-Montgomery) only at the boundary (fp_from_words / fp_to_words).
#pragma once
#include <stdint.h>
#include "constants.hpp"
#include "words.hpp"

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define HB_HD __host__ __device__ __forceinline__
#else
#define HB_HD inline
#endif

// Field products are real (non-inlined) device functions: one ~450-instruction copy stays hot in the
// instruction cache, and the Fp12-level code above is a compact call sequence.  Fully inlined, one
// final exponentiation is >2 MB of code and takes hipcc tens of minutes.
#if defined(__HIPCC__) || defined(__HIP__)
#define HB_MULFN static __host__ __device__ __noinline__
#else
#define HB_MULFN static
#endif

// Keep each field product a closed scheduling region: without it the machine scheduler interleaves
// dozens of independent products of an Fp12 operation, blowing the register budget (spills) and
// the compile time.  One product alone already saturates the SIMD (FIPS column chains).
#if defined(__HIP_DEVICE_COMPILE__)
#define HB_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define HB_SCHED_FENCE() ((void)0)
#endif

namespace hb {

struct Fp {
  uint32_t l[NL];
};

HB_HD Fp fp_const(const uint32_t (&c)[NL]) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = c[i];
  return r;
}

HB_HD Fp fp_zero() {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = 0;
  return r;
}

HB_HD Fp fp_one() { return fp_const(ONE_L); }

// The non-inlined products take their operands as 14 scalar arguments each: the AMDGPU calling
// convention passes scalars in VGPRs v0-v31 but an aggregate (struct Fp) beyond 16 argument
// registers through the stack, i.e. a scratch store + load of 56 B per operand per call.
#define HB_L14(p) p##0, p##1, p##2, p##3, p##4, p##5, p##6, p##7, p##8, p##9, p##10, p##11, p##12, p##13
#define HB_P14(p) uint32_t p##0, uint32_t p##1, uint32_t p##2, uint32_t p##3, uint32_t p##4, uint32_t p##5, \
                  uint32_t p##6, uint32_t p##7, uint32_t p##8, uint32_t p##9, uint32_t p##10, uint32_t p##11, \
                  uint32_t p##12, uint32_t p##13
#define HB_E14(x) x.l[0], x.l[1], x.l[2], x.l[3], x.l[4], x.l[5], x.l[6], x.l[7], x.l[8], x.l[9], x.l[10], x.l[11], \
                  x.l[12], x.l[13]

// Montgomery product, finely-integrated product scanning (one 64-bit column accumulator).
HB_MULFN Fp fp_mul_l(HB_P14(x), HB_P14(y)) {
  const Fp a = {{HB_L14(x)}};
  const Fp b = {{HB_L14(y)}};
  HB_SCHED_FENCE();
  uint32_t m[NL];
  Fp r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * P_L[k - i];
    m[k] = ((uint32_t)acc * NP0) & LIMB_MASK;
    acc += (uint64_t)m[k] * P_L[0];
    acc >>= LIMB_BITS;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int i = k - NL + 1; i < NL; i++) {
      acc += (uint64_t)a.l[i] * b.l[k - i];
      acc += (uint64_t)m[i] * P_L[k - i];
    }
    r.l[k - NL] = (uint32_t)acc & LIMB_MASK;
    acc >>= LIMB_BITS;
  }
  r.l[NL - 1] = (uint32_t)acc;
  HB_SCHED_FENCE();
  return r;
}

// Squaring: cross products a_i a_j (i < j) once, doubled; same reduction.
HB_MULFN Fp fp_sqr_l(HB_P14(x)) {
  const Fp a = {{HB_L14(x)}};
  HB_SCHED_FENCE();
  uint32_t m[NL];
  Fp r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    uint64_t cross = 0;
#pragma unroll
    for (int i = 0; i < (k + 1) / 2; i++) cross += (uint64_t)a.l[i] * a.l[k - i];
    acc += cross << 1;
    if ((k & 1) == 0) acc += (uint64_t)a.l[k / 2] * a.l[k / 2];
#pragma unroll
    for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * P_L[k - i];
    m[k] = ((uint32_t)acc * NP0) & LIMB_MASK;
    acc += (uint64_t)m[k] * P_L[0];
    acc >>= LIMB_BITS;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    uint64_t cross = 0;
#pragma unroll
    for (int i = k - NL + 1; i < (k + 1) / 2; i++) cross += (uint64_t)a.l[i] * a.l[k - i];
    acc += cross << 1;
    if ((k & 1) == 0) acc += (uint64_t)a.l[k / 2] * a.l[k / 2];
#pragma unroll
    for (int i = k - NL + 1; i < NL; i++) acc += (uint64_t)m[i] * P_L[k - i];
    r.l[k - NL] = (uint32_t)acc & LIMB_MASK;
    acc >>= LIMB_BITS;
  }
  r.l[NL - 1] = (uint32_t)acc;
  HB_SCHED_FENCE();
  return r;
}


HB_HD Fp fp_mul(const Fp& a, const Fp& b) { return fp_mul_l(HB_E14(a), HB_E14(b)); }
HB_HD Fp fp_sqr(const Fp& a) { return fp_sqr_l(HB_E14(a)); }

HB_HD void fp_normalize(Fp& a) {
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    a.l[i + 1] += a.l[i] >> LIMB_BITS;
    a.l[i] &= LIMB_MASK;
  }
}

// x normalised; returns x - K if x >= K else x (K normalised constant).
HB_HD Fp fp_csub(const Fp& x, const uint32_t (&K)[NL]) {
  Fp d;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    int32_t t = (int32_t)x.l[i] - (int32_t)K[i] + br;
    br = t >> 31;                        // 0 or -1 (limbs < 2^28, so |t| < 2^29)
    d.l[i] = (i < NL - 1) ? ((uint32_t)t & LIMB_MASK) : (uint32_t)t;
  }
  const bool ge = (br == 0);
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = ge ? d.l[i] : x.l[i];
  return r;
}

HB_HD Fp fp_add(const Fp& a, const Fp& b) {
  Fp s;
#pragma unroll
  for (int i = 0; i < NL; i++) s.l[i] = a.l[i] + b.l[i];
  fp_normalize(s);
  return fp_csub(s, P2_L);
}

HB_HD Fp fp_sub(const Fp& a, const Fp& b) {
  Fp s;
#pragma unroll
  for (int i = 0; i < NL; i++) s.l[i] = a.l[i] + KP2_L[i] - b.l[i];
  fp_normalize(s);
  return fp_csub(s, P2_L);
}

HB_HD Fp fp_dbl(const Fp& a) { return fp_add(a, a); }

HB_HD Fp fp_neg(const Fp& a) { return fp_sub(fp_zero(), a); }

// Lazy forms: results only valid as fp_mul inputs (limbs < 2^30, value < 45p).
HB_HD Fp fp_add_nr(const Fp& a, const Fp& b) {
  Fp s;
#pragma unroll
  for (int i = 0; i < NL; i++) s.l[i] = a.l[i] + b.l[i];
  return s;
}

HB_HD Fp fp_sel(bool c, const Fp& a, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

// Fully reduce a value < 2p (normalised) to [0, p).
HB_HD Fp fp_reduce_full(const Fp& a) { return fp_csub(a, P_L); }

// Montgomery -> canonical (< p), still in 28-bit limbs.
HB_HD Fp fp_from_mont(const Fp& a) {
  Fp one = fp_zero();
  one.l[0] = 1;
  return fp_reduce_full(fp_mul(a, one));
}

HB_HD Fp fp_to_mont(const Fp& a) { return fp_mul(a, fp_const(R2_L)); }

// 12 little-endian 32-bit words (canonical integer < 2^384) -> 28-bit limbs (not Montgomery).
HB_HD Fp fp_limbs_from_words(const uint32_t w[12]) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const int bit = LIMB_BITS * i;
    const int wi = bit >> 5, sh = bit & 31;
    uint64_t v = w[wi];
    if (wi + 1 < 12) v |= (uint64_t)w[wi + 1] << 32;
    r.l[i] = (uint32_t)(v >> sh) & LIMB_MASK;
  }
  return r;
}

HB_HD void fp_limbs_to_words(const Fp& a, uint32_t w[12]) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const int bit = 32 * i;
    const int li = bit / LIMB_BITS, sh = bit % LIMB_BITS;
    uint64_t v = (uint64_t)a.l[li] >> sh;
    if (li + 1 < NL) v |= (uint64_t)a.l[li + 1] << (LIMB_BITS - sh);
    if (li + 2 < NL) v |= (uint64_t)a.l[li + 2] << (2 * LIMB_BITS - sh);
    w[i] = (uint32_t)v;
  }
}

// canonical words -> Montgomery Fp
HB_HD Fp fp_from_words(const uint32_t w[12]) { return fp_to_mont(fp_limbs_from_words(w)); }

// Montgomery Fp -> canonical words
HB_HD void fp_to_words(const Fp& a, uint32_t w[12]) { fp_limbs_to_words(fp_from_mont(a), w); }

HB_HD bool fp_is_zero_canon(const Fp& c) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) o |= c.l[i];
  return o == 0;
}

// a (Montgomery, < 2p) == 0 mod p
HB_HD bool fp_is_zero(const Fp& a) { return fp_is_zero_canon(fp_reduce_full(a)); }

HB_HD bool fp_eq(const Fp& a, const Fp& b) { return fp_is_zero(fp_sub(a, b)); }

#ifndef HB_FP_LATENCY
// a^(p-2) by left-to-right binary exponentiation over a uniform (compile-time) exponent.
HB_HD Fp fp_inv(const Fp& a) {
  Fp r = a;  // top bit of p-2 is set
  for (int i = PM2_BITS - 2; i >= 0; i--) {
    r = fp_sqr(r);
    if ((PM2_W[i >> 5] >> (i & 31)) & 1) r = fp_mul(r, a);
  }
  return r;
}

#else
HB_HD Fp fp_inv(const Fp& a) {
  uint32_t w[12], p[12], r[12];
  fp_to_words(a, w);
  for (int i = 0; i < 12; i++) p[i] = PM2_W[i];
  p[0] += 2;  // p - 2 + 2 (no carry: the low word of p - 2 is 0xffffaaa9)
  words_inv_vartime<12>(w, p, r);
  return fp_from_words(r);
}
#endif
}  // namespace hb
