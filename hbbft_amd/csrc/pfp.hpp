// Lane-pair BLS12-381 tower for the fused pairing kernel (k_pair.hip), namespace hbs.
//
// Every Fp2 value a = a0 + a1 u is split over two adjacent lanes of a wave: the even lane holds a0,
// the odd lane a1 (signed 14 x 28-bit limbs of sfp.hpp).  An Fp6 / Fp12 value is then 3 / 6 such
// components per lane, so one check's whole Miller-loop and final-exponentiation state fits half a
// register file, and a 65,536-check batch runs two waves per SIMD -- the occupancy at which the MAD
// pipe is saturated (tools/ubench_v2.hip: 50 G Fp-mul/s at one wave per SIMD, 74 G at two).
//
// Fp2 arithmetic in this split does no redundant work:
//   a * b : the even lane forms a0 b0 - a1 b1, the odd lane a1 b0 + a0 b1 -- both are x y + z w with
//           x = own a, y = b0, z = -+partner a, w = b1; one lazily reduced product of 588 MADs per
//           lane (2 x 196 product + 196 reduction), exactly half of a 3 x 392-MAD Karatsuba product.
//   a^2   : even (a0 + a1)(a0 - a1), odd 2 a0 a1: one 392-MAD product per lane.
//   a * s (s in Fp), a + b, a - b: each lane on its own component.
// Partner operands travel through DPP quad permutations (one full-rate v_mov_dpp per limb): swap
// [1,0,3,2], broadcast-even [0,0,2,2], broadcast-odd [1,1,3,3].  Both lanes of a pair always take
// the same control flow (every branch below depends only on the check, never on the lane parity),
// so a DPP source lane is always active.
//
// Value contracts (per Fp component, signed, normalised = limbs 0..12 in [0, 2^28)):
//   h_mul(a, b): a normalised or lazy (|limb| <= 2^29), b normalised, |a|, |b| < 16p -> normalised,
//                |out| < 1.25p + |a||b| 2^-392 bound (column sums < 2^62.1).
//   h_sqr(a)   : a normalised, |a| < 16p -> normalised (fp_mul_l contract (M) on (a0+-a1, a0-a1)).
//   Fp12 values between operations are reduced (|.| < 2p).  The tower formulas are pairing 0.14's
//   (restated in oracle/c/bls_cpu.c: Karatsuba Fp6, complex Fp12 squaring, Granger-Scott squaring).
#pragma once
#include "sfp.hpp"
#include "words.hpp"

#define HP_D __device__ __forceinline__

namespace hbs {

// ---------------------------------------------------------------- lane pair
constexpr int DPP_SWAP = 0xB1;  // quad_perm [1,0,3,2]
constexpr int DPP_EVEN = 0xA0;  // quad_perm [0,0,2,2]
constexpr int DPP_ODD = 0xF5;   // quad_perm [1,1,3,3]

HP_D bool lp_even() { return (threadIdx.x & 1) == 0; }
template <int CTRL>
HP_D int32_t dpp(int32_t v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
HP_D Fp dpp_fp(const Fp& a) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = dpp<CTRL>(a.l[i]);
  return r;
}

// own component of a * b (Fp2)
HS_MULFN Fp h_mul_l(HS_P14(x), HS_P14(y)) {
  const Fp a = {{HS_L14(x)}};
  const Fp b = {{HS_L14(y)}};
  const int32_t sm = lp_even() ? -1 : 0;  // the even lane subtracts a1 b1
  int32_t Y[NL], W[NL], Z[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) {
    Y[i] = dpp<DPP_EVEN>(b.l[i]);
    W[i] = dpp<DPP_ODD>(b.l[i]);
    Z[i] = (dpp<DPP_SWAP>(a.l[i]) ^ sm) - sm;
  }
  int32_t m[NL];
  int64_t acc = 0;
  Fp r;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) {
      acc += (int64_t)a.l[i] * Y[k - i];
      acc += (int64_t)Z[i] * W[k - i];
    }
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
      acc += (int64_t)a.l[i] * Y[k - i];
      acc += (int64_t)Z[i] * W[k - i];
      acc += (int64_t)m[i] * (int32_t)P_L[k - i];
    }
    r.l[k - NL] = (int32_t)acc & MASK28;
    acc >>= 28;
  }
  r.l[NL - 1] = (int32_t)acc;
  return r;
}

HP_D Fp h_mul(const Fp& a, const Fp& b) { return h_mul_l(HS_E14(a), HS_E14(b)); }

// own component of a^2: even (a0 + a1)(a0 - a1), odd (a1 + a1) a0... written as x * y with
// x = pa + (even ? a : pa), y = a - (even ? pa : 0)  (odd lane: x = 2 a0, y = a1)
HP_D Fp h_sqr(const Fp& a) {
  const bool ev = lp_even();
  const Fp pa = dpp_fp<DPP_SWAP>(a);
  Fp x, y;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    x.l[i] = pa.l[i] + (ev ? a.l[i] : pa.l[i]);
    y.l[i] = a.l[i] - (ev ? pa.l[i] : 0);
  }
  return fp_mul(x, y);
}

// a * (1 + u): even a0 - a1, odd a1 + a0
HP_D Fp h_mul_xi(const Fp& a) {
  const int32_t sm = lp_even() ? -1 : 0;
  const Fp pa = dpp_fp<DPP_SWAP>(a);
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = a.l[i] + ((pa.l[i] ^ sm) - sm);
  fp_norm(r);
  return r;
}
// conjugate: the odd lane negates
HP_D Fp h_conj(const Fp& a) {
  const Fp n = fp_neg(a);
  return lp_even() ? a : n;
}
HP_D Fp h_zero() { return fp_zero(); }
HP_D Fp h_one() { return lp_even() ? fp_one() : fp_zero(); }
// Fp2 constant (c0, c1): each lane takes its own component
HP_D Fp h_const(const uint32_t (&c0)[NL], const uint32_t (&c1)[NL]) {
  Fp r;
  const bool ev = lp_even();
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = (int32_t)(ev ? c0[i] : c1[i]);
  return r;
}
// pair-wide AND of a per-lane flag
HP_D bool lp_both(bool v) { return (v ? 1 : 0) & dpp<DPP_SWAP>(v ? 1 : 0); }
HP_D bool h_is_zero(const Fp& a) { return lp_both(fp_is_zero(a)); }
// 1 / a in Fp2 with a variable-time inverse of the (public) norm: both lanes invert the same norm.
// a = 0 gives 0 (the binary Euclid loop would not terminate on a zero norm).
template <int MODE = 0>
HP_D Fp h_inv_vartime(const Fp& a) {
  const Fp s = fp_sqr(a);
  const Fp n = fp_add(s, dpp_fp<DPP_SWAP>(s));
  uint32_t w[12], p[12], r[12];
  fp_to_words(n, w);
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) nz |= w[i];
  if (nz == 0) return fp_zero();
#pragma unroll
  for (int i = 0; i < 12; i++) p[i] = hb::PM2_W[i];
  p[0] += 2;  // p - 2 + 2
  hb::words_inv_vartime<12, MODE>(w, p, r);
  return h_conj(fp_mul(a, fp_from_words(r)));
}

// ---------------------------------------------------------------- one-pass reductions
// reduce(M t + K a) in one carry pass: t unnormalised limbs (|t_i| < 2^31), a normalised, |M|, |K|
// <= 3.  The quotient comes from the top limb alone (as in fp_reduce); the lower limbs' excess moves
// the value by < 2^368 < 2^-12 p, so the output is normalised and in (-p/1000, p + p/1000) --
// inside (R).  Replaces a normalisation pass per sum plus fp_reduce's pass.
template <int M, int K>
HP_D Fp fp_red_mk(const Fp& t, const Fp& a) {
  const int64_t top = (int64_t)t.l[NL - 1] * M + (int64_t)K * a.l[NL - 1];
  const int32_t q = (int32_t)((top * QINV) >> 32);
  Fp r;
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    acc += (int64_t)t.l[i] * M + (int64_t)K * a.l[i] - (int64_t)q * (int32_t)P_L[i];
    r.l[i] = (int32_t)acc & MASK28;
    acc >>= 28;
  }
  r.l[NL - 1] = (int32_t)(acc + top - (int64_t)q * (int32_t)P_L[NL - 1]);
  return r;
}
HP_D Fp fp_red_l(const Fp& t) { return fp_red_mk<1, 0>(t, t); }
// own component of s + xi t without normalising (|s_i| + 2 |t_i| < 2^31)
HP_D Fp h_add_xi_l(const Fp& s, const Fp& t) {
  const int32_t sm = lp_even() ? -1 : 0;
  const Fp pt = dpp_fp<DPP_SWAP>(t);
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = s.l[i] + t.l[i] + ((pt.l[i] ^ sm) - sm);
  return r;
}
// a - b - c without normalising
HP_D Fp fp_sub2l(const Fp& a, const Fp& b, const Fp& c) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = a.l[i] - b.l[i] - c.l[i];
  return r;
}

// own component of xi t without normalising
HP_D Fp h_xi_l(const Fp& t) {
  const int32_t sm = lp_even() ? -1 : 0;
  const Fp pt = dpp_fp<DPP_SWAP>(t);
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = t.l[i] + ((pt.l[i] ^ sm) - sm);
  return r;
}

// ---------------------------------------------------------------- Fp6 / Fp12 (own components)
struct H6 { Fp c0, c1, c2; };
struct H12 { H6 c0, c1; };

HP_D H6 h6_zero() { return {h_zero(), h_zero(), h_zero()}; }
HP_D H6 h6_one() { return {h_one(), h_zero(), h_zero()}; }
HP_D H6 h6_add(const H6& a, const H6& b) { return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1), fp_add(a.c2, b.c2)}; }
HP_D H6 h6_sub(const H6& a, const H6& b) { return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1), fp_sub(a.c2, b.c2)}; }
HP_D H6 h6_neg(const H6& a) { return {fp_neg(a.c0), fp_neg(a.c1), fp_neg(a.c2)}; }
HP_D H6 h6_red(const H6& a) { return {fp_reduce(a.c0), fp_reduce(a.c1), fp_reduce(a.c2)}; }
HP_D H6 h6_mul_v(const H6& a) { return {h_mul_xi(a.c2), a.c0, a.c1}; }

// Karatsuba, inputs < 4p; outputs reduced (one carry pass each, fp_red_l).  Register-frugal order:
// each output is formed as soon as its products exist (c0 before t1, t2 are computed), so at most
// five Fp2 values are live beside the operands across the product calls.
HP_D H6 h6_mul(const H6& a, const H6& b) {
  const Fp v1 = h_mul(a.c1, b.c1);
  const Fp v2 = h_mul(a.c2, b.c2);
  const Fp d0 = fp_sub2l(h_mul(fp_addl(a.c1, a.c2), fp_add(b.c1, b.c2)), v1, v2);
  const Fp v0 = h_mul(a.c0, b.c0);
  const Fp c0 = fp_red_l(h_add_xi_l(v0, d0));  // v0 + xi (t0 - v1 - v2)
  const Fp c1 = fp_red_l(h_add_xi_l(fp_sub2l(h_mul(fp_addl(a.c0, a.c1), fp_add(b.c0, b.c1)), v0, v1), v2));
  const Fp c2 = fp_red_l(fp_addl(fp_sub2l(h_mul(fp_addl(a.c0, a.c2), fp_add(b.c0, b.c2)), v0, v2), v1));
  return {c0, c1, c2};
}
// x (a + b v)
HP_D H6 h6_mul_01(const H6& x, const Fp& a, const Fp& b) {
  const Fp t0 = h_mul(x.c0, a);
  const Fp t1 = h_mul(x.c1, b);
  const Fp u = h_mul(x.c2, b);
  const Fp w = h_mul(x.c2, a);
  const Fp s = h_mul(fp_addl(x.c0, x.c1), fp_add(a, b));
  return {fp_add(t0, h_mul_xi(u)), fp_sub(fp_subl(s, t0), t1), fp_add(t1, w)};
}
// x (b v)
HP_D H6 h6_mul_1(const H6& x, const Fp& b) {
  const Fp r0 = h_mul(x.c2, b);
  const Fp r1 = h_mul(x.c0, b);
  const Fp r2 = h_mul(x.c1, b);
  return {h_mul_xi(r0), r1, r2};
}
HP_D H6 h6_inv(const H6& a) {
  const Fp c0 = fp_reduce(fp_sub(h_sqr(a.c0), h_mul_xi(h_mul(a.c1, a.c2))));
  const Fp c1 = fp_reduce(fp_sub(h_mul_xi(h_sqr(a.c2)), h_mul(a.c0, a.c1)));
  const Fp c2 = fp_reduce(fp_sub(h_sqr(a.c1), h_mul(a.c0, a.c2)));
  const Fp t = fp_reduce(fp_add(h_mul(a.c0, c0), h_mul_xi(fp_add(h_mul(a.c2, c1), h_mul(a.c1, c2)))));
  // the final exponentiation's one inversion: values are public (share checks), so the binary-GCD
  // inverse (25 rounds of 31 divsteps) replaces Fermat's 380 squarings + ~190 products (A/B on one
  // box: sign 23.4 -> 22.7 ms, decrypt 21.6 -> 20.8 ms per 65,536 checks, profiles/r03/ab_inv.txt)
  const Fp ti = fp_reduce(h_inv_vartime(t));
  return {h_mul(c0, ti), h_mul(c1, ti), h_mul(c2, ti)};
}

HP_D H12 h12_one() { return {h6_one(), h6_zero()}; }
HP_D H12 h12_conj(const H12& a) { return {a.c0, h6_neg(a.c1)}; }
HP_D H12 h12_red(const H12& a) { return {h6_red(a.c0), h6_red(a.c1)}; }
// Karatsuba recombination (t0 + v t1, s - t0 - t1) of normalised Fp6 products, reduced in one pass
// per component
HP_D H12 h12_kcomb(const H6& t0, const H6& t1, const H6& s) {
  return {{fp_red_l(h_add_xi_l(t0.c0, t1.c2)), fp_red_l(fp_addl(t0.c1, t1.c0)), fp_red_l(fp_addl(t0.c2, t1.c1))},
          {fp_red_l(fp_sub2l(s.c0, t0.c0, t1.c0)), fp_red_l(fp_sub2l(s.c1, t0.c1, t1.c1)),
           fp_red_l(fp_sub2l(s.c2, t0.c2, t1.c2))}};
}

// inputs reduced; output reduced
HP_D H12 h12_mul(const H12& a, const H12& b) {
  const H6 t0 = h6_mul(a.c0, b.c0);
  const H6 t1 = h6_mul(a.c1, b.c1);
  const H6 s = h6_mul(h6_add(a.c0, a.c1), h6_add(b.c0, b.c1));
  return h12_kcomb(t0, t1, s);
}
// complex squaring: t = a0 a1, s = (a0 + a1)(a0 + v a1); c0 = s - t - v t, c1 = 2 t (one pass each)
HP_D H12 h12_sqr(const H12& a) {
  const H6 t = h6_mul(a.c0, a.c1);
  const H6 s = h6_mul(h6_add(a.c0, a.c1), h6_red(h6_add(a.c0, h6_mul_v(a.c1))));
  return {{fp_red_l(h_add_xi_l(fp_subl(s.c0, t.c0), fp_subl(fp_zero(), t.c2))), fp_red_l(fp_sub2l(s.c1, t.c1, t.c0)),
           fp_red_l(fp_sub2l(s.c2, t.c2, t.c1))},
          {fp_red_l(fp_addl(t.c0, t.c0)), fp_red_l(fp_addl(t.c1, t.c1)), fp_red_l(fp_addl(t.c2, t.c2))}};
}
// f (c0 + c1 w^2 + c4 w^3); c0, c1, c4 normalised, < 2p
HP_D H12 h12_mul_014(const H12& f, const Fp& c0, const Fp& c1, const Fp& c4) {
  const H6 fs = h6_add(f.c0, f.c1);
  const Fp c14 = fp_add(c1, c4);
  const H6 t0 = h6_red(h6_mul_01(f.c0, c0, c1));
  const H6 t1 = h6_red(h6_mul_1(f.c1, c4));
  const H6 s = h6_red(h6_mul_01(fs, c0, c14));
  return h12_red({h6_add(t0, h6_mul_v(t1)), h6_sub(h6_sub(s, t0), t1)});
}
// x (b1 v + b2 v^2): c0 = xi (a1 b2 + a2 b1), c1 = a0 b1 + xi a2 b2, c2 = a0 b2 + a1 b1 (5 products);
// outputs reduced
HP_D H6 h6_mul_12(const H6& x, const Fp& b1, const Fp& b2) {
  const Fp u = h_mul(x.c1, b1);
  const Fp w = h_mul(x.c2, b2);
  const Fp c0 = fp_red_l(h_xi_l(fp_sub2l(h_mul(fp_addl(x.c1, x.c2), fp_add(b1, b2)), u, w)));
  const Fp c1 = fp_red_l(h_add_xi_l(h_mul(x.c0, b1), w));
  const Fp c2 = fp_red_l(fp_addl(h_mul(x.c0, b2), u));
  return {c0, c1, c2};
}
// f * (la * lb) for two sparse lines (c0 + c1 w^2 + c4 w^3 each, normalised, < 2p): the line
// product L = (C0, C1) has C1.c0 = 0 (6 products), then one Karatsuba step with the sparse C1
// (6 + 5 + 6 products) -- 23 lane-pair products instead of 2 x 13 for two h12_mul_014.
HP_D H12 h12_mul_lines(const H12& f, const Fp& a0, const Fp& a1, const Fp& a4, const Fp& b0, const Fp& b1,
                       const Fp& b4) {
  const Fp a0b0 = h_mul(a0, b0);
  const Fp a1b1 = h_mul(a1, b1);
  const Fp a4b4 = h_mul(a4, b4);
  // the line product L = (C0, (0, c11, c12)), each coefficient reduced in one carry pass
  const Fp c11 = fp_red_l(fp_sub2l(h_mul(fp_addl(a0, a4), fp_add(b0, b4)), a0b0, a4b4));
  const Fp c12 = fp_red_l(fp_sub2l(h_mul(fp_addl(a1, a4), fp_add(b1, b4)), a1b1, a4b4));
  const H6 C0 = {fp_red_l(h_add_xi_l(a0b0, a4b4)),
                 fp_red_l(fp_sub2l(h_mul(fp_addl(a0, a1), fp_add(b0, b1)), a0b0, a1b1)), a1b1};
  // f L: Karatsuba over Fp6 with the sparse L.c1 (6 + 5 + 6 products); h6_mul / h6_mul_12 reduce
  const H6 t0 = h6_mul(f.c0, C0);
  const H6 t1 = h6_mul_12(f.c1, c11, c12);
  const H6 s = h6_mul(h6_add(f.c0, f.c1), {C0.c0, fp_add(C0.c1, c11), fp_add(C0.c2, c12)});
  return h12_kcomb(t0, t1, s);
}
HP_D H12 h12_inv(const H12& a) {
  const H6 t = h6_red(h6_sub(h6_red(h6_mul(a.c0, a.c0)), h6_red(h6_mul_v(h6_red(h6_mul(a.c1, a.c1))))));
  const H6 ti = h6_red(h6_inv(t));
  return h12_red({h6_mul(a.c0, ti), h6_neg(h6_mul(a.c1, ti))});
}

#define HP_FROB1(K) h_const(hb::FROB1_##K##_C0, hb::FROB1_##K##_C1)
HP_D H12 h12_frob1(const H12& f) {
  H12 r;
  r.c0.c0 = h_conj(f.c0.c0);
  r.c1.c0 = h_mul(h_conj(f.c1.c0), HP_FROB1(1));
  r.c0.c1 = h_mul(h_conj(f.c0.c1), HP_FROB1(2));
  r.c1.c1 = h_mul(h_conj(f.c1.c1), HP_FROB1(3));
  r.c0.c2 = h_mul(h_conj(f.c0.c2), HP_FROB1(4));
  r.c1.c2 = h_mul(h_conj(f.c1.c2), HP_FROB1(5));
  return h12_red(r);
}
HP_D H12 h12_frob2(const H12& f) {
  H12 r;
  r.c0.c0 = f.c0.c0;
  r.c1.c0 = fp_mul(f.c1.c0, fp_const(hb::FROB2_1_C0));
  r.c0.c1 = fp_mul(f.c0.c1, fp_const(hb::FROB2_2_C0));
  r.c1.c1 = fp_mul(f.c1.c1, fp_const(hb::FROB2_3_C0));
  r.c0.c2 = fp_mul(f.c0.c2, fp_const(hb::FROB2_4_C0));
  r.c1.c2 = fp_mul(f.c1.c2, fp_const(hb::FROB2_5_C0));
  return r;
}

// Granger-Scott cyclotomic squaring, input reduced, output reduced.
// Each output 3 A -/+ 2 a is formed from the unnormalised squares and reduced in one carry pass
// (fp_red_mk) instead of normalising A, the linear combination and the reduction separately.
HP_D H12 h12_cyclo_sqr(const H12& f) {
  const Fp& a0 = f.c0.c0; const Fp& a2 = f.c0.c1; const Fp& a4 = f.c0.c2;
  const Fp& a1 = f.c1.c0; const Fp& a3 = f.c1.c1; const Fp& a5 = f.c1.c2;
  H12 r;
  {
    const Fp s0 = h_sqr(a0), s3 = h_sqr(a3), s03 = h_sqr(fp_add(a0, a3));
    r.c0.c0 = fp_red_mk<3, -2>(h_add_xi_l(s0, s3), a0);
    r.c1.c1 = fp_red_mk<3, 2>(fp_sub2l(s03, s0, s3), a3);
  }
  {
    const Fp s1 = h_sqr(a1), s4 = h_sqr(a4), s14 = h_sqr(fp_add(a1, a4));
    r.c0.c1 = fp_red_mk<3, -2>(h_add_xi_l(s1, s4), a2);
    r.c1.c2 = fp_red_mk<3, 2>(fp_sub2l(s14, s1, s4), a5);
  }
  {
    const Fp s2 = h_sqr(a2), s5 = h_sqr(a5), s25 = h_sqr(fp_add(a2, a5));
    r.c0.c2 = fp_red_mk<3, -2>(h_add_xi_l(s2, s5), a4);
    r.c1.c0 = fp_red_mk<3, 2>(h_add_xi_l(fp_zero(), fp_sub2l(s25, s2, s5)), a1);
  }
  return r;
}

HP_D bool h12_is_one(const H12& f) {
  bool ok = fp_is_zero(fp_sub(f.c0.c0, h_one()));
  ok = ok && fp_is_zero(f.c0.c1) && fp_is_zero(f.c0.c2);
  ok = ok && fp_is_zero(f.c1.c0) && fp_is_zero(f.c1.c1) && fp_is_zero(f.c1.c2);
  return lp_both(ok);
}

// ---------------------------------------------------------------- G2 walk (pairing 0.14's line formulas)
// T in Jacobian coordinates; lines scaled as pairing 0.14 scales them (the Fp2 factors die in the final
// exponentiation).  Each lane holds its components of T, Q and the line.
struct HJac { Fp x, y, z; };
struct HLine { Fp c0, c1, c4; };

HP_D HLine h_dbl_step(HJac& T) {
  const Fp A = h_sqr(T.x);
  const Fp B = h_sqr(T.y);
  const Fp C = h_sqr(B);
  const Fp D = fp_lin(2, fp_sub(fp_sub(h_sqr(fp_add(T.x, B)), A), C), 0, C);
  const Fp E = fp_lin(3, A, 0, A);
  const Fp ZZ = h_sqr(T.z);
  HLine l;
  l.c0 = fp_sub(h_mul(E, T.x), fp_add(B, B));
  l.c1 = fp_neg(h_mul(E, ZZ));
  const Fp Z3 = fp_sub(fp_sub(h_sqr(fp_add(T.y, T.z)), B), ZZ);
  l.c4 = h_mul(Z3, ZZ);
  const Fp F = h_sqr(E);
  const Fp X3 = fp_sub(F, fp_add(D, D));
  T.y = fp_sub(h_mul(E, fp_sub(D, X3)), fp_lin(8, C, 0, C));
  T.x = X3;
  T.z = Z3;
  l.c0 = fp_reduce(l.c0);
  T.x = fp_reduce(T.x);
  T.y = fp_reduce(T.y);
  T.z = fp_reduce(T.z);
  return l;
}

HP_D HLine h_add_step(HJac& T, const Fp& xQ, const Fp& yQ) {
  const Fp Z1Z1 = h_sqr(T.z);
  const Fp U2 = h_mul(xQ, Z1Z1);
  const Fp S2 = h_mul(h_mul(yQ, T.z), Z1Z1);
  const Fp H = fp_sub(U2, T.x);
  const Fp r = fp_sub(S2, T.y);
  const Fp HH = h_sqr(H);
  const Fp HHH = h_mul(H, HH);
  const Fp V = h_mul(T.x, HH);
  const Fp X3 = fp_sub(fp_sub(h_sqr(r), HHH), fp_add(V, V));
  const Fp Y3 = fp_sub(h_mul(r, fp_sub(V, X3)), h_mul(T.y, HHH));
  const Fp Z3 = h_mul(T.z, H);
  HLine l;
  l.c0 = fp_reduce(fp_sub(h_mul(r, xQ), h_mul(yQ, Z3)));
  l.c1 = fp_neg(r);
  l.c4 = Z3;
  T.x = fp_reduce(X3);
  T.y = fp_reduce(Y3);
  T.z = Z3;
  return l;
}

// ---------------------------------------------------------------- boundary formats
// own component of an ABI G2 coordinate pair (x.c0 x.c1 y.c0 y.c1, 12 words each)
HP_D void h_g2_load(const uint32_t* __restrict__ w, Fp& x, Fp& y) {
  const int o = lp_even() ? 0 : 12;
  x = fp_from_words(w + o);
  y = fp_from_words(w + 24 + o);
}
HP_D bool words_zero(const uint32_t* __restrict__ w, int n) {
  uint32_t o = 0;
  for (int k = 0; k < n; k++) o |= w[k];
  return o == 0;
}

}  // namespace hbs
