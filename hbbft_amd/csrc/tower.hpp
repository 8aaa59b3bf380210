// Extension tower for BLS12-381 on gfx950:
//   Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3-xi) with xi = 1+u, Fp12 = Fp6[w]/(w^2-v).
// Same tower as pairing 0.14; only verdicts and canonical group elements cross
// the boundary, so the internal choice of formulas is free.  Formulas are validated on the CPU by
// tools/model_pairing.py against the oracle before being written here.
#pragma once
#include "fp.hpp"

namespace hb {

struct Fp2 { Fp c0, c1; };
struct Fp6 { Fp2 c0, c1, c2; };
struct Fp12 { Fp6 c0, c1; };

// ------------------------------------------------------------------ Fp2
HB_HD Fp2 f2_zero() { return {fp_zero(), fp_zero()}; }
HB_HD Fp2 f2_one() { return {fp_one(), fp_zero()}; }
HB_HD Fp2 f2_add(const Fp2& a, const Fp2& b) { return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
HB_HD Fp2 f2_sub(const Fp2& a, const Fp2& b) { return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
HB_HD Fp2 f2_dbl(const Fp2& a) { return {fp_dbl(a.c0), fp_dbl(a.c1)}; }
HB_HD Fp2 f2_neg(const Fp2& a) { return {fp_neg(a.c0), fp_neg(a.c1)}; }
HB_HD Fp2 f2_conj(const Fp2& a) { return {a.c0, fp_neg(a.c1)}; }
HB_HD Fp2 f2_sel(bool c, const Fp2& a, const Fp2& b) { return {fp_sel(c, a.c0, b.c0), fp_sel(c, a.c1, b.c1)}; }

HB_HD Fp2 f2_mul(const Fp2& a, const Fp2& b) {
  Fp t0 = fp_mul(a.c0, b.c0);
  Fp t1 = fp_mul(a.c1, b.c1);
  Fp t2 = fp_mul(fp_add_nr(a.c0, a.c1), fp_add_nr(b.c0, b.c1));
  return {fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}

HB_HD Fp2 f2_sqr(const Fp2& a) {
  // (a0 + a1)(a0 - a1) + 2 a0 a1 u
  Fp s = fp_add_nr(a.c0, a.c1);
  Fp d = fp_sub(a.c0, a.c1);
  Fp m = fp_mul(a.c0, a.c1);
  return {fp_mul(s, d), fp_dbl(m)};
}

HB_HD Fp2 f2_mul_fp(const Fp2& a, const Fp& s) { return {fp_mul(a.c0, s), fp_mul(a.c1, s)}; }

// multiply by xi = 1 + u: (a0 - a1) + (a0 + a1) u
HB_HD Fp2 f2_mul_xi(const Fp2& a) { return {fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }

HB_HD Fp2 f2_inv(const Fp2& a) {
  Fp t = fp_inv(fp_add(fp_sqr(a.c0), fp_sqr(a.c1)));
  return {fp_mul(a.c0, t), fp_neg(fp_mul(a.c1, t))};
}

HB_HD bool f2_is_zero(const Fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }

// ------------------------------------------------------------------ Fp6
HB_HD Fp6 f6_zero() { return {f2_zero(), f2_zero(), f2_zero()}; }
HB_HD Fp6 f6_one() { return {f2_one(), f2_zero(), f2_zero()}; }
HB_HD Fp6 f6_add(const Fp6& a, const Fp6& b) { return {f2_add(a.c0, b.c0), f2_add(a.c1, b.c1), f2_add(a.c2, b.c2)}; }
HB_HD Fp6 f6_sub(const Fp6& a, const Fp6& b) { return {f2_sub(a.c0, b.c0), f2_sub(a.c1, b.c1), f2_sub(a.c2, b.c2)}; }
HB_HD Fp6 f6_neg(const Fp6& a) { return {f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; }
HB_HD Fp6 f6_mul_v(const Fp6& a) { return {f2_mul_xi(a.c2), a.c0, a.c1}; }

HB_HD Fp6 f6_mul(const Fp6& a, const Fp6& b) {
  Fp2 v0 = f2_mul(a.c0, b.c0);
  Fp2 v1 = f2_mul(a.c1, b.c1);
  Fp2 v2 = f2_mul(a.c2, b.c2);
  Fp2 t0 = f2_sub(f2_sub(f2_mul(f2_add(a.c1, a.c2), f2_add(b.c1, b.c2)), v1), v2);
  Fp2 t1 = f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b.c0, b.c1)), v0), v1);
  Fp2 t2 = f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c2), f2_add(b.c0, b.c2)), v0), v2);
  return {f2_add(v0, f2_mul_xi(t0)), f2_add(t1, f2_mul_xi(v2)), f2_add(t2, v1)};
}

// x * (a + b v)
HB_HD Fp6 f6_mul_01(const Fp6& x, const Fp2& a, const Fp2& b) {
  Fp2 t0 = f2_mul(x.c0, a);
  Fp2 t1 = f2_mul(x.c1, b);
  Fp2 c0 = f2_add(t0, f2_mul_xi(f2_mul(x.c2, b)));
  Fp2 c1 = f2_sub(f2_sub(f2_mul(f2_add(x.c0, x.c1), f2_add(a, b)), t0), t1);
  Fp2 c2 = f2_add(t1, f2_mul(x.c2, a));
  return {c0, c1, c2};
}

// x * (b v)
HB_HD Fp6 f6_mul_1(const Fp6& x, const Fp2& b) {
  return {f2_mul_xi(f2_mul(x.c2, b)), f2_mul(x.c0, b), f2_mul(x.c1, b)};
}

HB_HD Fp6 f6_inv(const Fp6& a) {
  Fp2 c0 = f2_sub(f2_sqr(a.c0), f2_mul_xi(f2_mul(a.c1, a.c2)));
  Fp2 c1 = f2_sub(f2_mul_xi(f2_sqr(a.c2)), f2_mul(a.c0, a.c1));
  Fp2 c2 = f2_sub(f2_sqr(a.c1), f2_mul(a.c0, a.c2));
  Fp2 t = f2_add(f2_mul(a.c0, c0), f2_mul_xi(f2_add(f2_mul(a.c2, c1), f2_mul(a.c1, c2))));
  Fp2 ti = f2_inv(t);
  return {f2_mul(c0, ti), f2_mul(c1, ti), f2_mul(c2, ti)};
}

// ------------------------------------------------------------------ Fp12
HB_HD Fp12 f12_one() { return {f6_one(), f6_zero()}; }
HB_HD Fp12 f12_conj(const Fp12& a) { return {a.c0, f6_neg(a.c1)}; }

HB_HD Fp12 f12_mul(const Fp12& a, const Fp12& b) {
  Fp6 t0 = f6_mul(a.c0, b.c0);
  Fp6 t1 = f6_mul(a.c1, b.c1);
  Fp6 c1 = f6_sub(f6_sub(f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1)), t0), t1);
  return {f6_add(t0, f6_mul_v(t1)), c1};
}

// complex squaring: 2 Fp6 products
HB_HD Fp12 f12_sqr(const Fp12& a) {
  Fp6 t = f6_mul(a.c0, a.c1);
  Fp6 s = f6_mul(f6_add(a.c0, a.c1), f6_add(a.c0, f6_mul_v(a.c1)));
  return {f6_sub(f6_sub(s, t), f6_mul_v(t)), f6_add(t, t)};
}

// f * l with l = c0 + c1 w^2 + c4 w^3 (sparse slots 0, 1, 4)
HB_HD Fp12 f12_mul_014(const Fp12& f, const Fp2& c0, const Fp2& c1, const Fp2& c4) {
  Fp6 t0 = f6_mul_01(f.c0, c0, c1);
  Fp6 t1 = f6_mul_1(f.c1, c4);
  Fp6 s = f6_mul_01(f6_add(f.c0, f.c1), c0, f2_add(c1, c4));
  return {f6_add(t0, f6_mul_v(t1)), f6_sub(f6_sub(s, t0), t1)};
}

HB_HD Fp12 f12_inv(const Fp12& a) {
  Fp6 t = f6_sub(f6_mul(a.c0, a.c0), f6_mul_v(f6_mul(a.c1, a.c1)));
  Fp6 ti = f6_inv(t);
  return {f6_mul(a.c0, ti), f6_neg(f6_mul(a.c1, ti))};
}

// Frobenius maps: f = sum a_k w^k, (a0,a2,a4) = c0, (a1,a3,a5) = c1;
// f^(p^e) = sum (a_k or conj(a_k)) * gamma_{e,k} w^k.
#define HB_FROB_COEF(E, K) Fp2{fp_const(FROB##E##_##K##_C0), fp_const(FROB##E##_##K##_C1)}
HB_HD Fp12 f12_frob1(const Fp12& f) {
  Fp12 r;
  r.c0.c0 = f2_conj(f.c0.c0);
  r.c1.c0 = f2_mul(f2_conj(f.c1.c0), HB_FROB_COEF(1, 1));
  r.c0.c1 = f2_mul(f2_conj(f.c0.c1), HB_FROB_COEF(1, 2));
  r.c1.c1 = f2_mul(f2_conj(f.c1.c1), HB_FROB_COEF(1, 3));
  r.c0.c2 = f2_mul(f2_conj(f.c0.c2), HB_FROB_COEF(1, 4));
  r.c1.c2 = f2_mul(f2_conj(f.c1.c2), HB_FROB_COEF(1, 5));
  return r;
}

HB_HD Fp12 f12_frob2(const Fp12& f) {
  // gamma_{2,k} lie in Fp
  Fp12 r;
  r.c0.c0 = f.c0.c0;
  r.c1.c0 = f2_mul_fp(f.c1.c0, fp_const(FROB2_1_C0));
  r.c0.c1 = f2_mul_fp(f.c0.c1, fp_const(FROB2_2_C0));
  r.c1.c1 = f2_mul_fp(f.c1.c1, fp_const(FROB2_3_C0));
  r.c0.c2 = f2_mul_fp(f.c0.c2, fp_const(FROB2_4_C0));
  r.c1.c2 = f2_mul_fp(f.c1.c2, fp_const(FROB2_5_C0));
  return r;
}

// (x0 + x1 t)^2 with t^2 = xi
HB_HD void fp4_sqr(const Fp2& x0, const Fp2& x1, Fp2& r0, Fp2& r1) {
  Fp2 s0 = f2_sqr(x0);
  Fp2 s1 = f2_sqr(x1);
  r0 = f2_add(s0, f2_mul_xi(s1));
  r1 = f2_sub(f2_sub(f2_sqr(f2_add(x0, x1)), s0), s1);
}

// Granger-Scott squaring for elements of the cyclotomic subgroup (9 Fp2 squarings).
// View f = A + B w + C w^2 over Fp4 = Fp2[t], t = w^3:
//   A = a0 + a3 t, B = a1 + a4 t, C = a2 + a5 t
//   A' = 3A^2 - 2conj(A), B' = 3 t C^2 + 2 conj(B), C' = 3B^2 - 2conj(C).
HB_HD Fp12 f12_cyclo_sqr(const Fp12& f) {
  const Fp2& a0 = f.c0.c0; const Fp2& a2 = f.c0.c1; const Fp2& a4 = f.c0.c2;
  const Fp2& a1 = f.c1.c0; const Fp2& a3 = f.c1.c1; const Fp2& a5 = f.c1.c2;
  Fp2 A0, A1, B0, B1, C0, C1;
  fp4_sqr(a0, a3, A0, A1);
  fp4_sqr(a1, a4, B0, B1);
  fp4_sqr(a2, a5, C0, C1);
  Fp12 r;
  // 3z - 2y  = 2(z - y) + z ; 3z + 2y = 2(z + y) + z
  r.c0.c0 = f2_add(f2_dbl(f2_sub(A0, a0)), A0);
  r.c1.c1 = f2_add(f2_dbl(f2_add(A1, a3)), A1);
  Fp2 xC1 = f2_mul_xi(C1);
  r.c1.c0 = f2_add(f2_dbl(f2_add(xC1, a1)), xC1);
  r.c0.c2 = f2_add(f2_dbl(f2_sub(C0, a4)), C0);
  r.c0.c1 = f2_add(f2_dbl(f2_sub(B0, a2)), B0);
  r.c1.c2 = f2_add(f2_dbl(f2_add(B1, a5)), B1);
  return r;
}

HB_HD bool f12_is_one(const Fp12& f) {
  bool ok = fp_is_zero(fp_sub(f.c0.c0.c0, fp_one())) && fp_is_zero(f.c0.c0.c1);
  ok = ok && f2_is_zero(f.c0.c1) && f2_is_zero(f.c0.c2);
  ok = ok && f2_is_zero(f.c1.c0) && f2_is_zero(f.c1.c1) && f2_is_zero(f.c1.c2);
  return ok;
}

}  // namespace hb
