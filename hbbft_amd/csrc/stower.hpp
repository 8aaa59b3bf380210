// Fp6 / Fp12 on the signed-limb Fp2 of sfp.hpp, for the one-thread-per-check pairing (k_ts_*.hip).
//   Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v), xi = 1 + u (pairing 0.14's tower).
// Value contracts (|.| per Fp component, all normalised):
//   Fp2 products (t2_*) inputs < 8p -> outputs < 2.5p      (sfp.hpp (M))
//   f6_mul / f6_mul_01 / f6_mul_1 inputs < 4p -> outputs < 18p
//   Fp12 values between operations: reduced, |.| < 2p (f12_red after every operation)
#pragma once
#include "sfp.hpp"

namespace hbs {

struct Fp6 { Fp2 c0, c1, c2; };
struct Fp12 { Fp6 c0, c1; };

// Fp2 products.  All go through the single non-inlined fp_mul: a paired variant (two independent
// products interleaved column by column, ILP 2) measured 77 vs 62 G Fp-mul/s in isolation but made
// the pairing 1.6x slower -- the larger call footprint doubled the caller's spills.
HS_HD Fp2 t2_mul(const Fp2& a, const Fp2& b) { return f2_mul(a, b); }
HS_HD void t2_mul_pair(const Fp2& a, const Fp2& b, const Fp2& c, const Fp2& d, Fp2& r, Fp2& s) {
  r = f2_mul(a, b);
  s = f2_mul(c, d);
}
HS_HD Fp2 t2_sqr(const Fp2& a) { return f2_sqr(a); }
HS_HD void t2_sqr_pair(const Fp2& a, const Fp2& b, Fp2& r, Fp2& s) {
  r = f2_sqr(a);
  s = f2_sqr(b);
}
HS_HD Fp2 t2_mul_fp(const Fp2& a, const Fp& k) { return f2_mul_fp(a, k); }

HS_HD Fp6 f6_zero() { return {f2_zero(), f2_zero(), f2_zero()}; }
HS_HD Fp6 f6_one() { return {f2_one(), f2_zero(), f2_zero()}; }
HS_HD Fp6 f6_add(const Fp6& a, const Fp6& b) { return {f2_add(a.c0, b.c0), f2_add(a.c1, b.c1), f2_add(a.c2, b.c2)}; }
HS_HD Fp6 f6_sub(const Fp6& a, const Fp6& b) { return {f2_sub(a.c0, b.c0), f2_sub(a.c1, b.c1), f2_sub(a.c2, b.c2)}; }
HS_HD Fp6 f6_neg(const Fp6& a) { return {f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; }
HS_HD Fp6 f6_red(const Fp6& a) { return {f2_red(a.c0), f2_red(a.c1), f2_red(a.c2)}; }
HS_HD Fp6 f6_mul_v(const Fp6& a) { return {f2_mul_xi(a.c2), a.c0, a.c1}; }

// Karatsuba, inputs < 4p
HS_HD Fp6 f6_mul(const Fp6& a, const Fp6& b) {
  Fp2 v0, v1, v2, t0, t1, t2;
  t2_mul_pair(a.c0, b.c0, a.c1, b.c1, v0, v1);
  t2_mul_pair(a.c2, b.c2, f2_add(a.c1, a.c2), f2_add(b.c1, b.c2), v2, t0);
  t2_mul_pair(f2_add(a.c0, a.c1), f2_add(b.c0, b.c1), f2_add(a.c0, a.c2), f2_add(b.c0, b.c2), t1, t2);
  t0 = f2_sub(f2_sub(t0, v1), v2);
  t1 = f2_sub(f2_sub(t1, v0), v1);
  t2 = f2_sub(f2_sub(t2, v0), v2);
  return {f2_add(v0, f2_mul_xi(t0)), f2_add(t1, f2_mul_xi(v2)), f2_add(t2, v1)};
}
// x (a + b v); x < 4p, a, b < 4p
HS_HD Fp6 f6_mul_01(const Fp6& x, const Fp2& a, const Fp2& b) {
  Fp2 t0, t1, u, w;
  t2_mul_pair(x.c0, a, x.c1, b, t0, t1);
  t2_mul_pair(x.c2, b, x.c2, a, u, w);
  const Fp2 s = t2_mul(f2_add(x.c0, x.c1), f2_add(a, b));
  return {f2_add(t0, f2_mul_xi(u)), f2_sub(f2_sub(s, t0), t1), f2_add(t1, w)};
}
// x (b v)
HS_HD Fp6 f6_mul_1(const Fp6& x, const Fp2& b) {
  Fp2 r0, r1;
  t2_mul_pair(x.c2, b, x.c0, b, r0, r1);
  return {f2_mul_xi(r0), r1, t2_mul(x.c1, b)};
}
HS_HD Fp6 f6_inv(const Fp6& a) {
  const Fp2 c0 = f2_red(f2_sub(t2_sqr(a.c0), f2_mul_xi(t2_mul(a.c1, a.c2))));
  const Fp2 c1 = f2_red(f2_sub(f2_mul_xi(t2_sqr(a.c2)), t2_mul(a.c0, a.c1)));
  const Fp2 c2 = f2_red(f2_sub(t2_sqr(a.c1), t2_mul(a.c0, a.c2)));
  const Fp2 t = f2_red(f2_add(t2_mul(a.c0, c0), f2_mul_xi(f2_add(t2_mul(a.c2, c1), t2_mul(a.c1, c2)))));
  const Fp2 ti = f2_red(f2_inv(t));
  return {t2_mul(c0, ti), t2_mul(c1, ti), t2_mul(c2, ti)};
}

HS_HD Fp12 f12_one() { return {f6_one(), f6_zero()}; }
HS_HD Fp12 f12_conj(const Fp12& a) { return {a.c0, f6_neg(a.c1)}; }
HS_HD Fp12 f12_red(const Fp12& a) { return {f6_red(a.c0), f6_red(a.c1)}; }

// inputs reduced; output reduced
HS_HD Fp12 f12_mul(const Fp12& a, const Fp12& b) {
  const Fp6 t0 = f6_mul(a.c0, b.c0);
  const Fp6 t1 = f6_mul(a.c1, b.c1);
  const Fp6 s = f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1));
  return f12_red({f6_add(t0, f6_mul_v(t1)), f6_sub(f6_sub(s, t0), t1)});
}
// complex squaring; (c0 + v c1) is reduced to meet f6_mul's < 4p contract
HS_HD Fp12 f12_sqr(const Fp12& a) {
  const Fp6 t = f6_red(f6_mul(a.c0, a.c1));
  const Fp6 s = f6_mul(f6_add(a.c0, a.c1), f6_red(f6_add(a.c0, f6_mul_v(a.c1))));
  return f12_red({f6_sub(f6_sub(s, t), f6_mul_v(t)), f6_add(t, t)});
}
// f (c0 + c1 w^2 + c4 w^3); c0, c1, c4 < 2p
HS_HD Fp12 f12_mul_014(const Fp12& f, const Fp2& c0, const Fp2& c1, const Fp2& c4) {
  // sums first: f.c0 and f.c1 then die at their last product (lower peak register pressure)
  const Fp6 fs = f6_add(f.c0, f.c1);
  const Fp2 c14 = f2_add(c1, c4);
  const Fp6 t0 = f6_red(f6_mul_01(f.c0, c0, c1));
  const Fp6 t1 = f6_red(f6_mul_1(f.c1, c4));
  const Fp6 s = f6_red(f6_mul_01(fs, c0, c14));
  return f12_red({f6_add(t0, f6_mul_v(t1)), f6_sub(f6_sub(s, t0), t1)});
}
HS_HD Fp12 f12_inv(const Fp12& a) {
  const Fp6 t = f6_red(f6_sub(f6_red(f6_mul(a.c0, a.c0)), f6_red(f6_mul_v(f6_red(f6_mul(a.c1, a.c1))))));
  const Fp6 ti = f6_red(f6_inv(t));
  return f12_red({f6_mul(a.c0, ti), f6_neg(f6_mul(a.c1, ti))});
}

#define HS_FROB(E, K) Fp2{fp_const(hb::FROB##E##_##K##_C0), fp_const(hb::FROB##E##_##K##_C1)}
HS_HD Fp12 f12_frob1(const Fp12& f) {
  Fp12 r;
  r.c0.c0 = f2_conj(f.c0.c0);
  t2_mul_pair(f2_conj(f.c1.c0), HS_FROB(1, 1), f2_conj(f.c0.c1), HS_FROB(1, 2), r.c1.c0, r.c0.c1);
  t2_mul_pair(f2_conj(f.c1.c1), HS_FROB(1, 3), f2_conj(f.c0.c2), HS_FROB(1, 4), r.c1.c1, r.c0.c2);
  r.c1.c2 = t2_mul(f2_conj(f.c1.c2), HS_FROB(1, 5));
  return f12_red(r);
}
HS_HD Fp12 f12_frob2(const Fp12& f) {
  Fp12 r;
  r.c0.c0 = f.c0.c0;
  r.c1.c0 = t2_mul_fp(f.c1.c0, fp_const(hb::FROB2_1_C0));
  r.c0.c1 = t2_mul_fp(f.c0.c1, fp_const(hb::FROB2_2_C0));
  r.c1.c1 = t2_mul_fp(f.c1.c1, fp_const(hb::FROB2_3_C0));
  r.c0.c2 = t2_mul_fp(f.c0.c2, fp_const(hb::FROB2_4_C0));
  r.c1.c2 = t2_mul_fp(f.c1.c2, fp_const(hb::FROB2_5_C0));
  return r;
}

// Granger-Scott cyclotomic squaring (input reduced, output reduced): three Fp4 squarings
// (x0 + x1 y)^2 = (x0^2 + xi x1^2) + ((x0 + x1)^2 - x0^2 - x1^2) y over (a0, a3), (a1, a4), (a2, a5)
HS_HD Fp12 f12_cyclo_sqr(const Fp12& f) {
  const Fp2& a0 = f.c0.c0; const Fp2& a2 = f.c0.c1; const Fp2& a4 = f.c0.c2;
  const Fp2& a1 = f.c1.c0; const Fp2& a3 = f.c1.c1; const Fp2& a5 = f.c1.c2;
  Fp2 s0, s3, s03, s1, s4, s14, s2, s5;
  t2_sqr_pair(a0, a3, s0, s3);
  t2_sqr_pair(f2_add(a0, a3), a1, s03, s1);
  t2_sqr_pair(a4, f2_add(a1, a4), s4, s14);
  t2_sqr_pair(a2, a5, s2, s5);
  const Fp2 s25 = t2_sqr(f2_add(a2, a5));
  const Fp2 A0 = f2_add(s0, f2_mul_xi(s3)), A1 = f2_sub(f2_sub(s03, s0), s3);
  const Fp2 B0 = f2_add(s1, f2_mul_xi(s4)), B1 = f2_sub(f2_sub(s14, s1), s4);
  const Fp2 C0 = f2_add(s2, f2_mul_xi(s5)), C1 = f2_sub(f2_sub(s25, s2), s5);
  const Fp2 xC1 = f2_mul_xi(C1);
  Fp12 r;
  r.c0.c0 = f2_lin(3, A0, -2, a0);
  r.c1.c1 = f2_lin(3, A1, 2, a3);
  r.c1.c0 = f2_lin(3, xC1, 2, a1);
  r.c0.c2 = f2_lin(3, C0, -2, a4);
  r.c0.c1 = f2_lin(3, B0, -2, a2);
  r.c1.c2 = f2_lin(3, B1, 2, a5);
  return f12_red(r);
}

HS_HD bool f12_is_one(const Fp12& f) {
  bool ok = fp_is_zero(fp_sub(f.c0.c0.c0, fp_one())) && fp_is_zero(f.c0.c0.c1);
  ok = ok && f2_is_zero(f.c0.c1) && f2_is_zero(f.c0.c2);
  ok = ok && f2_is_zero(f.c1.c0) && f2_is_zero(f.c1.c1) && f2_is_zero(f.c1.c2);
  return ok;
}

}  // namespace hbs
