// G1 / G2 arithmetic for gfx950 in Jacobian coordinates (y^2 = x^3 + b, a = 0), generic over the
// coordinate field (Fp for G1, Fp2 for G2).  Formulas: dbl-2009-l, add-2007-bl, madd-2007-bl
// (explicit-formulas database), the same group law pairing 0.14 uses, so every result is the same
// group element the reference computes; outputs cross the boundary as canonical affine words.
// Infinity is Z == 0.  Exceptional additions (P == Q, P == -Q, O) are handled explicitly.
#pragma once
#include "points.hpp"
#include "tower.hpp"

namespace hb {

// ------------------------------------------------------------------ field overloads
HB_HD Fp fadd(const Fp& a, const Fp& b) { return fp_add(a, b); }
HB_HD Fp fsub(const Fp& a, const Fp& b) { return fp_sub(a, b); }
HB_HD Fp fdbl(const Fp& a) { return fp_dbl(a); }
HB_HD Fp fneg(const Fp& a) { return fp_neg(a); }
HB_HD Fp fmul(const Fp& a, const Fp& b) { return fp_mul(a, b); }
HB_HD Fp fsqr(const Fp& a) { return fp_sqr(a); }
HB_HD Fp finv(const Fp& a) { return fp_inv(a); }
HB_HD bool fisz(const Fp& a) { return fp_is_zero(a); }
HB_HD Fp fsel(bool c, const Fp& a, const Fp& b) { return fp_sel(c, a, b); }
HB_HD void fset_one(Fp& a) { a = fp_one(); }
HB_HD void fset_zero(Fp& a) { a = fp_zero(); }

HB_HD Fp2 fadd(const Fp2& a, const Fp2& b) { return f2_add(a, b); }
HB_HD Fp2 fsub(const Fp2& a, const Fp2& b) { return f2_sub(a, b); }
HB_HD Fp2 fdbl(const Fp2& a) { return f2_dbl(a); }
HB_HD Fp2 fneg(const Fp2& a) { return f2_neg(a); }
HB_HD Fp2 fmul(const Fp2& a, const Fp2& b) { return f2_mul(a, b); }
HB_HD Fp2 fsqr(const Fp2& a) { return f2_sqr(a); }
HB_HD Fp2 finv(const Fp2& a) { return f2_inv(a); }
HB_HD bool fisz(const Fp2& a) { return f2_is_zero(a); }
HB_HD Fp2 fsel(bool c, const Fp2& a, const Fp2& b) { return f2_sel(c, a, b); }
HB_HD void fset_one(Fp2& a) { a = f2_one(); }
HB_HD void fset_zero(Fp2& a) { a = f2_zero(); }

template <class F>
struct Jac {
  F x, y, z;
};

template <class F>
HB_HD Jac<F> jac_zero() {
  Jac<F> r;
  fset_one(r.x);
  fset_one(r.y);
  fset_zero(r.z);
  return r;
}
template <class F>
HB_HD bool jac_is_zero(const Jac<F>& p) { return fisz(p.z); }

template <class F>
HB_HD Jac<F> jac_from_affine(const F& x, const F& y, bool inf) {
  Jac<F> r;
  r.x = x;
  r.y = y;
  fset_one(r.z);
  if (inf) r = jac_zero<F>();
  return r;
}

// dbl-2009-l (O doubles to O since Z3 = 2 Y Z)
template <class F>
HB_HD Jac<F> jac_dbl(const Jac<F>& p) {
  const F A = fsqr(p.x);
  const F B = fsqr(p.y);
  const F C = fsqr(B);
  const F D = fdbl(fsub(fsub(fsqr(fadd(p.x, B)), A), C));
  const F E = fadd(fdbl(A), A);
  const F Fv = fsqr(E);
  Jac<F> r;
  r.x = fsub(Fv, fdbl(D));
  const F C8 = fdbl(fdbl(fdbl(C)));
  r.y = fsub(fmul(E, fsub(D, r.x)), C8);
  r.z = fdbl(fmul(p.y, p.z));
  return r;
}

// add-2007-bl: general Jacobian addition
template <class F>
HB_HD Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) {
  if (jac_is_zero(p)) return q;
  if (jac_is_zero(q)) return p;
  const F Z1Z1 = fsqr(p.z);
  const F Z2Z2 = fsqr(q.z);
  const F U1 = fmul(p.x, Z2Z2);
  const F U2 = fmul(q.x, Z1Z1);
  const F S1 = fmul(fmul(p.y, q.z), Z2Z2);
  const F S2 = fmul(fmul(q.y, p.z), Z1Z1);
  const F H = fsub(U2, U1);
  const F rr = fdbl(fsub(S2, S1));
  if (fisz(H)) {
    if (fisz(rr)) return jac_dbl(p);
    return jac_zero<F>();
  }
  const F I = fsqr(fdbl(H));
  const F J = fmul(H, I);
  const F V = fmul(U1, I);
  Jac<F> r;
  r.x = fsub(fsub(fsub(fsqr(rr), J), V), V);
  r.y = fsub(fmul(rr, fsub(V, r.x)), fdbl(fmul(S1, J)));
  r.z = fmul(fsub(fsub(fsqr(fadd(p.z, q.z)), Z1Z1), Z2Z2), H);
  return r;
}

// madd-2007-bl: p Jacobian + (x2, y2) affine (not infinity)
template <class F>
HB_HD Jac<F> jac_add_affine(const Jac<F>& p, const F& x2, const F& y2) {
  if (jac_is_zero(p)) return jac_from_affine(x2, y2, false);
  const F Z1Z1 = fsqr(p.z);
  const F U2 = fmul(x2, Z1Z1);
  const F S2 = fmul(fmul(y2, p.z), Z1Z1);
  const F H = fsub(U2, p.x);
  const F rr = fdbl(fsub(S2, p.y));
  if (fisz(H)) {
    if (fisz(rr)) return jac_dbl(p);
    return jac_zero<F>();
  }
  const F HH = fsqr(H);
  const F I = fdbl(fdbl(HH));
  const F J = fmul(H, I);
  const F V = fmul(p.x, I);
  Jac<F> r;
  r.x = fsub(fsub(fsub(fsqr(rr), J), V), V);
  r.y = fsub(fmul(rr, fsub(V, r.x)), fdbl(fmul(p.y, J)));
  r.z = fsub(fsub(fsqr(fadd(p.z, H)), Z1Z1), HH);
  return r;
}

// k * P for an affine P and a 256-bit scalar (8 LE words), double-and-add from the top set bit.
template <class F>
HB_HD Jac<F> jac_mul_affine(const F& x, const F& y, bool inf, const uint32_t* k) {
  Jac<F> acc = jac_zero<F>();
  if (inf) return acc;
  int top = 255;
  while (top >= 0 && !((k[top >> 5] >> (top & 31)) & 1)) top--;
  for (int i = top; i >= 0; i--) {
    acc = jac_dbl(acc);
    if ((k[i >> 5] >> (i & 31)) & 1) acc = jac_add_affine(acc, x, y);
  }
  return acc;
}

// k * P for a Jacobian P and a small scalar (used by Horner steps with x, y <= 2^32)
template <class F>
HB_HD Jac<F> jac_mul_small(const Jac<F>& p, uint32_t k) {
  Jac<F> acc = jac_zero<F>();
  if (k == 0) return acc;
  const int top = 31 - __builtin_clz(k);
  acc = p;
  for (int i = top - 1; i >= 0; i--) {
    acc = jac_dbl(acc);
    if ((k >> i) & 1) acc = jac_add(acc, p);
  }
  return acc;
}

template <class F>
HB_HD Jac<F> jac_neg(const Jac<F>& p) {
  Jac<F> r = p;
  r.y = fneg(p.y);
  return r;
}

// P == Q as group elements (cross-multiplied Jacobian coordinates)
template <class F>
HB_HD bool jac_eq(const Jac<F>& p, const Jac<F>& q) {
  const bool pz = jac_is_zero(p), qz = jac_is_zero(q);
  if (pz || qz) return pz && qz;
  const F Z1Z1 = fsqr(p.z);
  const F Z2Z2 = fsqr(q.z);
  if (!fisz(fsub(fmul(p.x, Z2Z2), fmul(q.x, Z1Z1)))) return false;
  return fisz(fsub(fmul(fmul(p.y, q.z), Z2Z2), fmul(fmul(q.y, p.z), Z1Z1)));
}

// ------------------------------------------------------------------ boundary words
HB_HD void g1_jac_to_words(const Jac<Fp>& p, uint32_t* w) {
  if (jac_is_zero(p)) {
    for (int i = 0; i < G1_WORDS; i++) w[i] = 0;
    return;
  }
  const Fp zi = fp_inv(p.z);
  const Fp zi2 = fp_sqr(zi);
  fp_to_words(fp_mul(p.x, zi2), w);
  fp_to_words(fp_mul(p.y, fp_mul(zi2, zi)), w + 12);
}
HB_HD void g2_jac_to_words(const Jac<Fp2>& p, uint32_t* w) {
  if (jac_is_zero(p)) {
    for (int i = 0; i < G2_WORDS; i++) w[i] = 0;
    return;
  }
  const Fp2 zi = f2_inv(p.z);
  const Fp2 zi2 = f2_sqr(zi);
  const Fp2 x = f2_mul(p.x, zi2);
  const Fp2 y = f2_mul(p.y, f2_mul(zi2, zi));
  fp_to_words(x.c0, w);
  fp_to_words(x.c1, w + 12);
  fp_to_words(y.c0, w + 24);
  fp_to_words(y.c1, w + 36);
}

}  // namespace hb
