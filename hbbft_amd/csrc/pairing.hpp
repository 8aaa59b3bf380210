// Optimal-ate pairing pieces for gfx950 (device side).
//
// Split into two phases so that no kernel has to hold f (Fp12) and T (G2 point) at once:
//   1. g2_prepare: walk T over the Miller loop of a G2 point Q and emit the 68 P-independent
//      line triples (c0, c1, c4) (63 doublings + 5 additions for |x| = 0xd201000000010000).
//      A doubling line through psi(T), scaled by 2YZ^3, is (3X^3 - 2Y^2) - 3X^2Z^2 xP w^2 + 2YZ^3 yP w^3;
//      an addition line through T and Q, scaled by Z1*H, is (r xQ - yQ Z3) - r xP w^2 + Z3 yP w^3.
//      (Fp2 scalings and the omitted vertical lines die in the final exponentiation.)
//   2. miller_fe: f = prod over pairs of lines evaluated at P (c1*xP, c4*yP), squared per bit; then
//      the final exponentiation; verdict = (f^e == 1).
// Formulas: tools/model_pairing.py (checked against the oracle).  The reference computes each
// pairing separately (threshold_crypto PEngine::pairing); verdicts agree
// because prod e(P_i,Q_i) == 1  <=>  e(P1,Q1) == e(-P2,Q2)^-1 ... == e(P2,Q2).
#pragma once
#include "tower.hpp"

namespace hb {

constexpr int MILLER_STEPS = 68;  // 63 doubling + 5 addition steps
constexpr int LINE_WORDS = 3 * 2 * NL;  // 84 words per line (c0, c1, c4 in Fp2)

struct G2Jac { Fp2 x, y, z; };
struct Line { Fp2 c0, c1, c4; };

HB_HD Line dbl_step(G2Jac& T) {
  Fp2 A = f2_sqr(T.x);
  Fp2 B = f2_sqr(T.y);
  Fp2 C = f2_sqr(B);
  Fp2 D = f2_dbl(f2_sub(f2_sub(f2_sqr(f2_add(T.x, B)), A), C));
  Fp2 E = f2_add(f2_dbl(A), A);
  Fp2 ZZ = f2_sqr(T.z);
  Line l;
  l.c0 = f2_sub(f2_mul(E, T.x), f2_dbl(B));
  l.c1 = f2_neg(f2_mul(E, ZZ));
  Fp2 Z3 = f2_sub(f2_sub(f2_sqr(f2_add(T.y, T.z)), B), ZZ);
  l.c4 = f2_mul(Z3, ZZ);
  Fp2 F = f2_sqr(E);
  Fp2 X3 = f2_sub(F, f2_dbl(D));
  Fp2 C8 = f2_dbl(f2_dbl(f2_dbl(C)));
  T.y = f2_sub(f2_mul(E, f2_sub(D, X3)), C8);
  T.x = X3;
  T.z = Z3;
  return l;
}

HB_HD Line add_step(G2Jac& T, const Fp2& xQ, const Fp2& yQ) {
  Fp2 Z1Z1 = f2_sqr(T.z);
  Fp2 U2 = f2_mul(xQ, Z1Z1);
  Fp2 S2 = f2_mul(f2_mul(yQ, T.z), Z1Z1);
  Fp2 H = f2_sub(U2, T.x);
  Fp2 r = f2_sub(S2, T.y);
  Fp2 HH = f2_sqr(H);
  Fp2 HHH = f2_mul(H, HH);
  Fp2 V = f2_mul(T.x, HH);
  Fp2 X3 = f2_sub(f2_sub(f2_sqr(r), HHH), f2_dbl(V));
  Fp2 Y3 = f2_sub(f2_mul(r, f2_sub(V, X3)), f2_mul(T.y, HHH));
  Fp2 Z3 = f2_mul(T.z, H);
  Line l;
  l.c0 = f2_sub(f2_mul(r, xQ), f2_mul(yQ, Z3));
  l.c1 = f2_neg(r);
  l.c4 = Z3;
  T.x = X3; T.y = Y3; T.z = Z3;
  return l;
}

// Line at P: c0 + (c1 xP) w^2 + (c4 yP) w^3, multiplied into f.
HB_HD Fp12 mul_line(const Fp12& f, const Line& l, const Fp& xP, const Fp& yP) {
  return f12_mul_014(f, l.c0, f2_mul_fp(l.c1, xP), f2_mul_fp(l.c4, yP));
}

// f^|x| for f in the cyclotomic subgroup; |x| = 0xd201000000010000 (plus one if PLUS1).
template <bool PLUS1>
HB_HD Fp12 cyclo_exp_abs_x(const Fp12& f) {
  Fp12 r = f;
  for (int i = 62; i >= 0; i--) {
    r = f12_cyclo_sqr(r);
    const bool bit = PLUS1 ? (((X_ABS + 1) >> i) & 1) : ((X_ABS >> i) & 1);
    if (bit) r = f12_mul(r, f);
  }
  return r;
}

// f^x (x < 0): conj(f^|x|);  f^(x-1) = conj(f^(|x|+1))
HB_HD Fp12 exp_by_x(const Fp12& f) { return f12_conj(cyclo_exp_abs_x<false>(f)); }
HB_HD Fp12 exp_by_x_minus_1(const Fp12& f) { return f12_conj(cyclo_exp_abs_x<true>(f)); }

// f^(3 (p^12-1)/r): easy part (p^6-1)(p^2+1), then 3(p^4-p^2+1)/r = (x-1)^2 (x+p)(x^2+p^2-1) + 3.
// Cubing is a bijection on mu_r, so the "== 1" verdict equals that of the plain exponentiation.
HB_HD Fp12 final_exp_x3(const Fp12& f) {
  Fp12 f1 = f12_mul(f12_conj(f), f12_inv(f));
  Fp12 f2 = f12_mul(f12_frob2(f1), f1);
  Fp12 a = exp_by_x_minus_1(exp_by_x_minus_1(f2));
  Fp12 b = f12_mul(exp_by_x(a), f12_frob1(a));
  Fp12 c = f12_mul(f12_mul(exp_by_x(exp_by_x(b)), f12_frob2(b)), f12_conj(b));
  return f12_mul(c, f12_mul(f12_cyclo_sqr(f2), f2));
}

}  // namespace hb
