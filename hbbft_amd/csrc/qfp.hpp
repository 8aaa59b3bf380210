// Lane-QUAD extension of the lane-pair tower (pfp.hpp), namespace hbs: FOUR lanes per pairing check
// for the mid-size batches (k_quad.hip).
//
// A quad is two lane pairs (lanes 4i, 4i+1 = pair 0; 4i+2, 4i+3 = pair 1), each laid out as in
// pfp.hpp (even lane c0, odd lane c1).  Both pairs hold the whole check state (replicated); every
// operation whose Fp2 / Fp6 products are independent runs them side by side -- pair 0 the first,
// pair 1 the second -- and the results cross over with one DPP quad permutation per limb
// ([2,3,0,1], the same component of the other pair), after which both pairs hold both results
// again.  Every pfp.hpp DPP pattern is pair-local ([1,0,3,2], [0,0,2,2], [1,1,3,3]), so the
// lane-pair products run unchanged on both pairs at once.
//
// The split is made where the formulas are widest:
//   h6_mul2      two whole Fp6 products (one per pair): complex squaring's t and s, Karatsuba's t0
//                and t1 -- the sums and reductions inside are split too, not repeated;
//   h6_mul_q     one Fp6 product as three dual Fp2 rounds (Karatsuba's third product);
//   h_mul2 / h_sqr2 / fp_mul2   single dual products (line products, doubling step, cyclotomic
//                squaring's nine squares in five rounds, line evaluation at P).
// A check's per-lane product count falls to ~0.55 of the lane pair's, so a batch of 16,384 checks
// (1,024 waves: one per SIMD) finishes in a little over half the lane-pair kernel's latency floor.
// Formulas and value contracts are pfp.hpp's (pairing 0.14's, restated in oracle/c/bls_cpu.c).
#pragma once
#include "pfp.hpp"

namespace hbs {

constexpr int DPP_QSWAP = 0x4E;  // quad_perm [2,3,0,1]: the other pair's lane with the same component

HP_D bool q_hi() { return (threadIdx.x & 2) != 0; }

HP_D Fp q_sel(bool hi, const Fp& a, const Fp& b) {  // hi ? b : a
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = hi ? b.l[i] : a.l[i];
  return r;
}
HP_D H6 q_sel6(bool hi, const H6& a, const H6& b) { return {q_sel(hi, a.c0, b.c0), q_sel(hi, a.c1, b.c1), q_sel(hi, a.c2, b.c2)}; }

// this pair computed `mine` (pair 0: value 0, pair 1: value 1); both pairs get (v0, v1)
HP_D void q_join(bool hi, const Fp& mine, Fp& v0, Fp& v1) {
  const Fp o = dpp_fp<DPP_QSWAP>(mine);
  v0 = q_sel(hi, mine, o);
  v1 = q_sel(hi, o, mine);
}
HP_D void q_join6(bool hi, const H6& mine, H6& v0, H6& v1) {
  q_join(hi, mine.c0, v0.c0, v1.c0);
  q_join(hi, mine.c1, v0.c1, v1.c1);
  q_join(hi, mine.c2, v0.c2, v1.c2);
}

// (x0 y0, x1 y1) in one product time (h_mul contracts per product)
HP_D void h_mul2(const Fp& x0, const Fp& y0, const Fp& x1, const Fp& y1, Fp& r0, Fp& r1) {
  const bool hi = q_hi();
  q_join(hi, h_mul(q_sel(hi, x0, x1), q_sel(hi, y0, y1)), r0, r1);
}
HP_D void h_sqr2(const Fp& a0, const Fp& a1, Fp& r0, Fp& r1) {
  const bool hi = q_hi();
  q_join(hi, h_sqr(q_sel(hi, a0, a1)), r0, r1);
}
HP_D void fp_mul2(const Fp& x0, const Fp& y0, const Fp& x1, const Fp& y1, Fp& r0, Fp& r1) {
  const bool hi = q_hi();
  q_join(hi, fp_mul(q_sel(hi, x0, x1), q_sel(hi, y0, y1)), r0, r1);
}
// (a0 b0, a1 b1) over Fp6: pair k runs pfp.hpp's h6_mul on its operands
HP_D void h6_mul2(const H6& a0, const H6& b0, const H6& a1, const H6& b1, H6& r0, H6& r1) {
  const bool hi = q_hi();
  q_join6(hi, h6_mul(q_sel6(hi, a0, a1), q_sel6(hi, b0, b1)), r0, r1);
}

// one Fp6 Karatsuba product (h6_mul) as three dual rounds: (v1, v2), (t12, v0), (t01, t02)
HP_D H6 h6_mul_q(const H6& a, const H6& b) {
  Fp v1, v2, t12, v0, t01, t02;
  h_mul2(a.c1, b.c1, a.c2, b.c2, v1, v2);
  h_mul2(fp_addl(a.c1, a.c2), fp_add(b.c1, b.c2), a.c0, b.c0, t12, v0);
  const Fp c0 = fp_red_l(h_add_xi_l(v0, fp_sub2l(t12, v1, v2)));
  h_mul2(fp_addl(a.c0, a.c1), fp_add(b.c0, b.c1), fp_addl(a.c0, a.c2), fp_add(b.c0, b.c2), t01, t02);
  const Fp c1 = fp_red_l(h_add_xi_l(fp_sub2l(t01, v0, v1), v2));
  const Fp c2 = fp_red_l(fp_addl(fp_sub2l(t02, v0, v2), v1));
  return {c0, c1, c2};
}

HP_D H12 h12_mul_q(const H12& a, const H12& b) {
  H6 t0, t1;
  h6_mul2(a.c0, b.c0, a.c1, b.c1, t0, t1);
  const H6 s = h6_mul_q(h6_add(a.c0, a.c1), h6_add(b.c0, b.c1));
  return h12_kcomb(t0, t1, s);
}

// complex squaring (h12_sqr): t = a0 a1 on pair 0, s = (a0 + a1)(a0 + v a1) on pair 1
HP_D H12 h12_sqr_q(const H12& a) {
  H6 t, s;
  h6_mul2(a.c0, a.c1, h6_add(a.c0, a.c1), h6_red(h6_add(a.c0, h6_mul_v(a.c1))), t, s);
  return {{fp_red_l(h_add_xi_l(fp_subl(s.c0, t.c0), fp_subl(fp_zero(), t.c2))), fp_red_l(fp_sub2l(s.c1, t.c1, t.c0)),
           fp_red_l(fp_sub2l(s.c2, t.c2, t.c1))},
          {fp_red_l(fp_addl(t.c0, t.c0)), fp_red_l(fp_addl(t.c1, t.c1)), fp_red_l(fp_addl(t.c2, t.c2))}};
}

// f * (la * lb) (h12_mul_lines): the six line products in three dual rounds; then t0 = f0 C0 on
// pair 0 beside t1 = f1 (0, c11, c12) on pair 1 (h6_mul with a zero coefficient: the product with
// it is the one wasted of the 17), and s split
HP_D H12 h12_mul_lines_q(const H12& f, const Fp& a0, const Fp& a1, const Fp& a4, const Fp& b0, const Fp& b1,
                         const Fp& b4) {
  Fp a0b0, a1b1, a4b4, t04, t14, t01;
  h_mul2(a0, b0, a1, b1, a0b0, a1b1);
  h_mul2(a4, b4, fp_addl(a0, a4), fp_add(b0, b4), a4b4, t04);
  h_mul2(fp_addl(a1, a4), fp_add(b1, b4), fp_addl(a0, a1), fp_add(b0, b1), t14, t01);
  const Fp c11 = fp_red_l(fp_sub2l(t04, a0b0, a4b4));
  const Fp c12 = fp_red_l(fp_sub2l(t14, a1b1, a4b4));
  const H6 C0 = {fp_red_l(h_add_xi_l(a0b0, a4b4)), fp_red_l(fp_sub2l(t01, a0b0, a1b1)), a1b1};
  H6 t0, t1;
  h6_mul2(f.c0, C0, f.c1, {h_zero(), c11, c12}, t0, t1);
  const H6 s = h6_mul_q(h6_add(f.c0, f.c1), {C0.c0, fp_add(C0.c1, c11), fp_add(C0.c2, c12)});
  return h12_kcomb(t0, t1, s);
}

// Granger-Scott squaring (h12_cyclo_sqr): nine Fp2 squares in five rounds
HP_D H12 h12_cyclo_sqr_q(const H12& f) {
  const Fp& a0 = f.c0.c0; const Fp& a2 = f.c0.c1; const Fp& a4 = f.c0.c2;
  const Fp& a1 = f.c1.c0; const Fp& a3 = f.c1.c1; const Fp& a5 = f.c1.c2;
  Fp s0, s3, s03, s1, s4, s14, s2, s5;
  h_sqr2(a0, a3, s0, s3);
  h_sqr2(fp_add(a0, a3), a1, s03, s1);
  h_sqr2(a4, fp_add(a1, a4), s4, s14);
  h_sqr2(a2, a5, s2, s5);
  const Fp s25 = h_sqr(fp_add(a2, a5));
  H12 r;
  r.c0.c0 = fp_red_mk<3, -2>(h_add_xi_l(s0, s3), a0);
  r.c1.c1 = fp_red_mk<3, 2>(fp_sub2l(s03, s0, s3), a3);
  r.c0.c1 = fp_red_mk<3, -2>(h_add_xi_l(s1, s4), a2);
  r.c1.c2 = fp_red_mk<3, 2>(fp_sub2l(s14, s1, s4), a5);
  r.c0.c2 = fp_red_mk<3, -2>(h_add_xi_l(s2, s5), a4);
  r.c1.c0 = fp_red_mk<3, 2>(h_add_xi_l(fp_zero(), fp_sub2l(s25, s2, s5)), a1);
  return r;
}

HP_D H12 h12_inv_q(const H12& a) {
  H6 s0, s1;
  h6_mul2(a.c0, a.c0, a.c1, a.c1, s0, s1);
  const H6 t = h6_red(h6_sub(h6_red(s0), h6_red(h6_mul_v(h6_red(s1)))));
  const H6 ti = h6_red(h6_inv(t));
  H6 r0, r1;
  h6_mul2(a.c0, ti, a.c1, ti, r0, r1);
  return h12_red({r0, h6_neg(r1)});
}

HP_D H12 h12_frob1_q(const H12& f) {
  H12 r;
  r.c0.c0 = h_conj(f.c0.c0);
  h_mul2(h_conj(f.c1.c0), HP_FROB1(1), h_conj(f.c0.c1), HP_FROB1(2), r.c1.c0, r.c0.c1);
  h_mul2(h_conj(f.c1.c1), HP_FROB1(3), h_conj(f.c0.c2), HP_FROB1(4), r.c1.c1, r.c0.c2);
  r.c1.c2 = h_mul(h_conj(f.c1.c2), HP_FROB1(5));
  return h12_red(r);
}
HP_D H12 h12_frob2_q(const H12& f) {
  H12 r;
  r.c0.c0 = f.c0.c0;
  fp_mul2(f.c1.c0, fp_const(hb::FROB2_1_C0), f.c0.c1, fp_const(hb::FROB2_2_C0), r.c1.c0, r.c0.c1);
  fp_mul2(f.c1.c1, fp_const(hb::FROB2_3_C0), f.c0.c2, fp_const(hb::FROB2_4_C0), r.c1.c1, r.c0.c2);
  r.c1.c2 = fp_mul(f.c1.c2, fp_const(hb::FROB2_5_C0));
  return r;
}

// doubling step (h_dbl_step): eleven products in six rounds
HP_D HLine h_dbl_step_q(HJac& T) {
  Fp A, B, C, ZZ, XB, YZ, EX, EZ, C4, F;
  h_sqr2(T.x, T.y, A, B);
  h_sqr2(B, T.z, C, ZZ);
  h_sqr2(fp_add(T.x, B), fp_add(T.y, T.z), XB, YZ);
  const Fp D = fp_lin(2, fp_sub(fp_sub(XB, A), C), 0, C);
  const Fp E = fp_lin(3, A, 0, A);
  h_mul2(E, T.x, E, ZZ, EX, EZ);
  HLine l;
  l.c0 = fp_sub(EX, fp_add(B, B));
  l.c1 = fp_neg(EZ);
  const Fp Z3 = fp_sub(fp_sub(YZ, B), ZZ);
  h_mul2(Z3, ZZ, E, E, C4, F);
  l.c4 = C4;
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

// addition step (h_add_step): thirteen products in seven rounds
HP_D HLine h_add_step_q(HJac& T, const Fp& xQ, const Fp& yQ) {
  Fp YZ, U2, S2, Z3, HH, R2, HHH, V, RV, YH, RX, YZ3;
  const Fp Z1Z1 = h_sqr(T.z);
  h_mul2(yQ, T.z, xQ, Z1Z1, YZ, U2);
  const Fp H = fp_sub(U2, T.x);
  h_mul2(YZ, Z1Z1, T.z, H, S2, Z3);
  const Fp r = fp_sub(S2, T.y);
  h_sqr2(H, r, HH, R2);
  h_mul2(H, HH, T.x, HH, HHH, V);
  const Fp X3 = fp_sub(fp_sub(R2, HHH), fp_add(V, V));
  h_mul2(r, fp_sub(V, X3), T.y, HHH, RV, YH);
  h_mul2(r, xQ, yQ, Z3, RX, YZ3);
  HLine l;
  l.c0 = fp_reduce(fp_sub(RX, YZ3));
  l.c1 = fp_neg(r);
  l.c4 = Z3;
  T.x = fp_reduce(X3);
  T.y = fp_reduce(fp_sub(RV, YH));
  T.z = Z3;
  return l;
}

}  // namespace hbs
