// Lane-OCTO extension of the lane-pair tower (pfp.hpp), namespace hbs: EIGHT lanes per pairing
// check (k_oct.hpp) for batches of a few thousand checks.
//
// An octo is four lane pairs (lanes 8i .. 8i+7; pair index o = lane bits 1..2), each laid out as in
// pfp.hpp.  As in the lane quad (qfp.hpp), every pair holds the check's whole state and each step's
// independent products are spread over the pairs -- here four per round -- after which all four
// results are gathered into every pair: pair o^1 through a DPP quad permutation ([2,3,0,1]), pairs
// o^2 and o^3 through ds_swizzle (lane ^ 4, LDS crossbar, no memory).  Rounds per operation (lane
// quad / lane pair in brackets): Fp12 squaring 3 (6 / 12 products), Fp12 product 5 (9 / 18), the
// two-line product 7 (12 / 23), cyclotomic squaring 3 (5 / 9), doubling step 3 (6 / 11), addition
// step 5 (7 / 13), line evaluation of both sides 1 (2 / 4).
// Formulas and value contracts are pfp.hpp's (pairing 0.14's, restated in oracle/c/bls_cpu.c).
#pragma once
#include "qfp.hpp"

namespace hbs {

HP_D int o_idx() { return (int)((threadIdx.x >> 1) & 3); }

// the value of the pair two positions away in the octo (lane ^ 4)
HP_D int32_t o_swz4(int32_t v) { return __builtin_amdgcn_ds_swizzle(v, 0x101F); }  // and 0x1F, xor 4
HP_D Fp o_swz4_fp(const Fp& a) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = o_swz4(a.l[i]);
  return r;
}

// x_o for this lane's pair o from four candidates
HP_D Fp o_sel(int o, const Fp& a0, const Fp& a1, const Fp& a2, const Fp& a3) {
  const bool b0 = (o & 1) != 0, b1 = (o & 2) != 0;
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const int32_t lo = b0 ? a1.l[i] : a0.l[i];
    const int32_t hi = b0 ? a3.l[i] : a2.l[i];
    r.l[i] = b1 ? hi : lo;
  }
  return r;
}

// pair o computed `mine` (value o of four); every pair gets r[0..3].  Butterfly: the pairs of each
// half of the octo first hold their half's two values in order (DPP quad swap), then exchange halves
// (ds_swizzle, lane ^ 4) -- 1 DPP + 1 swizzle + 6 selects per limb.
HP_D void o_gather(int o, const Fp& mine, Fp (&r)[4]) {
  const Fp m1 = dpp_fp<DPP_QSWAP>(mine);  // pair o ^ 1
  const bool b0 = (o & 1) != 0, b1 = (o & 2) != 0;
  Fp e, d;  // the values of pairs (o & 2) and (o & 2) | 1
#pragma unroll
  for (int i = 0; i < NL; i++) {
    e.l[i] = b0 ? m1.l[i] : mine.l[i];
    d.l[i] = b0 ? mine.l[i] : m1.l[i];
  }
  const Fp e2 = o_swz4_fp(e), d2 = o_swz4_fp(d);  // the other half's
#pragma unroll
  for (int i = 0; i < NL; i++) {
    r[0].l[i] = b1 ? e2.l[i] : e.l[i];
    r[1].l[i] = b1 ? d2.l[i] : d.l[i];
    r[2].l[i] = b1 ? e.l[i] : e2.l[i];
    r[3].l[i] = b1 ? d.l[i] : d2.l[i];
  }
}

// four independent Fp2 products x_k y_k (h_mul contracts), one product time
HP_D void h_mul4(const Fp (&x)[4], const Fp (&y)[4], Fp (&r)[4]) {
  const int o = o_idx();
  o_gather(o, h_mul(o_sel(o, x[0], x[1], x[2], x[3]), o_sel(o, y[0], y[1], y[2], y[3])), r);
}
HP_D void h_sqr4(const Fp (&x)[4], Fp (&r)[4]) {
  const int o = o_idx();
  o_gather(o, h_sqr(o_sel(o, x[0], x[1], x[2], x[3])), r);
}
HP_D void fp_mul4(const Fp (&x)[4], const Fp (&y)[4], Fp (&r)[4]) {
  const int o = o_idx();
  o_gather(o, fp_mul(o_sel(o, x[0], x[1], x[2], x[3]), o_sel(o, y[0], y[1], y[2], y[3])), r);
}

// Karatsuba of two Fp6 products (a b, c d) in three rounds of four
HP_D void h6_mul_pair_o(const H6& a, const H6& b, const H6& c, const H6& d, H6& ab, H6& cd) {
  Fp r[4];
  {
    const Fp x[4] = {a.c1, a.c2, c.c1, c.c2}, y[4] = {b.c1, b.c2, d.c1, d.c2};
    h_mul4(x, y, r);
  }
  const Fp av1 = r[0], av2 = r[1], cv1 = r[2], cv2 = r[3];
  {
    const Fp x[4] = {fp_addl(a.c1, a.c2), a.c0, fp_addl(c.c1, c.c2), c.c0};
    const Fp y[4] = {fp_add(b.c1, b.c2), b.c0, fp_add(d.c1, d.c2), d.c0};
    h_mul4(x, y, r);
  }
  const Fp av0 = r[1], cv0 = r[3];
  ab.c0 = fp_red_l(h_add_xi_l(av0, fp_sub2l(r[0], av1, av2)));
  cd.c0 = fp_red_l(h_add_xi_l(cv0, fp_sub2l(r[2], cv1, cv2)));
  {
    const Fp x[4] = {fp_addl(a.c0, a.c1), fp_addl(a.c0, a.c2), fp_addl(c.c0, c.c1), fp_addl(c.c0, c.c2)};
    const Fp y[4] = {fp_add(b.c0, b.c1), fp_add(b.c0, b.c2), fp_add(d.c0, d.c1), fp_add(d.c0, d.c2)};
    h_mul4(x, y, r);
  }
  ab.c1 = fp_red_l(h_add_xi_l(fp_sub2l(r[0], av0, av1), av2));
  ab.c2 = fp_red_l(fp_addl(fp_sub2l(r[1], av0, av2), av1));
  cd.c1 = fp_red_l(h_add_xi_l(fp_sub2l(r[2], cv0, cv1), cv2));
  cd.c2 = fp_red_l(fp_addl(fp_sub2l(r[3], cv0, cv2), cv1));
}

// one Fp6 product in two rounds (the second half-used)
HP_D H6 h6_mul_o(const H6& a, const H6& b) {
  Fp r[4];
  {
    const Fp x[4] = {a.c1, a.c2, fp_addl(a.c1, a.c2), a.c0};
    const Fp y[4] = {b.c1, b.c2, fp_add(b.c1, b.c2), b.c0};
    h_mul4(x, y, r);
  }
  const Fp v1 = r[0], v2 = r[1], t12 = r[2], v0 = r[3];
  {
    const Fp x[4] = {fp_addl(a.c0, a.c1), fp_addl(a.c0, a.c2), a.c0, a.c0};
    const Fp y[4] = {fp_add(b.c0, b.c1), fp_add(b.c0, b.c2), b.c0, b.c0};
    h_mul4(x, y, r);
  }
  return {fp_red_l(h_add_xi_l(v0, fp_sub2l(t12, v1, v2))), fp_red_l(h_add_xi_l(fp_sub2l(r[0], v0, v1), v2)),
          fp_red_l(fp_addl(fp_sub2l(r[1], v0, v2), v1))};
}

HP_D H12 h12_mul_o(const H12& a, const H12& b) {
  H6 t0, t1;
  h6_mul_pair_o(a.c0, b.c0, a.c1, b.c1, t0, t1);
  return h12_kcomb(t0, t1, h6_mul_o(h6_add(a.c0, a.c1), h6_add(b.c0, b.c1)));
}

HP_D H12 h12_sqr_o(const H12& a) {
  H6 t, s;
  h6_mul_pair_o(a.c0, a.c1, h6_add(a.c0, a.c1), h6_red(h6_add(a.c0, h6_mul_v(a.c1))), t, s);
  return {{fp_red_l(h_add_xi_l(fp_subl(s.c0, t.c0), fp_subl(fp_zero(), t.c2))), fp_red_l(fp_sub2l(s.c1, t.c1, t.c0)),
           fp_red_l(fp_sub2l(s.c2, t.c2, t.c1))},
          {fp_red_l(fp_addl(t.c0, t.c0)), fp_red_l(fp_addl(t.c1, t.c1)), fp_red_l(fp_addl(t.c2, t.c2))}};
}

// f * (la * lb): the six line products in two rounds, then t0 = f0 C0 beside t1 = f1 (0, c11, c12)
// (three rounds) and s (two)
HP_D H12 h12_mul_lines_o(const H12& f, const Fp& a0, const Fp& a1, const Fp& a4, const Fp& b0, const Fp& b1,
                         const Fp& b4) {
  Fp r[4];
  {
    const Fp x[4] = {a0, a1, a4, fp_addl(a0, a4)}, y[4] = {b0, b1, b4, fp_add(b0, b4)};
    h_mul4(x, y, r);
  }
  const Fp a0b0 = r[0], a1b1 = r[1], a4b4 = r[2], t04 = r[3];
  {
    const Fp x[4] = {fp_addl(a1, a4), fp_addl(a0, a1), a0, a0}, y[4] = {fp_add(b1, b4), fp_add(b0, b1), b0, b0};
    h_mul4(x, y, r);
  }
  const Fp c11 = fp_red_l(fp_sub2l(t04, a0b0, a4b4));
  const Fp c12 = fp_red_l(fp_sub2l(r[0], a1b1, a4b4));
  const H6 C0 = {fp_red_l(h_add_xi_l(a0b0, a4b4)), fp_red_l(fp_sub2l(r[1], a0b0, a1b1)), a1b1};
  H6 t0, t1;
  h6_mul_pair_o(f.c0, C0, f.c1, {h_zero(), c11, c12}, t0, t1);
  const H6 s = h6_mul_o(h6_add(f.c0, f.c1), {C0.c0, fp_add(C0.c1, c11), fp_add(C0.c2, c12)});
  return h12_kcomb(t0, t1, s);
}

// Granger-Scott squaring: nine squares in three rounds (the last one square, computed by every pair)
HP_D H12 h12_cyclo_sqr_o(const H12& f) {
  const Fp& a0 = f.c0.c0; const Fp& a2 = f.c0.c1; const Fp& a4 = f.c0.c2;
  const Fp& a1 = f.c1.c0; const Fp& a3 = f.c1.c1; const Fp& a5 = f.c1.c2;
  Fp r1[4], r2[4];
  {
    const Fp x[4] = {a0, a3, a1, a4};
    h_sqr4(x, r1);
  }
  {
    const Fp x[4] = {fp_add(a0, a3), fp_add(a1, a4), a2, a5};
    h_sqr4(x, r2);
  }
  const Fp s25 = h_sqr(fp_add(a2, a5));  // the ninth square on every pair (no exchange)
  const Fp &s0 = r1[0], &s3 = r1[1], &s1 = r1[2], &s4 = r1[3];
  const Fp &s03 = r2[0], &s14 = r2[1], &s2 = r2[2], &s5 = r2[3];
  H12 r;
  r.c0.c0 = fp_red_mk<3, -2>(h_add_xi_l(s0, s3), a0);
  r.c1.c1 = fp_red_mk<3, 2>(fp_sub2l(s03, s0, s3), a3);
  r.c0.c1 = fp_red_mk<3, -2>(h_add_xi_l(s1, s4), a2);
  r.c1.c2 = fp_red_mk<3, 2>(fp_sub2l(s14, s1, s4), a5);
  r.c0.c2 = fp_red_mk<3, -2>(h_add_xi_l(s2, s5), a4);
  r.c1.c0 = fp_red_mk<3, 2>(h_add_xi_l(fp_zero(), fp_sub2l(s25, s2, s5)), a1);
  return r;
}

HP_D H12 h12_inv_o(const H12& a) {
  H6 s0, s1;
  h6_mul_pair_o(a.c0, a.c0, a.c1, a.c1, s0, s1);
  const H6 t = h6_red(h6_sub(h6_red(s0), h6_red(h6_mul_v(h6_red(s1)))));
  const H6 ti = h6_red(h6_inv(t));
  H6 r0, r1;
  h6_mul_pair_o(a.c0, ti, a.c1, ti, r0, r1);
  return h12_red({r0, h6_neg(r1)});
}

HP_D H12 h12_frob1_o(const H12& f) {
  Fp r[4];
  const Fp x[4] = {h_conj(f.c1.c0), h_conj(f.c0.c1), h_conj(f.c1.c1), h_conj(f.c0.c2)};
  const Fp y[4] = {HP_FROB1(1), HP_FROB1(2), HP_FROB1(3), HP_FROB1(4)};
  h_mul4(x, y, r);
  H12 o;
  o.c0.c0 = h_conj(f.c0.c0);
  o.c1.c0 = r[0];
  o.c0.c1 = r[1];
  o.c1.c1 = r[2];
  o.c0.c2 = r[3];
  o.c1.c2 = h_mul(h_conj(f.c1.c2), HP_FROB1(5));
  return h12_red(o);
}
HP_D H12 h12_frob2_o(const H12& f) {
  Fp r[4];
  const Fp x[4] = {f.c1.c0, f.c0.c1, f.c1.c1, f.c0.c2};
  const Fp y[4] = {fp_const(hb::FROB2_1_C0), fp_const(hb::FROB2_2_C0), fp_const(hb::FROB2_3_C0),
                   fp_const(hb::FROB2_4_C0)};
  fp_mul4(x, y, r);
  H12 o;
  o.c0.c0 = f.c0.c0;
  o.c1.c0 = r[0];
  o.c0.c1 = r[1];
  o.c1.c1 = r[2];
  o.c0.c2 = r[3];
  o.c1.c2 = fp_mul(f.c1.c2, fp_const(hb::FROB2_5_C0));
  return o;
}

// doubling step (h_dbl_step): eleven products in three rounds
HP_D HLine h_dbl_step_o(HJac& T) {
  Fp r[4];
  {
    const Fp x[4] = {T.x, T.y, T.z, fp_add(T.y, T.z)};
    h_sqr4(x, r);
  }
  const Fp A = r[0], B = r[1], ZZ = r[2], YZ = r[3];
  const Fp E = fp_lin(3, A, 0, A);
  {
    const Fp xb = fp_add(T.x, B);
    const Fp x[4] = {B, xb, E, E}, y[4] = {B, xb, E, T.x};
    h_mul4(x, y, r);
  }
  const Fp C = r[0], XB = r[1], F = r[2], EX = r[3];
  const Fp D = fp_lin(2, fp_sub(fp_sub(XB, A), C), 0, C);
  const Fp Z3 = fp_sub(fp_sub(YZ, B), ZZ);
  const Fp X3 = fp_sub(F, fp_add(D, D));
  {
    const Fp x[4] = {E, Z3, E, E}, y[4] = {ZZ, ZZ, fp_sub(D, X3), ZZ};
    h_mul4(x, y, r);
  }
  HLine l;
  l.c0 = fp_reduce(fp_sub(EX, fp_add(B, B)));
  l.c1 = fp_neg(r[0]);
  l.c4 = r[1];
  T.y = fp_reduce(fp_sub(r[2], fp_lin(8, C, 0, C)));
  T.x = fp_reduce(X3);
  T.z = fp_reduce(Z3);
  return l;
}

// addition step (h_add_step): thirteen products in five rounds
HP_D HLine h_add_step_o(HJac& T, const Fp& xQ, const Fp& yQ) {
  Fp r[4];
  {
    const Fp x[4] = {T.z, yQ, T.z, T.z}, y[4] = {T.z, T.z, T.z, T.z};
    h_mul4(x, y, r);
  }
  const Fp Z1Z1 = r[0], YZ = r[1];
  {
    const Fp x[4] = {xQ, YZ, xQ, xQ}, y[4] = {Z1Z1, Z1Z1, Z1Z1, Z1Z1};
    h_mul4(x, y, r);
  }
  const Fp H = fp_sub(r[0], T.x);
  const Fp rr = fp_sub(r[1], T.y);
  {
    const Fp x[4] = {H, rr, T.z, H}, y[4] = {H, rr, H, H};
    h_mul4(x, y, r);
  }
  const Fp HH = r[0], R2 = r[1], Z3 = r[2];
  {
    const Fp x[4] = {H, T.x, yQ, rr}, y[4] = {HH, HH, Z3, xQ};
    h_mul4(x, y, r);
  }
  const Fp HHH = r[0], V = r[1], YZ3 = r[2], RX = r[3];
  const Fp X3 = fp_sub(fp_sub(R2, HHH), fp_add(V, V));
  {
    const Fp x[4] = {rr, T.y, rr, rr}, y[4] = {fp_sub(V, X3), HHH, fp_sub(V, X3), fp_sub(V, X3)};
    h_mul4(x, y, r);
  }
  HLine l;
  l.c0 = fp_reduce(fp_sub(RX, YZ3));
  l.c1 = fp_neg(rr);
  l.c4 = Z3;
  T.x = fp_reduce(X3);
  T.y = fp_reduce(fp_sub(r[0], r[1]));
  T.z = Z3;
  return l;
}

}  // namespace hbs
