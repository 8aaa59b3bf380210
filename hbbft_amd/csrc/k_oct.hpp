// HBH_IMPL_OCT: the lane-octo pairing-equality kernel (gfx950) for batches of a few thousand checks.
//
// The check of k_pair.hip / k_quad.hpp on EIGHT lanes: four lane pairs holding the check's state side
// by side, each step's independent products spread four per round (ofp.hpp).  A check's latency is
// ~0.6 of the lane quad's, and 8,192 checks are 1,024 waves (one per SIMD), so it serves the band
// between the wave-per-check kernel (interpreter-bound above ~4,000 checks) and the lane quad.
// (Kernel template; k_oct_g0/g1/g2.hip instantiate it per generator mode.)
#pragma once
#include "launch.hpp"
#include "pair_side.hpp"
#include "ofp.hpp"

namespace hbs {

template <bool PLUS1>
HP_D H12 o_exp_abs_x(const H12& base) {
  const uint64_t e = PLUS1 ? hb::X_ABS + 1 : hb::X_ABS;
  H12 r = base;
#pragma unroll 1
  for (int k = 62; k >= 0; k--) {
    r = h12_cyclo_sqr_o(r);
    if ((e >> k) & 1) r = h12_mul_o(r, base);
  }
  return r;
}
HP_D H12 o_exp_x(const H12& f) { return h12_conj(o_exp_abs_x<false>(f)); }
HP_D H12 o_exp_xm1(const H12& f) { return h12_conj(o_exp_abs_x<true>(f)); }

// k_pair.hip h_final_exp's chain with the lane-octo operations
HP_D H12 o_final_exp(const H12& f, uint32_t* __restrict__ stash) {
  const H12 f1 = h12_mul_o(h12_conj(f), h12_inv_o(f));
  const H12 g = h12_mul_o(h12_frob2_o(f1), f1);
  stash12(stash, g);
  H12 a = o_exp_xm1(o_exp_xm1(g));
  const H12 b = h12_mul_o(o_exp_x(a), h12_frob1_o(a));
  {
    const H12 gs = unstash12(stash);
    const H12 w = h12_mul_o(h12_mul_o(h12_frob2_o(b), h12_conj(b)), h12_mul_o(h12_cyclo_sqr_o(gs), gs));
    stash12(stash, w);
  }
  const H12 c = o_exp_x(o_exp_x(b));
  return h12_mul_o(c, unstash12(stash));
}

// a side's raw line of this step: the walk of T (WALK) or the table entry (TABLE)
template <bool WALK, bool DBL>
HP_D HLine oct_raw_line(const PairSide& s, SideState& st, int step) {
  if (WALK) {
    if (DBL) return h_dbl_step_o(st.T);
    Fp xQ, yQ;
    side_q(s, st, xQ, yQ);
    return h_add_step_o(st.T, xQ, yQ);
  }
  HLine l;
  const int4* p = s.lines + ((size_t)(st.q * PAIR_STEPS + step) * 2 + (lp_even() ? 0 : 1)) * PL_Q4;
  int32_t w[4 * PL_Q4];
#pragma unroll
  for (int k = 0; k < PL_Q4; k++) {
    const int4 v = p[k];
    w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
  }
#pragma unroll
  for (int j = 0; j < NL; j++) {
    l.c0.l[j] = w[j];
    l.c1.l[j] = w[NL + j];
    l.c4.l[j] = w[2 * NL + j];
  }
  return l;
}

// both sides' lines of this step evaluated at their P in one round of four Fp products
template <bool W1, bool W2, bool G1, bool G2, bool DBL>
HP_D void oct_lines(const PairArgs& a, SideState& A, SideState& B, int step, bool neg2, HLine& la, HLine& lb) {
  const HLine ra = oct_raw_line<W1, DBL>(a.s1, A, step);
  const HLine rb = oct_raw_line<W2, DBL>(a.s2, B, step);
  Fp r[4];
  const Fp x[4] = {ra.c1, ra.c4, rb.c1, rb.c4};
  const Fp y[4] = {side_xP<G1>(A), side_yP<G1>(A, false), side_xP<G2>(B), side_yP<G2>(B, neg2)};
  fp_mul4(x, y, r);
  la.c0 = A.act ? ra.c0 : h_one();
  la.c1 = A.act ? r[0] : fp_zero();
  la.c4 = A.act ? r[1] : fp_zero();
  lb.c0 = B.act ? rb.c0 : h_one();
  lb.c1 = B.act ? r[2] : fp_zero();
  lb.c4 = B.act ? r[3] : fp_zero();
}

// GEN: 0 = both P read per check, 1 = P1 is the generator, 2 = P2 is the generator
template <bool W1, bool W2, int GEN>
// (one wave per SIMD: the four pairs' gather buffers are live across every round)
__global__ void __launch_bounds__(256, 1) k_oct_verify(PairArgs a) {
  extern __shared__ uint32_t stash_lds[];
  const int i = (int)((blockIdx.x * 256u + threadIdx.x) >> 3);
  if (i >= a.n) return;  // the eight lanes of an octo leave together
  constexpr bool G1 = GEN == 1, G2 = GEN == 2;
  const bool neg2 = (a.flags & 1) != 0;
  SideState A, B;
  const bool ok1 = side_init<W1, G1>(a.s1, i, false, A);
  const bool ok2 = side_init<W2, G2>(a.s2, i, neg2, B);
  if (!ok1 || !ok2) {  // index out of range: reject, never read past a table
    if ((threadIdx.x & 7) == 0 && a.verdict) a.verdict[i] = 0;
    return;
  }
  H12 f = h12_one();
  int step = 0;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
    if (b != 62) f = h12_sqr_o(f);
    {
      HLine la, lb;
      oct_lines<W1, W2, G1, G2, true>(a, A, B, step, neg2, la, lb);
      f = h12_mul_lines_o(f, la.c0, la.c1, la.c4, lb.c0, lb.c1, lb.c4);
    }
    step++;
    if ((hb::X_ABS >> b) & 1) {
      HLine la, lb;
      oct_lines<W1, W2, G1, G2, false>(a, A, B, step, neg2, la, lb);
      f = h12_mul_lines_o(f, la.c0, la.c1, la.c4, lb.c0, lb.c1, lb.c4);
      step++;
    }
  }
  if (a.flags & 2) f = h12_conj(f);
  const H12 e = o_final_exp(f, stash_lds + threadIdx.x);
  if (a.value_out && o_idx() == 0) {
    uint32_t* o = a.value_out + (size_t)i * 144 + (lp_even() ? 0 : 12);
    fp_to_words(e.c0.c0, o + 0);
    fp_to_words(e.c0.c1, o + 24);
    fp_to_words(e.c0.c2, o + 48);
    fp_to_words(e.c1.c0, o + 72);
    fp_to_words(e.c1.c1, o + 96);
    fp_to_words(e.c1.c2, o + 120);
  }
  const bool one = h12_is_one(e);
  if ((threadIdx.x & 7) == 0 && a.verdict) a.verdict[i] = one ? 1 : 0;
}

}  // namespace hbs


namespace hbl {

// launch the four WALK / TABLE variants of one generator mode G
template <int G>
hipError_t oct_launch(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
                       uint8_t* verdict, uint32_t* value_out) {
  hbs::PairArgs a;
  a.n = n;
  const PairSideDesc* d[2] = {&d1, &d2};
  hbs::PairSide* o[2] = {&a.s1, &a.s2};
  for (int k = 0; k < 2; k++) {
    o[k]->p = (const uint32_t*)d[k]->p;
    o[k]->q = (const uint32_t*)d[k]->q;
    o[k]->lines = (const int4*)d[k]->lines;
    o[k]->qinf = d[k]->qinf;
    o[k]->idx = d[k]->idx;
    o[k]->nq = (uint32_t)d[k]->nq;
  }
  a.flags = flags;
  a.verdict = verdict;
  a.value_out = value_out;
  const dim3 grid((unsigned)((8 * (size_t)n + 255) / 256)), block(256);
  const size_t lds = (size_t)hbs::STASH_WORDS * 256 * 4;
  const bool w1 = d1.lines == nullptr, w2 = d2.lines == nullptr;
  if (w1 && w2)
    hipLaunchKernelGGL((hbs::k_oct_verify<true, true, G>), grid, block, lds, s, a);
  else if (w1)
    hipLaunchKernelGGL((hbs::k_oct_verify<true, false, G>), grid, block, lds, s, a);
  else if (w2)
    hipLaunchKernelGGL((hbs::k_oct_verify<false, true, G>), grid, block, lds, s, a);
  else
    hipLaunchKernelGGL((hbs::k_oct_verify<false, false, G>), grid, block, lds, s, a);
  return hipGetLastError();
}

// one per translation unit (k_oct_g0/g1/g2.hip)
hipError_t oct_verify_g0(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
                          uint8_t* verdict, uint32_t* value_out);
hipError_t oct_verify_g1(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
                          uint8_t* verdict, uint32_t* value_out);
hipError_t oct_verify_g2(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
                          uint8_t* verdict, uint32_t* value_out);

}  // namespace hbl
