// HBH_IMPL_QUAD: the lane-quad pairing-equality kernel (gfx950) for mid-size batches.
// (Kernel template; k_quad_g0/g1/g2.hip instantiate it per generator mode so the three ~3-minute
// compiles run in parallel.)
//
// The same check as k_pair.hip -- FE(f_{|x|,Q1}(P1) f_{|x|,Q2}(-P2)) == 1, pairing 0.14's Miller loop
// and final exponentiation -- on FOUR lanes per check: two lane pairs that hold the check's state
// side by side and split each step's independent products between them (qfp.hpp).  The lane-pair
// kernel's latency floor is one lane pair's whole check (10.6 ms); below ~32,768 checks it cannot
// fill the SIMDs, and the wave-per-check kernel's interpreter overhead caps it at ~0.8 M checks/s.
// Here a batch of 16,384 checks is 1,024 waves, one per SIMD, and a check takes ~0.55 of the lane
// pair's per-lane products (7.1 ms per batch of <= 16,384, profiles/r04/c8_sweep_wave_quad_pair.txt):
// the protocol's natural batch points (BA replays, remove_invalid_shares:
// src/binary_agreement/binary_agreement.rs:250-264, 507-519; src/threshold_decrypt.rs:204-217).
//
// One wave per SIMD is the design point: __launch_bounds__(256, 1) gives a lane up to 512 registers
// (256 VGPR + 256 AGPR), so the two pairs' operand sets of a dual product stay in registers.  The
// final exponentiation parks one Fp12 per lane in LDS (72 KiB per 256-lane workgroup), as k_pair.
#pragma once
#include "launch.hpp"
#include "pair_side.hpp"

namespace hbs {

template <bool PLUS1>
HP_D H12 q_exp_abs_x(const H12& base) {
  const uint64_t e = PLUS1 ? hb::X_ABS + 1 : hb::X_ABS;
  H12 r = base;
#pragma unroll 1
  for (int k = 62; k >= 0; k--) {
    r = h12_cyclo_sqr_q(r);
    if ((e >> k) & 1) r = h12_mul_q(r, base);
  }
  return r;
}
HP_D H12 q_exp_x(const H12& f) { return h12_conj(q_exp_abs_x<false>(f)); }
HP_D H12 q_exp_xm1(const H12& f) { return h12_conj(q_exp_abs_x<true>(f)); }

// k_pair.hip h_final_exp's chain with the lane-quad operations
HP_D H12 q_final_exp(const H12& f, uint32_t* __restrict__ stash) {
  const H12 f1 = h12_mul_q(h12_conj(f), h12_inv_q(f));
  const H12 g = h12_mul_q(h12_frob2_q(f1), f1);
  stash12(stash, g);
  H12 a = q_exp_xm1(q_exp_xm1(g));
  const H12 b = h12_mul_q(q_exp_x(a), h12_frob1_q(a));
  {
    const H12 gs = unstash12(stash);
    const H12 w = h12_mul_q(h12_mul_q(h12_frob2_q(b), h12_conj(b)), h12_mul_q(h12_cyclo_sqr_q(gs), gs));
    stash12(stash, w);
  }
  const H12 c = q_exp_x(q_exp_x(b));
  return h12_mul_q(c, unstash12(stash));
}

// GEN: 0 = both P read per check, 1 = P1 is the generator, 2 = P2 is the generator
template <bool W1, bool W2, int GEN>
// (two waves per SIMD -- 256 registers, 4,112 VGPR spills -- measured slower: 16,384 checks 9.29 vs
// 7.09 ms, 32,768 checks 15.5 vs 14.2 ms, profiles/r04/c10_ab.txt)
__global__ void __launch_bounds__(256, 1) k_quad_verify(PairArgs a) {
  extern __shared__ uint32_t stash_lds[];
  const int i = (int)((blockIdx.x * 256u + threadIdx.x) >> 2);
  if (i >= a.n) return;  // the four lanes of a quad leave together
  constexpr bool G1 = GEN == 1, G2 = GEN == 2;
  const bool neg2 = (a.flags & 1) != 0;
  SideState A, B;
  const bool ok1 = side_init<W1, G1>(a.s1, i, false, A);
  const bool ok2 = side_init<W2, G2>(a.s2, i, neg2, B);
  if (!ok1 || !ok2) {  // index out of range: reject, never read past a table
    if ((threadIdx.x & 3) == 0 && a.verdict) a.verdict[i] = 0;
    return;
  }
  H12 f = h12_one();
  int step = 0;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
    if (b != 62) f = h12_sqr_q(f);
    {
      const HLine la = side_line<W1, G1, true, true>(a.s1, A, step, false);
      const HLine lb = side_line<W2, G2, true, true>(a.s2, B, step, neg2);
      f = h12_mul_lines_q(f, la.c0, la.c1, la.c4, lb.c0, lb.c1, lb.c4);
    }
    step++;
    if ((hb::X_ABS >> b) & 1) {
      const HLine la = side_line<W1, G1, false, true>(a.s1, A, step, false);
      const HLine lb = side_line<W2, G2, false, true>(a.s2, B, step, neg2);
      f = h12_mul_lines_q(f, la.c0, la.c1, la.c4, lb.c0, lb.c1, lb.c4);
      step++;
    }
  }
  if (a.flags & 2) f = h12_conj(f);
  const H12 e = q_final_exp(f, stash_lds + threadIdx.x);
  if (a.value_out && !q_hi()) {
    uint32_t* o = a.value_out + (size_t)i * 144 + (lp_even() ? 0 : 12);
    fp_to_words(e.c0.c0, o + 0);
    fp_to_words(e.c0.c1, o + 24);
    fp_to_words(e.c0.c2, o + 48);
    fp_to_words(e.c1.c0, o + 72);
    fp_to_words(e.c1.c1, o + 96);
    fp_to_words(e.c1.c2, o + 120);
  }
  const bool one = h12_is_one(e);
  if ((threadIdx.x & 3) == 0 && a.verdict) a.verdict[i] = one ? 1 : 0;
}

}  // namespace hbs


namespace hbl {

// launch the four WALK / TABLE variants of one generator mode G
template <int G>
hipError_t quad_launch(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
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
  const dim3 grid((unsigned)((4 * (size_t)n + 255) / 256)), block(256);
  const size_t lds = (size_t)hbs::STASH_WORDS * 256 * 4;
  const bool w1 = d1.lines == nullptr, w2 = d2.lines == nullptr;
  if (w1 && w2)
    hipLaunchKernelGGL((hbs::k_quad_verify<true, true, G>), grid, block, lds, s, a);
  else if (w1)
    hipLaunchKernelGGL((hbs::k_quad_verify<true, false, G>), grid, block, lds, s, a);
  else if (w2)
    hipLaunchKernelGGL((hbs::k_quad_verify<false, true, G>), grid, block, lds, s, a);
  else
    hipLaunchKernelGGL((hbs::k_quad_verify<false, false, G>), grid, block, lds, s, a);
  return hipGetLastError();
}

// one per translation unit (k_quad_g0/g1/g2.hip)
hipError_t quad_verify_g0(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
                          uint8_t* verdict, uint32_t* value_out);
hipError_t quad_verify_g1(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
                          uint8_t* verdict, uint32_t* value_out);
hipError_t quad_verify_g2(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
                          uint8_t* verdict, uint32_t* value_out);

}  // namespace hbl
