// HBH_IMPL_PAIR: the fused lane-pair pairing-equality kernel (gfx950).
//
// verdict[i] = e(P1_i, Q1_i) == e(P2_i, Q2_i), computed as FE(f_{|x|,Q1}(P1) f_{|x|,Q2}(-P2)) == 1 with
// one 2-pair multi-Miller loop and one final exponentiation per check -- SURVEY §8(d)'s unit of work,
// pairing 0.14's Miller loop and final exponentiation (oracle/c/bls_cpu.c miller_loop /
// final_exponentiation restate them) on the lane-pair tower of
// pfp.hpp: TWO lanes per check, so a 65,536-check batch is 2,048 waves = two waves per SIMD.
//
// Each G2 side is one of
//   TABLE: Q is shared by many checks (H per document, W / H_uv per ciphertext): its 68 lines are
//          computed once by k_pair_prep into a table that the checks of a wave read as broadcasts;
//   WALK : Q is per check (sigma_i, or both sides of Ciphertext::verify): T walks inside the Miller
//          loop in registers -- no per-share line table ever reaches HBM.
// The whole check is one kernel: the Fp12 state never leaves the CU.  During the final
// exponentiation one Fp12 (6 components per lane, packed to 72 words) is parked in LDS:
// 256 lanes x 288 B = 72 KiB per workgroup, two workgroups per CU.
#define HS_MULFN static __device__ __noinline__
#include "launch.hpp"
#include "pfp.hpp"

namespace hbs {

constexpr int PAIR_STEPS = 68;   // 63 doubling + 5 addition steps of |x|
constexpr int PL_Q4 = 11;        // 16-byte chunks per (line, lane component): c0, c1, c4 = 42 words (+2 pad)
constexpr int STASH_WORDS = 72;  // 6 packed Fp per lane

// ---------------------------------------------------------------- LDS stash (6 components)
// component reduced to [0, 2p) (< 2^382) and packed 14 x 28 -> 12 x 32 bits; Montgomery form kept
HP_D void stash_fp(uint32_t* __restrict__ s, const Fp& a) {
  const Fp r = fp_reduce(a);
  Fp rp = fp_addl(r, fp_const(P_L));
  fp_norm(rp);
  const Fp c = (r.l[NL - 1] < 0) ? rp : r;
#pragma unroll
  for (int w = 0; w < 12; w++) {
    const int bit = 32 * w, li = bit / 28, sh = bit % 28;
    uint64_t v = (uint64_t)(uint32_t)c.l[li] >> sh;
    if (li + 1 < NL) v |= (uint64_t)(uint32_t)c.l[li + 1] << (28 - sh);
    if (li + 2 < NL) v |= (uint64_t)(uint32_t)c.l[li + 2] << (56 - sh);
    s[w * 256] = (uint32_t)v;
  }
}
HP_D Fp unstash_fp(const uint32_t* __restrict__ s) {
  uint32_t w[12];
#pragma unroll
  for (int k = 0; k < 12; k++) w[k] = s[k * 256];
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const int bit = 28 * i, wi = bit >> 5, sh = bit & 31;
    uint64_t v = w[wi];
    if (wi + 1 < 12) v |= (uint64_t)w[wi + 1] << 32;
    r.l[i] = (int32_t)((uint32_t)(v >> sh) & (uint32_t)MASK28);
  }
  return r;
}
// s = this lane's column of the workgroup's stash (word k of lane l at stash[k * 256 + l])
HP_D void stash12(uint32_t* __restrict__ s, const H12& f) {
  stash_fp(s + 0 * 12 * 256, f.c0.c0);
  stash_fp(s + 1 * 12 * 256, f.c0.c1);
  stash_fp(s + 2 * 12 * 256, f.c0.c2);
  stash_fp(s + 3 * 12 * 256, f.c1.c0);
  stash_fp(s + 4 * 12 * 256, f.c1.c1);
  stash_fp(s + 5 * 12 * 256, f.c1.c2);
}
HP_D H12 unstash12(const uint32_t* __restrict__ s) {
  H12 f;
  f.c0.c0 = unstash_fp(s + 0 * 12 * 256);
  f.c0.c1 = unstash_fp(s + 1 * 12 * 256);
  f.c0.c2 = unstash_fp(s + 2 * 12 * 256);
  f.c1.c0 = unstash_fp(s + 3 * 12 * 256);
  f.c1.c1 = unstash_fp(s + 4 * 12 * 256);
  f.c1.c2 = unstash_fp(s + 5 * 12 * 256);
  return f;
}

// ---------------------------------------------------------------- final exponentiation
// f^|x| (|x| + 1 if PLUS1) for f in the cyclotomic subgroup, square-and-multiply from the top
template <bool PLUS1>
HP_D H12 h_exp_abs_x(const H12& base) {
  const uint64_t e = PLUS1 ? hb::X_ABS + 1 : hb::X_ABS;
  H12 r = base;
#pragma unroll 1
  for (int k = 62; k >= 0; k--) {
    r = h12_cyclo_sqr(r);
    if ((e >> k) & 1) r = h12_mul(r, base);
  }
  return r;
}
// f^x = conj(f^|x|), f^(x-1) = conj(f^(|x|+1))  (x < 0)
HP_D H12 h_exp_x(const H12& f) { return h12_conj(h_exp_abs_x<false>(f)); }
HP_D H12 h_exp_xm1(const H12& f) { return h12_conj(h_exp_abs_x<true>(f)); }

// e = f^(3 (p^12 - 1) / r), pairing 0.14's hard-part chain (x3) reordered so that at most one
// Fp12 has to outlive an exponentiation (it waits in the LDS stash):
//   g = f^((p^6 - 1)(p^2 + 1));  a = (g^(x-1))^(x-1);  b = a^x frob1(a);
//   w = frob2(b) conj(b) g^3;    e = (b^x)^x w
HP_D H12 h_final_exp(const H12& f, uint32_t* __restrict__ stash) {
  const H12 f1 = h12_mul(h12_conj(f), h12_inv(f));
  const H12 g = h12_mul(h12_frob2(f1), f1);
  stash12(stash, g);
  H12 a = h_exp_xm1(h_exp_xm1(g));
  const H12 b = h12_mul(h_exp_x(a), h12_frob1(a));
  {
    const H12 gs = unstash12(stash);
    const H12 w = h12_mul(h12_mul(h12_frob2(b), h12_conj(b)), h12_mul(h12_cyclo_sqr(gs), gs));
    stash12(stash, w);
  }
  const H12 c = h_exp_x(h_exp_x(b));
  return h12_mul(c, unstash12(stash));
}

// ---------------------------------------------------------------- Miller-loop sides
struct PairSide {
  const uint32_t* p;    // G1 points, 24 words each; nullptr: the generator g1 for every check
  const uint32_t* q;    // WALK: G2 points, 48 words each
  const int4* lines;    // TABLE: line tables written by k_pair_prep
  const uint8_t* qinf;  // TABLE: 1 = table point at infinity
  const uint32_t* idx;  // Q index per check (nullptr = identity)
  uint32_t nq;          // number of Q points / tables
};

// Register budget (2 waves per SIMD = 256 VGPRs per lane): a side whose P is the generator (GEN)
// keeps no P in registers -- the line evaluation multiplies by constants -- and a walked side keeps
// only T: Q itself is re-read from memory at the 5 addition steps instead of living in 28 VGPRs
// through the 63 doublings.
struct SideState {
  Fp xP, yP;      // P (Montgomery), both lanes (unused when GEN)
  bool act;       // pair contributes (P != O and Q != O)
  bool qinf;      // WALK: Q is the point at infinity (the walk runs from (1, 1), masked out)
  uint32_t q;     // Q index
  HJac T;         // WALK: the running multiple of Q (own components)
};

template <bool GEN>
HP_D Fp side_xP(const SideState& st) { return GEN ? fp_const(hb::G1X_M) : st.xP; }
template <bool GEN>
HP_D Fp side_yP(const SideState& st, bool negate) {
  return GEN ? (negate ? fp_neg(fp_const(hb::G1Y_M)) : fp_const(hb::G1Y_M)) : st.yP;
}

HP_D void side_q(const PairSide& s, const SideState& st, Fp& xQ, Fp& yQ) {
  h_g2_load(s.q + (size_t)st.q * 48, xQ, yQ);
  if (st.qinf) {
    xQ = h_one();
    yQ = h_one();
  }
}

template <bool WALK, bool GEN>
HP_D bool side_init(const PairSide& s, int i, bool negate, SideState& st) {
  st.q = s.idx ? s.idx[i] : (uint32_t)i;
  if (st.q >= s.nq) return false;
  bool pinf;
  if (GEN) {
    pinf = false;
  } else if (s.p) {
    const uint32_t* w = s.p + (size_t)i * 24;
    pinf = words_zero(w, 24);
    st.xP = fp_from_words(w);
    st.yP = fp_from_words(w + 12);
  } else {
    pinf = false;
    st.xP = fp_const(hb::G1X_M);
    st.yP = fp_const(hb::G1Y_M);
  }
  if (!GEN && negate) st.yP = fp_neg(st.yP);
  if (WALK) {
    const uint32_t* w = s.q + (size_t)st.q * 48;
    st.qinf = lp_both(words_zero(w + (lp_even() ? 0 : 12), 12) && words_zero(w + (lp_even() ? 24 : 36), 12));
    Fp xQ, yQ;
    side_q(s, st, xQ, yQ);  // dummy walk from (1, 1) when Q = O: the pair is masked out
    st.T = {xQ, yQ, h_one()};
  } else {
    st.qinf = s.qinf[st.q] != 0;
  }
  st.act = !pinf && !st.qinf;
  return true;
}

// the side's line of this step, evaluated at P: (c0, c1 xP, c4 yP), or 1 for an inactive pair
template <bool WALK, bool GEN, bool DBL>
HP_D HLine side_line(const PairSide& s, SideState& st, int step, bool negate) {
  HLine l;
  if (WALK) {
    if (DBL) {
      l = h_dbl_step(st.T);
    } else {
      Fp xQ, yQ;
      side_q(s, st, xQ, yQ);
      l = h_add_step(st.T, xQ, yQ);
    }
  } else {
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
  }
  HLine e;
  e.c0 = st.act ? l.c0 : h_one();
  e.c1 = st.act ? fp_mul(l.c1, side_xP<GEN>(st)) : fp_zero();
  e.c4 = st.act ? fp_mul(l.c4, side_yP<GEN>(st, negate)) : fp_zero();
  return e;
}

struct PairArgs {
  int n;
  PairSide s1, s2;
  int flags;            // bit 0: negate P2 (pairing equality); bit 1: conjugate f (single pairing value)
  uint8_t* verdict;     // 1 byte per check (may be null)
  uint32_t* value_out;  // 144 canonical words per check (may be null)
};

// GEN: 0 = both P read per check, 1 = P1 is the generator, 2 = P2 is the generator
template <bool W1, bool W2, int GEN>
__global__ void __launch_bounds__(256, 2) k_pair_verify(PairArgs a) {
  extern __shared__ uint32_t stash_lds[];
  const int i = (int)((blockIdx.x * 256u + threadIdx.x) >> 1);
  if (i >= a.n) return;  // both lanes of a pair leave together
  constexpr bool G1 = GEN == 1, G2 = GEN == 2;
  const bool neg2 = (a.flags & 1) != 0;
  SideState A, B;
  const bool ok1 = side_init<W1, G1>(a.s1, i, false, A);
  const bool ok2 = side_init<W2, G2>(a.s2, i, neg2, B);
  if (!ok1 || !ok2) {  // index out of range: reject, never read past a table
    if (lp_even() && a.verdict) a.verdict[i] = 0;
    return;
  }
  H12 f = h12_one();
  int step = 0;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
    // the two sides' lines are multiplied together first, then into f (h12_mul_lines)
    if (b != 62) f = h12_sqr(f);
    {
      const HLine la = side_line<W1, G1, true>(a.s1, A, step, false);
      const HLine lb = side_line<W2, G2, true>(a.s2, B, step, neg2);
      f = h12_mul_lines(f, la.c0, la.c1, la.c4, lb.c0, lb.c1, lb.c4);
    }
    step++;
    if ((hb::X_ABS >> b) & 1) {
      const HLine la = side_line<W1, G1, false>(a.s1, A, step, false);
      const HLine lb = side_line<W2, G2, false>(a.s2, B, step, neg2);
      f = h12_mul_lines(f, la.c0, la.c1, la.c4, lb.c0, lb.c1, lb.c4);
      step++;
    }
  }
  if (a.flags & 2) f = h12_conj(f);
  const H12 e = h_final_exp(f, stash_lds + threadIdx.x);
  if (a.value_out) {
    uint32_t* o = a.value_out + (size_t)i * 144 + (lp_even() ? 0 : 12);
    fp_to_words(e.c0.c0, o + 0);
    fp_to_words(e.c0.c1, o + 24);
    fp_to_words(e.c0.c2, o + 48);
    fp_to_words(e.c1.c0, o + 72);
    fp_to_words(e.c1.c1, o + 96);
    fp_to_words(e.c1.c2, o + 120);
  }
  const bool one = h12_is_one(e);
  if (lp_even() && a.verdict) a.verdict[i] = one ? 1 : 0;
}

// ---------------------------------------------------------------- line tables of shared G2 points
__global__ void __launch_bounds__(256, 2) k_pair_prep(int n, const uint32_t* __restrict__ q, int4* __restrict__ lines,
                                                      uint8_t* __restrict__ qinf) {
  const int j = (int)((blockIdx.x * 256u + threadIdx.x) >> 1);
  if (j >= n) return;
  const uint32_t* w = q + (size_t)j * 48;
  const bool inf = lp_both(words_zero(w + (lp_even() ? 0 : 12), 12) && words_zero(w + (lp_even() ? 24 : 36), 12));
  Fp xQ, yQ;
  h_g2_load(w, xQ, yQ);
  if (inf) {
    xQ = h_one();
    yQ = h_one();
  }
  if (lp_even()) qinf[j] = inf ? 1 : 0;
  HJac T{xQ, yQ, h_one()};
  int4* base = lines + (size_t)j * PAIR_STEPS * 2 * PL_Q4 + (lp_even() ? 0 : PL_Q4);
  int step = 0;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
#pragma unroll 1
    for (int add = 0; add < (((hb::X_ABS >> b) & 1) ? 2 : 1); add++) {
      const HLine l = add ? h_add_step(T, xQ, yQ) : h_dbl_step(T);
      int32_t o[4 * PL_Q4];
#pragma unroll
      for (int k = 0; k < NL; k++) {
        o[k] = l.c0.l[k];
        o[NL + k] = l.c1.l[k];
        o[2 * NL + k] = l.c4.l[k];
      }
      o[3 * NL] = 0;
      o[3 * NL + 1] = 0;
      int4* dst = base + (size_t)step * 2 * PL_Q4;
#pragma unroll
      for (int k = 0; k < PL_Q4; k++) dst[k] = make_int4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
      step++;
    }
  }
}

}  // namespace hbs

namespace hbl {

size_t pair_table_bytes(size_t nq) { return nq * (size_t)hbs::PAIR_STEPS * 2 * hbs::PL_Q4 * 16; }

hipError_t pair_prep(hipStream_t s, int n, const void* q, void* lines, uint8_t* qinf) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hbs::k_pair_prep, dim3((unsigned)((2 * (size_t)n + 255) / 256)), dim3(256), 0, s, n,
                     (const uint32_t*)q, (int4*)lines, qinf);
  return hipGetLastError();
}

hipError_t pair_verify(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
                       uint8_t* verdict, uint32_t* value_out) {
  if (n <= 0) return hipSuccess;
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
  const dim3 grid((unsigned)((2 * (size_t)n + 255) / 256)), block(256);
  const size_t lds = (size_t)hbs::STASH_WORDS * 256 * 4;
  const bool w1 = d1.lines == nullptr, w2 = d2.lines == nullptr;
  // a null P on exactly one side selects the generator instantiation; both null keeps the
  // run-time generator path of side_init (P1 and P2 held in registers)
  const int gen = (d1.p == nullptr) == (d2.p == nullptr) ? 0 : (d1.p == nullptr ? 1 : 2);
#define HBS_PAIR_LAUNCH(G)                                                                 \
  do {                                                                                     \
    if (w1 && w2)                                                                          \
      hipLaunchKernelGGL((hbs::k_pair_verify<true, true, G>), grid, block, lds, s, a);     \
    else if (w1)                                                                           \
      hipLaunchKernelGGL((hbs::k_pair_verify<true, false, G>), grid, block, lds, s, a);    \
    else if (w2)                                                                           \
      hipLaunchKernelGGL((hbs::k_pair_verify<false, true, G>), grid, block, lds, s, a);    \
    else                                                                                   \
      hipLaunchKernelGGL((hbs::k_pair_verify<false, false, G>), grid, block, lds, s, a);   \
  } while (0)
  if (gen == 1)
    HBS_PAIR_LAUNCH(1);
  else if (gen == 2)
    HBS_PAIR_LAUNCH(2);
  else
    HBS_PAIR_LAUNCH(0);
#undef HBS_PAIR_LAUNCH
  return hipGetLastError();
}

}  // namespace hbl
