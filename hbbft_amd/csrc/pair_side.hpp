// Shared by the lane-pair (k_pair.hip) and lane-quad (k_quad.hip) pairing kernels: the LDS stash
// of the final exponentiation and the Miller-loop sides (line tables, walked G2 points, P).
#pragma once
#include "qfp.hpp"

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

// ---------------------------------------------------------------- Miller-loop sides
struct PairSide {
  const uint32_t* p;    // G1 points, 24 words each; nullptr: the generator g1 for every check
  const uint32_t* q;    // WALK: G2 points, 48 words each
  const int4* lines;    // TABLE: line tables written by k_oct_prep
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
// QUAD: the lane-quad variants (qfp.hpp) of the walk and of the evaluation at P
template <bool WALK, bool GEN, bool DBL, bool QUAD = false>
HP_D HLine side_line(const PairSide& s, SideState& st, int step, bool negate) {
  HLine l;
  if (WALK) {
    if (DBL) {
      if constexpr (QUAD) l = h_dbl_step_q(st.T); else l = h_dbl_step(st.T);
    } else {
      Fp xQ, yQ;
      side_q(s, st, xQ, yQ);
      if constexpr (QUAD) l = h_add_step_q(st.T, xQ, yQ); else l = h_add_step(st.T, xQ, yQ);
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
  if constexpr (QUAD) {
    Fp c1, c4;
    fp_mul2(l.c1, side_xP<GEN>(st), l.c4, side_yP<GEN>(st, negate), c1, c4);
    e.c1 = st.act ? c1 : fp_zero();
    e.c4 = st.act ? c4 : fp_zero();
  } else {
    e.c1 = st.act ? fp_mul(l.c1, side_xP<GEN>(st)) : fp_zero();
    e.c4 = st.act ? fp_mul(l.c4, side_yP<GEN>(st, negate)) : fp_zero();
  }
  return e;
}

struct PairArgs {
  int n;
  PairSide s1, s2;
  int flags;            // bit 0: negate P2 (pairing equality); bit 1: conjugate f (single pairing value)
  uint8_t* verdict;     // 1 byte per check (may be null)
  uint32_t* value_out;  // 144 canonical words per check (may be null)
};

}  // namespace hbs
