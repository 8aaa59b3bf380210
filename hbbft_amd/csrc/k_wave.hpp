// The wave-per-check pairing kernel's body (k_wave.hip: 32 lane pairs = one wave per check;
// k_wave64.hip: 64 lane pairs = two waves per check), instantiated per translation unit with
//   WV_NS      the kernel's namespace (hbs / hbs64),
//   WV_PROG    the namespace of the stage programs (hbw from wave_prog.inc / hbw64 from wave_prog64.inc),
//   WV_THREADS threads per check (64 / 128),
//   WV_FULL    1: the Miller-only, tree and product modes of the split master check (32-pair set only).
#pragma once
#ifndef WV_NS
#error "define WV_NS, WV_PROG, WV_THREADS and WV_FULL before including k_wave.hpp"
#endif
#include "launch.hpp"
#include "pfp.hpp"

namespace WV_NS {
using namespace hbs;

constexpr int WV_STRIDE = 36;  // words per slot (2 components x 16, +4 against bank conflicts)
constexpr int WV_LINE_Q4 = 11;  // k_oct_prep table: 16-byte chunks per (line, lane component)
constexpr uint32_t WV_ZW[NL] = {0};

struct WaveSide {
  const uint32_t* p;    // G1 points (24 words), nullptr = the generator
  const uint32_t* q;    // WALK: G2 points (48 words)
  const int4* lines;    // TABLE: k_oct_prep line tables (nullptr = WALK)
  const uint8_t* qinf;  // TABLE: 1 = table point at infinity
  const uint32_t* idx;  // Q index per check (nullptr = identity)
  uint32_t nq;
};

struct WaveArgs {
  int n;
  WaveSide s[2];
  int flags;            // bit 0: negate P2; bit 1: conjugated value (single pairing); bit 2: Miller only;
                        // bit 3: Jacobian P (36 words, both sides WALK); bit 4 (with 3): side 0 only
  uint8_t* verdict;
  uint32_t* value_out;  // 144 canonical words per check (may be null)
  const uint32_t* fin;  // product mode: nf Miller values (144 words, w-basis) per check; null otherwise
  int nf;
  uint32_t* tree_cnt;   // tree mode (wave_miller_tree): arrival counters, TREE_LEVELS x tree_nw per group
  int tree_nw;          // checks per group (0: no tree)
};
constexpr int TREE_LEVELS = 16;

// ---------------------------------------------------------------- LDS slots
HP_D Fp ld_own(const uint32_t* sm, int slot, int h) {
  const int4* p = (const int4*)(sm + slot * WV_STRIDE + h * 16);
  Fp r;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int4 v = p[q];
    r.l[4 * q] = v.x;
    r.l[4 * q + 1] = v.y;
    if (4 * q + 2 < NL) r.l[4 * q + 2] = v.z;
    if (4 * q + 3 < NL) r.l[4 * q + 3] = v.w;
  }
  return r;
}
HP_D void st_own(uint32_t* sm, int slot, int h, const Fp& a) {
  int4* p = (int4*)(sm + slot * WV_STRIDE + h * 16);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int i = 4 * q;
    p[q] = make_int4(a.l[i], a.l[i + 1], i + 2 < NL ? a.l[i + 2] : 0, i + 3 < NL ? a.l[i + 3] : 0);
  }
}

// One carry step on every limb at once: limb i keeps its low 28 bits plus the carry out of limb i - 1
// (taken from limb i - 1's value BEFORE this step).  For |limb| < 2^31 the result has limbs in
// [-8, 2^28 + 8) and the same value -- "almost normalised", which is all the product bounds need
// (sfp.hpp (M): |limb| <= 2^29), at the latency of one step instead of fp_norm's 13 dependent ones.
HP_D void fp_carry1(Fp& a) {
  int32_t c[NL];
#pragma unroll
  for (int i = 0; i < NL - 1; i++) c[i] = a.l[i] >> 28;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) a.l[i] &= MASK28;
#pragma unroll
  for (int i = 1; i < NL; i++) a.l[i] += c[i - 1];
}

// X = sgn * (S[a] + s * S[b]); s in {0, 1, -1} (codes 0, 1, 2), sgn = -1 for neg, -1 on the odd
// lane for conj.  Lazy limbs (|limb| < 2^29); normalised when `norm`.
HP_D Fp operand(const uint32_t* sm, int h, int a, int b, int scode, int negb, int conjb, bool sum, bool sgnflag,
                bool norm) {
  Fp x = ld_own(sm, a, h);
  if (sum) {
    const Fp y = ld_own(sm, b, h);
    const int32_t z = scode ? -1 : 0;
    const int32_t m = scode == 2 ? -1 : 0;
#pragma unroll
    for (int i = 0; i < NL; i++) x.l[i] += ((y.l[i] ^ m) - m) & z;
  }
  if (sgnflag) {
    const int32_t m = (negb ^ (conjb & h)) ? -1 : 0;
#pragma unroll
    for (int i = 0; i < NL; i++) x.l[i] = (x.l[i] ^ m) - m;
  }
  if (norm) fp_carry1(x);  // |limb| < 2^29 -> [-2, 2^28 + 1): the y operand of wv_mul
  return x;
}

// own component of sum_t x_t * y_t (Fp2, lane-pair split of pfp.hpp h_mul_l), one reduction.
// Each column may be summed in WV_NACC independent int64 chains, joined before the Montgomery digit.
// One chain is fastest (round 6 A/B, profiles/r06/ab_nacc_dpp.txt: single check 1.62 -> 1.53 ms,
// 4,096 checks 5.50 -> 5.18 ms against four): at one wave per SIMD a dependent v_mad_i64_i32 costs
// ~11 cycles against ~9 for independent ones (tools/ubench_issue.hip), while every extra chain costs
// a two-instruction 64-bit join per column -- the wave is issue-bound, not latency-bound.
#ifndef WV_NACC
#define WV_NACC 1
#endif
template <int K>
HP_D Fp wv_mul(const Fp (&x)[K], const Fp (&y)[K]) {
  const int32_t sm = lp_even() ? -1 : 0;
  int32_t Y[K][NL], W[K][NL], Z[K][NL];
#pragma unroll
  for (int t = 0; t < K; t++)
#pragma unroll
    for (int i = 0; i < NL; i++) {
      Y[t][i] = dpp<DPP_EVEN>(y[t].l[i]);
      W[t][i] = dpp<DPP_ODD>(y[t].l[i]);
      Z[t][i] = (dpp<DPP_SWAP>(x[t].l[i]) ^ sm) - sm;
    }
  int32_t m[NL];
  int64_t carry = 0;
  Fp r;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; k++) {
    int64_t acc[WV_NACC];
#pragma unroll
    for (int c = 0; c < WV_NACC; c++) acc[c] = 0;
    int q = 0;
    const int lo = k < NL ? 0 : k - NL + 1, hi = k < NL ? k : NL - 1;
#pragma unroll
    for (int t = 0; t < K; t++)
#pragma unroll
      for (int i = lo; i <= hi; i++) {
        acc[q++ % WV_NACC] += (int64_t)x[t].l[i] * Y[t][k - i];
        acc[q++ % WV_NACC] += (int64_t)Z[t][i] * W[t][k - i];
      }
#pragma unroll
    for (int i = lo; i <= hi; i++)
      if (i < k) acc[q++ % WV_NACC] += (int64_t)m[i] * (int32_t)P_L[k - i];
    int64_t col = carry;
#pragma unroll
    for (int c = 0; c < WV_NACC; c++) {
      if (WV_NACC > 1) asm("" : "+v"(acc[c]));  // keep the chains apart (no reassociation into one)
      col += acc[c];
    }
    if (k < NL) {
      m[k] = mont_digit(col);
      col += (int64_t)m[k] * (int32_t)P_L[0];
    } else {
      r.l[k - NL] = (int32_t)col & MASK28;
    }
    carry = col >> 28;
  }
  r.l[NL - 1] = (int32_t)carry;
  return r;
}

// x * y in Fp (one lane, sfp.hpp fp_mul's product scanning) with each column in WV_NACC chains: the
// same column sums, so the same output limbs as fp_mul, with a quarter of its dependent-MAD chain --
// the lane-pair squares (h_sqr) of the CYC runs and square stages, where nothing else hides it
HP_D Fp wv_fpmul(const Fp& x, const Fp& y) {
  int32_t m[NL];
  int64_t carry = 0;
  Fp r;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; k++) {
    int64_t acc[WV_NACC];
#pragma unroll
    for (int c = 0; c < WV_NACC; c++) acc[c] = 0;
    int q = 0;
    const int lo = k < NL ? 0 : k - NL + 1, hi = k < NL ? k : NL - 1;
#pragma unroll
    for (int i = lo; i <= hi; i++) acc[q++ % WV_NACC] += (int64_t)x.l[i] * y.l[k - i];
#pragma unroll
    for (int i = lo; i <= hi; i++)
      if (i < k) acc[q++ % WV_NACC] += (int64_t)m[i] * (int32_t)P_L[k - i];
    int64_t col = carry;
#pragma unroll
    for (int c = 0; c < WV_NACC; c++) {
      if (WV_NACC > 1) asm("" : "+v"(acc[c]));
      col += acc[c];
    }
    if (k < NL) {
      m[k] = mont_digit(col);
      col += (int64_t)m[k] * (int32_t)P_L[0];
    } else {
      r.l[k - NL] = (int32_t)col & MASK28;
    }
    carry = col >> 28;
  }
  r.l[NL - 1] = (int32_t)carry;
  return r;
}
// pfp.hpp h_sqr with wv_fpmul
HP_D Fp wv_sqr(const Fp& a) {
  const bool ev = lp_even();
  const Fp pa = dpp_fp<DPP_SWAP>(a);
  Fp x, y;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    x.l[i] = pa.l[i] + (ev ? a.l[i] : pa.l[i]);
    y.l[i] = a.l[i] - (ev ? pa.l[i] : 0);
  }
  return wv_fpmul(x, y);
}

template <int K>
HP_D Fp product(const uint32_t* sm, int h, const uint64_t* d, uint32_t fl) {
  const bool xs = fl & 0x100, ys = fl & 0x200, sg = fl & 0xC00;
  Fp x[K], y[K];
#pragma unroll
  for (int t = 0; t < K; t++) {
    const uint64_t w = d[t];
    const int hi = (int)(w >> 32);
    x[t] = operand(sm, h, (int)(w & 0xFF), (int)((w >> 8) & 0xFF), hi & 3, (hi >> 4) & 1, (hi >> 5) & 1, xs, sg, false);
    y[t] = operand(sm, h, (int)((w >> 16) & 0xFF), (int)((w >> 24) & 0xFF), (hi >> 2) & 3, (hi >> 6) & 1,
                   (hi >> 7) & 1, ys, sg, ys || sg);
  }
  return wv_mul<K>(x, y);
}

HP_D Fp product_sq(const uint32_t* sm, int h, uint64_t w, uint32_t fl) {
  const int hi = (int)(w >> 32);
  const bool xs = fl & 0x100, sg = fl & 0xC00;
  const Fp x = operand(sm, h, (int)(w & 0xFF), (int)((w >> 8) & 0xFF), hi & 3, (hi >> 4) & 1, (hi >> 5) & 1, xs, sg,
                       xs || sg);
  return wv_sqr(x);
}

// dst = sum c V + xi sum c' V' (8 x u16 descriptor: dst | gate << 8 | defone << 10, then terms
// src | coef (4-bit signed) << 8 | conj << 12), reduced; gated outputs of an inactive pair take 1 / 0
HP_D void assemble(uint32_t* sm, int h, uint4 dw, int j1, int j2, bool act0, bool act1) {
  const uint16_t ws[8] = {(uint16_t)dw.x, (uint16_t)(dw.x >> 16), (uint16_t)dw.y, (uint16_t)(dw.y >> 16),
                          (uint16_t)dw.z, (uint16_t)(dw.z >> 16), (uint16_t)dw.w, (uint16_t)(dw.w >> 16)};
  int64_t ap[NL], at[NL];  // c * v fused into one v_mad_i64_i32 per limb; the sums fit int32
#pragma unroll
  for (int i = 0; i < NL; i++) {
    ap[i] = 0;
    at[i] = 0;
  }
  // the seven terms' reads are written unconditionally (an unused term reads slot 0 and is never
  // added); the compiler places them.  Forcing all seven ahead of the sums (an empty asm using each
  // value) measured slower: single check 1.43 -> 1.48 ms (WAVE2), 1.65 -> 1.73 ms (WAVE),
  // profiles/r06/c14_inv/ab.txt -- register pressure at two waves per SIMD.
  Fp v[7];
  int cf[7];
#pragma unroll
  for (int t = 0; t < 7; t++) {
    const int tm = ws[1 + t];
    int c = (tm >> 8) & 0xF;
    c = c >= 8 ? c - 16 : c;
    if ((tm >> 12) & h & 1) c = -c;
    cf[t] = c;
    v[t] = ld_own(sm, t < j1 + j2 ? (tm & 0xFF) : 0, h);
  }
#pragma unroll
  for (int t = 0; t < 7; t++) {
    if (t < j1 + j2) {  // uniform across the wave
      if (t < j1) {
#pragma unroll
        for (int i = 0; i < NL; i++) ap[i] += (int64_t)cf[t] * v[t].l[i];
      } else {
#pragma unroll
        for (int i = 0; i < NL; i++) at[i] += (int64_t)cf[t] * v[t].l[i];
      }
    }
  }
  // Both sums fit int32 limbs (|limb| < 8 x 2^28: tools/gen_wave_prog.py check_bounds).  The twisted
  // sum joins as xi (t0 + t1 u) = (t0 - t1) + (t0 + t1) u on its unnormalised limbs (|u_i| < 2^33 in
  // int64), and ONE carry pass reduces: the quotient comes from the top limb alone, as in fp_red_mk
  // (the lower limbs move the value by < 2^369, far below p), so the output is normalised and in
  // (-p/256, p + p/256).  Round 5 normalised the twisted sum, the total and then reduced: three
  // serial carry chains where one is enough (round 6: the assembly phase was ~39 % of a Miller stage).
  int64_t u[NL];
  if (j2) {
    int32_t t[NL];
#pragma unroll
    for (int i = 0; i < NL; i++) t[i] = (int32_t)at[i];
#pragma unroll
    for (int i = 0; i < NL; i++) {
      const int32_t pt = dpp<DPP_SWAP>(t[i]);
      u[i] = ap[i] + (int64_t)t[i] + (int64_t)(h ? pt : -pt);
    }
  } else {
#pragma unroll
    for (int i = 0; i < NL; i++) u[i] = ap[i];
  }
  const int32_t q = (int32_t)((u[NL - 1] * QINV) >> 32);
  Fp r;
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    acc += u[i] - (int64_t)q * (int32_t)P_L[i];
    r.l[i] = (int32_t)acc & MASK28;
    acc >>= 28;
  }
  r.l[NL - 1] = (int32_t)(acc + u[NL - 1] - (int64_t)q * (int32_t)P_L[NL - 1]);
  const int gate = (ws[0] >> 8) & 3;
  if ((gate == 1 && !act0) || (gate == 2 && !act1)) r = ((ws[0] >> 10) & 1) ? h_one() : h_zero();
  st_own(sm, ws[0] & 0xFF, h, r);
}

// ---------------------------------------------------------------- CYC runs (register-resident squarings)
// Granger-Scott squaring splits into three Fp4 squarings: (f0, f3) -> (r0, r3), (f1, f4) -> (r2, r5),
// (f2, f5) -> (r1, r4), each of three Fp2 squares sA = A^2, sB = B^2, sAB = (A + B)^2 and outputs
//   X = 3 (sA + xi sB) - 2 L,  Y = 3 (sAB - sA - sB) + 2 L,  Z = 3 xi (sAB - sA - sB) + 2 L
// with L the input at the output's position.  Lane row g (16 lanes) runs one Fp4 squaring: lane quads
// 0 / 1 hold A / B (own Fp2 component), quad 2 squares A + B; the squares and the two inputs move by lane shuffles (ds_bpermute) inside
// the wave -- no LDS slot traffic and no barrier per squaring (DPP row shifts instead of the
// ds_bpermute exchanges inside a row measured neutral: single check -1.5 % on WAVE2, +1.8 % on WAVE,
// profiles/r06/ab_dpp.txt).  Row 0
// keeps (f0, f3).  Rows 1 and 2 swap roles each squaring: the row squaring (f1, f4) produces the next
// (f2, f5) and vice versa, so squaring inputs never move; only L crosses between rows 1 and 2.
HP_D Fp shfl_fp(const Fp& a, int src_lane) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = __builtin_amdgcn_ds_bpermute(src_lane << 2, a.l[i]);
  return r;
}
// reduce(3 t + k a) for k = +-2 chosen at run time: fp_red_mk's quotient from the top limb, then one
// parallel carry step (fp_carry1's) instead of a carry chain: limbs in [-32, 2^28 + 32), value as
// fp_red_mk's -- a squaring input again (cyc_run normalises once, when the run stores its result)
HP_D Fp fp_red_3k(const Fp& t, const Fp& a, int k) {
  const int64_t top = (int64_t)t.l[NL - 1] * 3 + (int64_t)k * a.l[NL - 1];
  const int32_t q = (int32_t)((top * QINV) >> 32);
  int64_t v[NL];
#pragma unroll
  for (int i = 0; i < NL - 1; i++) v[i] = (int64_t)t.l[i] * 3 + (int64_t)k * a.l[i] - (int64_t)q * (int32_t)P_L[i];
  v[NL - 1] = top - (int64_t)q * (int32_t)P_L[NL - 1];
  Fp r;
  r.l[0] = (int32_t)v[0] & MASK28;
#pragma unroll
  for (int i = 1; i < NL - 1; i++) r.l[i] = ((int32_t)v[i] & MASK28) + (int32_t)(v[i - 1] >> 28);
  r.l[NL - 1] = (int32_t)(v[NL - 1] + (v[NL - 2] >> 28));
  return r;
}
// position of the value a holder lane keeps: role 0 holds (f0, f3), role 1 (f1, f4), role 2 (f2, f5)
HP_D int cyc_pos(int role, int j) { return role + 3 * j; }

// w0 = six source slots (a byte each, w-basis order); w1 = six destination slots | count << 48 |
// conjugate-the-result << 56
HP_D void cyc_run(uint32_t* sm, int lane, uint64_t w0, uint64_t w1) {
  // lane = 16 row + 4 j + 2 rr + h: squaring j of the row, component h (rr: idle copy)
  const int h = lane & 1, rr = (lane >> 1) & 1, row = lane >> 4, j = (lane >> 2) & 3;
  const bool holder = row < 3 && j < 2;
  // the run's count and conjugation flag are the same on every lane: read them into scalar registers
  // so the squaring loop is a scalar loop (no per-iteration exec-mask bookkeeping)
  const int count = __builtin_amdgcn_readfirstlane((int)((w1 >> 48) & 0xFF));
  const bool conj = (__builtin_amdgcn_readfirstlane((int)(w1 >> 56)) & 1) != 0;
  int role = row < 3 ? row : 0;
  Fp v = fp_zero();
  if (holder) v = ld_own(sm, (int)((w0 >> (8 * cyc_pos(role, j))) & 0xFF), h);
  const int base = (lane & 0x30) | h;  // this row's squaring 0, product half 0, own component
  const int partner = (row == 1 || row == 2) ? (((3 - row) << 4) | (lane & 15)) : lane;
#pragma unroll 1
  for (int it = 0; it < count; it++) {
    const Fp A = shfl_fp(v, base), B = shfl_fp(v, base + 4);
    Fp x = fp_addl(A, B);
    fp_carry1(x);
    x = fp_sel(j == 2, x, v);
    const Fp sq = wv_sqr(x);
    const Fp sA = shfl_fp(sq, base), sB = shfl_fp(sq, base + 4), sAB = shfl_fp(sq, base + 8);
    const Fp L = shfl_fp(v, partner);
    // role 0 / 1: pair 0 -> X (r0 / r2), pair 1 -> Y (r3 / r5); role 2: pair 0 -> Z (r1), pair 1 -> X (r4)
    const bool isX = role != 2 ? j == 0 : j == 1;
    const bool isZ = role == 2 && j == 0;
    const Fp u = fp_sub2l(sAB, sA, sB);
    const Fp T = isX ? h_add_xi_l(sA, sB) : (isZ ? h_xi_l(u) : u);
    Fp r = fp_red_3k(T, L, isX ? -2 : 2);
    if (conj && it == count - 1 && (role == 2 ? j == 0 : j == 1)) r = fp_neg(r);  // odd positions
    v = r;
    if (row == 1 || row == 2) role = 3 - role;  // (f1, f4) <-> (f2, f5)
  }
  fp_norm(v);  // the run's values are almost normalised (fp_red_3k); slots hold normalised limbs
  if (holder && rr == 0) st_own(sm, (int)((w1 >> (8 * cyc_pos(role, j))) & 0xFF), h, v);
}

// the final exponentiation's one inversion (pair 0; both lanes invert the same norm, so the batched
// variable-time form; k_wave64 also keeps its coefficients unreduced, words.hpp INV_LAZY, which makes
// the 256-register k_wave spill -- round 6 A/B, profiles/r06/ab_inv.txt)
HP_D Fp wv_inv(const Fp& v) {
  return fp_reduce(h_inv_vartime<WV_THREADS == 128 ? (hb::INV_BATCH | hb::INV_LAZY) : hb::INV_BATCH>(v));
}

// this lane's descriptors of one stage (product: K u64 of its pair; assembly: 8 u16 of its output)
struct StageDesc {
  uint4 hd;
  uint64_t p0, p1;
  uint4 ad;
};
HP_D StageDesc load_stage(const uint4* hdr, int st, int pair) {
  StageDesc d;
  d.hd = hdr[st];
  const uint32_t fl = d.hd.x;
  const int kind = fl & 3, npairs = (fl >> 16) & 127, nouts = (fl >> 23) & 127;
  d.p0 = d.p1 = 0;
  d.ad = make_uint4(0, 0, 0, 0);
  if (((fl >> 12) & 0xF) == 2) {  // CYC run: source and destination slots, count, conjugation
    d.p0 = WV_PROG::WP_PDESC[d.hd.y];
    d.p1 = WV_PROG::WP_PDESC[d.hd.y + 1];
  } else if (kind != 3 && pair < npairs) {
    if (kind == 1) {
      d.p0 = WV_PROG::WP_PDESC[d.hd.y + 2 * pair];
      d.p1 = WV_PROG::WP_PDESC[d.hd.y + 2 * pair + 1];
    } else {
      d.p0 = WV_PROG::WP_PDESC[d.hd.y + pair];
    }
  }
  if (pair < nouts) d.ad = ((const uint4*)WV_PROG::WP_ADESC)[d.hd.z + pair];
  return d;
}

HP_D void run_stages(uint32_t* sm, int off, int nst, int h, int pair, bool act0, bool act1, const int4* tl0,
                     const int4* tl1) {
  const uint4* hdr = (const uint4*)WV_PROG::WP_HDR;
  // descriptors are fetched one stage ahead: their L2 latency hides behind the current stage
  StageDesc cur = load_stage(hdr, off, pair);
#ifdef WV_STAGE_CLOCK  // timing-only builds: core cycles per stage kind (M1 M2 SQ NONE INV CYC), block 0
  uint64_t clk[6] = {0, 0, 0, 0, 0, 0};
  int cnt[6] = {0, 0, 0, 0, 0, 0};
  uint64_t ph[4] = {0, 0, 0, 0};  // M1/M2/SQ stages: product, first barrier, assembly, second barrier
  uint64_t tp1 = 0, tp2 = 0, tp3 = 0;
  const uint64_t t_all = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll 1
  for (int st = off; st < off + nst; st++) {
#ifdef WV_STAGE_CLOCK
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
    const StageDesc nxt = load_stage(hdr, st + 1 < off + nst ? st + 1 : st, pair);
    const uint4 hd = cur.hd;
    const uint32_t fl = hd.x;
    const int kind = fl & 3, j1 = (fl >> 2) & 7, j2 = (fl >> 5) & 7, special = (fl >> 12) & 0xF;
    const int npairs = (fl >> 16) & 127, nouts = (fl >> 23) & 127;
    // table lines requested by this stage, fetched now and written after the assembly phase
    int4 tline[WV_LINE_Q4];
    int tslot = -1;
#pragma unroll
    for (int side = 0; side < 2; side++) {
      const uint32_t e = (hd.w >> (16 * side)) & 0xFFFF;
      if (special == 0 && (e & 1) && pair == side) {
        const int4* src = (side ? tl1 : tl0) + ((size_t)((e >> 1) & 0x7F) * 2 + h) * WV_LINE_Q4;
#pragma unroll
        for (int k = 0; k < WV_LINE_Q4; k++) tline[k] = src[k];
        tslot = (int)(e >> 8);
      }
    }
    if (special == 2) {
      if (WV_THREADS == 64 || threadIdx.x < 64) cyc_run(sm, 2 * pair + h, cur.p0, cur.p1);  // wave 0's rows
    } else if (special == 1) {
      if (pair == 0) {
        const Fp v = ld_own(sm, hd.w & 0xFF, h);
        st_own(sm, (hd.w >> 8) & 0xFF, h, wv_inv(v));  // pair 0 only: uniform
      }
    } else if (kind != 3 && pair < npairs) {
      Fp r;
      if (kind == 1) {
        const uint64_t dd[2] = {cur.p0, cur.p1};
        r = product<2>(sm, h, dd, fl);
      } else if (kind == 2) {
        r = product_sq(sm, h, cur.p0, fl);
      } else {
        const uint64_t dd[1] = {cur.p0};
        r = product<1>(sm, h, dd, fl);
      }
      st_own(sm, WV_PROG::WP_PROD + pair, h, r);
    }
#ifdef WV_STAGE_CLOCK
    tp1 = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();
#ifdef WV_STAGE_CLOCK
    tp2 = __builtin_amdgcn_s_memtime();
#endif
    if (pair < nouts) assemble(sm, h, cur.ad, j1, j2, act0, act1);
    if (tslot >= 0) {
      int32_t w[4 * WV_LINE_Q4];
#pragma unroll
      for (int k = 0; k < WV_LINE_Q4; k++) {
        w[4 * k] = tline[k].x;
        w[4 * k + 1] = tline[k].y;
        w[4 * k + 2] = tline[k].z;
        w[4 * k + 3] = tline[k].w;
      }
#pragma unroll
      for (int c = 0; c < 3; c++) {
        Fp v;
#pragma unroll
        for (int i = 0; i < NL; i++) v.l[i] = w[c * NL + i];
        st_own(sm, tslot + c, h, v);
      }
    }
#ifdef WV_STAGE_CLOCK
    tp3 = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();
#ifdef WV_STAGE_CLOCK
    {
      const int sp = (cur.hd.x >> 12) & 0xF, cat = sp == 2 ? 5 : sp == 1 ? 4 : (int)(cur.hd.x & 3);
      const uint64_t t4 = __builtin_amdgcn_s_memtime();
      clk[cat] += t4 - t0;
      cnt[cat]++;
      if (cat < 3) {
        ph[0] += tp1 - t0;
        ph[1] += tp2 - tp1;
        ph[2] += tp3 - tp2;
        ph[3] += t4 - tp3;
      }
    }
#endif
    cur = nxt;
  }
#ifdef WV_STAGE_CLOCK
  if (blockIdx.x == 0 && threadIdx.x == 0)
    printf("STAGECLK threads %d off %d nst %d total %lu | M1 %d %lu | M2 %d %lu | SQ %d %lu | NONE %d %lu | INV %d %lu | CYC %d %lu\n",
           (int)WV_THREADS, off, nst, (unsigned long)(__builtin_amdgcn_s_memtime() - t_all), cnt[0], (unsigned long)clk[0],
           cnt[1], (unsigned long)clk[1], cnt[2], (unsigned long)clk[2], cnt[3], (unsigned long)clk[3], cnt[4],
           (unsigned long)clk[4], cnt[5], (unsigned long)clk[5]);
  if (blockIdx.x == 0 && (threadIdx.x & 63) == 0)
    printf("PHASES wave %d product %lu barrier1 %lu assembly %lu barrier2 %lu\n", (int)(threadIdx.x >> 6),
           (unsigned long)ph[0], (unsigned long)ph[1], (unsigned long)ph[2], (unsigned long)ph[3]);
#endif
}

// constant slots (tools/gen_wave_prog.py CONSTS): pair k writes slot k
HP_D void put_const(uint32_t* sm, int h, int slot, const uint32_t (&c0)[NL], const uint32_t (&c1)[NL]) {
  Fp v;
#pragma unroll
  for (int i = 0; i < NL; i++) v.l[i] = (int32_t)(h ? c1[i] : c0[i]);
  st_own(sm, slot, h, v);
}

// side K of check i: writes its slots (pair K: XP, YP (ZP); pair 2 + K: QX, QY, T), returns the line
// table of a TABLE side; bad = Q index out of range
template <int K>
HP_D const int4* wave_side(const WaveArgs& a, uint32_t* sm, int i, int h, int pair, bool& act, bool& bad) {
  const WaveSide& s = a.s[K];
  const uint32_t q = s.idx ? s.idx[i] : (uint32_t)i;
  act = false;
  bad = q >= s.nq;
  if (bad) return nullptr;
  const bool neg = K == 1 && (a.flags & 1);
  bool pinf = false;
  Fp xp, yp, zp3;
  if (s.p && (a.flags & 8)) {  // Jacobian P (X, Y, Z; Z = 0 at infinity): XP = X Z, YP = Y, ZP = Z^3
    const uint32_t* w = s.p + (size_t)i * 36;
    pinf = words_zero(w + 24, 12);
    const Fp z = fp_from_words(w + 24);
    xp = fp_mul(fp_from_words(w), z);
    yp = fp_from_words(w + 12);
    zp3 = fp_mul(fp_sqr(z), z);
    if (neg) yp = fp_neg(yp);
  } else if (s.p) {
    const uint32_t* w = s.p + (size_t)i * 24;
    pinf = words_zero(w, 24);
    xp = fp_from_words(w);
    yp = fp_from_words(w + 12);
    if (neg) yp = fp_neg(yp);
  } else {
    xp = fp_const(hb::G1X_M);
    yp = fp_const(neg ? hb::G1NY_M : hb::G1Y_M);
  }
  const int base = K ? WV_PROG::WP_SIDE1 : WV_PROG::WP_SIDE0;
  const int4* tl = nullptr;
  bool qinf;
  if (s.lines) {
    qinf = s.qinf[q] != 0;
    tl = s.lines + (size_t)q * 68 * 2 * WV_LINE_Q4;
  } else {
    const uint32_t* w = s.q + (size_t)q * 48;
    qinf = words_zero(w, 48);
    if (pair == 2 + K) {
      Fp xq, yq;
      h_g2_load(w, xq, yq);
      if (qinf) {
        xq = h_one();
        yq = h_one();
      }
      st_own(sm, base + 2, h, xq);
      st_own(sm, base + 3, h, yq);
      st_own(sm, base + 4, h, xq);
      st_own(sm, base + 5, h, yq);
      st_own(sm, base + 6, h, h_one());
    }
  }
  if (pair == K) {
    st_own(sm, base + 0, h, h ? fp_zero() : xp);
    st_own(sm, base + 1, h, h ? fp_zero() : yp);
    if (s.p && (a.flags & 8)) st_own(sm, base + 7, h, h ? fp_zero() : zp3);
  }
  act = !pinf && !qinf;
  return tl;
}

// the constant slots of tools/gen_wave_prog.py CONSTS and F = 1 (pair k writes slot k)
static_assert(WV_PROG::WP_F == 18, "CONSTS of tools/gen_wave_prog.py: 18 constant slots before F");
HP_D void wave_consts(uint32_t* sm, int h, int pair) {
  switch (pair) {
    case 0: put_const(sm, h, 0, WV_ZW, WV_ZW); break;
    case 1: put_const(sm, h, 1, hb::ONE_L, WV_ZW); break;
    case 2: put_const(sm, h, 2, hb::FROB1_0_C0, hb::FROB1_0_C1); break;
    case 3: put_const(sm, h, 3, hb::FROB1_1_C0, hb::FROB1_1_C1); break;
    case 4: put_const(sm, h, 4, hb::FROB1_2_C0, hb::FROB1_2_C1); break;
    case 5: put_const(sm, h, 5, hb::FROB1_3_C0, hb::FROB1_3_C1); break;
    case 6: put_const(sm, h, 6, hb::FROB1_4_C0, hb::FROB1_4_C1); break;
    case 7: put_const(sm, h, 7, hb::FROB1_5_C0, hb::FROB1_5_C1); break;
    case 8: put_const(sm, h, 8, hb::FROB2_0_C0, WV_ZW); break;
    case 9: put_const(sm, h, 9, hb::FROB2_1_C0, WV_ZW); break;
    case 10: put_const(sm, h, 10, hb::FROB2_2_C0, WV_ZW); break;
    case 11: put_const(sm, h, 11, hb::FROB2_3_C0, WV_ZW); break;
    case 12: put_const(sm, h, 12, hb::FROB2_4_C0, WV_ZW); break;
    case 13: put_const(sm, h, 13, hb::FROB2_5_C0, WV_ZW); break;
    case 14: put_const(sm, h, 14, hb::G1X_M, WV_ZW); break;
    case 15: put_const(sm, h, 15, hb::G1Y_M, WV_ZW); break;
    case 16: put_const(sm, h, 16, hb::G1NY_M, WV_ZW); break;
    case 17: {  // 12 xi = 3 b' (both components 12), the homogeneous walk of mode W1J
      const Fp six = fp_lin(6, fp_one(), 0, fp_one());
      st_own(sm, 17, h, fp_reduce(fp_add(six, six)));
      break;
    }
    case 18: put_const(sm, h, WV_PROG::WP_F, hb::ONE_L, WV_ZW); break;
    default:
      if (pair < 24) put_const(sm, h, WV_PROG::WP_F + pair - 18, WV_ZW, WV_ZW);
      break;
  }
}

// Fp12 value k of check i (w-basis, 144 canonical words: component k at 24 k, lane h's half at
// 12 h) into six consecutive slots from `slot` (pairs 0..5 load one component each)
HP_D void wave_load12(uint32_t* sm, int h, int pair, int slot, const uint32_t* v) {
  if (pair < 6) st_own(sm, slot + pair, h, fp_from_words(v + 24 * pair + 12 * h));
}

__global__ void __launch_bounds__(WV_THREADS, WV_THREADS == 64 ? 2 : 1) k_wave(WaveArgs a) {
  extern __shared__ uint32_t sm[];
  const int i = blockIdx.x;
  if (i >= a.n) return;
  const int lane = threadIdx.x, h = lane & 1, pair = lane >> 1;
  wave_consts(sm, h, pair);
  if (WV_FULL && a.fin) {
    // product mode: F = prod_k fin[i][k] (one MULF program per factor), then the final
    // exponentiation -- the second half of the split master check (hbh_combine_verify_g2)
    const uint32_t* f = a.fin + (size_t)i * a.nf * 144;
    wave_load12(sm, h, pair, WV_PROG::WP_F, f);
    for (int k = 1; k < a.nf; k++) {
      wave_load12(sm, h, pair, WV_PROG::WP_SIDE0, f + (size_t)k * 144);
      __syncthreads();
      run_stages(sm, WV_PROG::WP_MULF_OFF, WV_PROG::WP_MULF_N, h, pair, true, true, nullptr, nullptr);
    }
    __syncthreads();
    run_stages(sm, WV_PROG::WP_FE_OFF, WV_PROG::WP_FE_N, h, pair, true, true, nullptr, nullptr);
  } else {
    // the two sides: P (G1) -> XP, YP as Fp2 (x, 0); Q -> QX, QY and T = (Q, 1); activity flags
    bool act0, act1, bad0, bad1;
    const int4* tl0 = wave_side<0>(a, sm, i, h, pair, act0, bad0);
    const int4* tl1 = nullptr;
    act1 = bad1 = false;
    if (!(a.flags & 16)) tl1 = wave_side<1>(a, sm, i, h, pair, act1, bad1);
    const bool bad = bad0 || bad1;
    if (bad) {  // index out of range: reject, never read past a table (uniform per workgroup)
      if (lane == 0 && a.verdict && !a.tree_nw) a.verdict[i] = 0;  // tree mode: the group's stays 0
      return;
    }
    __syncthreads();
    const int mv = (a.flags & 16) ? 5 : (a.flags & 8) ? 4 : (a.s[0].lines ? 2 : 0) + (a.s[1].lines ? 1 : 0);
    run_stages(sm, WV_PROG::WP_MILLER_OFF[mv], WV_PROG::WP_MILLER_N[mv], h, pair, act0, act1, tl0, tl1);
    if (WV_FULL && a.tree_nw) {
      // tree mode: node `node` of level L holds the product of checks [node 2^L, (node + 1) 2^L) of the
      // group, published at the slot of its first check.  Of two siblings the later arrival (counter
      // old value 1) multiplies and climbs; the earlier one leaves -- no wave ever waits on another.
      const int nw = a.tree_nw, g = i / nw;
      uint32_t* vals = a.value_out + (size_t)g * nw * 144;
      int node = i - g * nw;
      for (int L = 0; (1 << L) < nw; L++, node >>= 1) {
        const int sib = node ^ 1;
        if ((sib << L) >= nw) continue;  // no sibling at this level: the value climbs as it is
        if (pair < 6) fp_to_words(ld_own(sm, WV_PROG::WP_F + pair, h), vals + (size_t)(node << L) * 144 + 24 * pair + 12 * h);
        __threadfence();  // release: the value is visible device-wide (every XCD) before the count
        __syncthreads();
        int old = 0;
        if (lane == 0) old = (int)atomicAdd(a.tree_cnt + ((size_t)g * TREE_LEVELS + L) * nw + (node >> 1), 1u);
        old = __shfl(old, 0);
        if (old == 0) return;  // the sibling arrives later and carries on
        __threadfence();       // acquire: the sibling's published value
        wave_load12(sm, h, pair, WV_PROG::WP_SIDE0, vals + (size_t)(sib << L) * 144);
        __syncthreads();
        run_stages(sm, WV_PROG::WP_MULF_OFF, WV_PROG::WP_MULF_N, h, pair, true, true, nullptr, nullptr);
      }
      __syncthreads();
      run_stages(sm, WV_PROG::WP_FE_OFF, WV_PROG::WP_FE_N, h, pair, true, true, nullptr, nullptr);
      bool ok = true;
      if (pair < 6) ok = fp_is_zero(fp_sub(ld_own(sm, WV_PROG::WP_E + pair, h), pair == 0 ? h_one() : h_zero()));
      const bool all = __all(ok);
      if (lane == 0 && a.verdict) a.verdict[g] = all ? 1 : 0;
      return;
    }
    if (a.flags & 4) {  // Miller only: f (w-basis) out, no final exponentiation
      if (pair < 6 && a.value_out)
        fp_to_words(ld_own(sm, WV_PROG::WP_F + pair, h), a.value_out + (size_t)i * 144 + 24 * pair + 12 * h);
      return;
    }
    run_stages(sm, WV_PROG::WP_FE_OFF, WV_PROG::WP_FE_N, h, pair, act0, act1, tl0, tl1);
  }
  // e = f^(3 (p^12 - 1) / r) in slots E0..E5 (w-basis)
  bool ok = true;
  if (pair < 6) {
    Fp v = ld_own(sm, WV_PROG::WP_E + pair, h);
    if (a.value_out) {
      if ((a.flags & 2) && (pair & 1)) v = fp_neg(v);
      const int pos = (pair & 1) ? 3 + (pair >> 1) : (pair >> 1);
      fp_to_words(v, a.value_out + (size_t)i * 144 + 24 * pos + 12 * h);
    }
    const Fp want = (pair == 0) ? h_one() : h_zero();
    ok = fp_is_zero(fp_sub(v, want));
  }
  const bool all = __all(ok);
  if (lane == 0 && a.verdict) a.verdict[i] = all ? 1 : 0;
}

}  // namespace WV_NS

