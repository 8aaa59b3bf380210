// Lane-cooperative pairing check (gfx950): SIX lanes per check, lane k holding the Fp2 coefficient
// f_k of the Fp12 accumulator f = sum f_k w^k (w^6 = xi = 1 + u).  A wave carries 10 checks
// (lanes 60..63 idle).  Every Fp12 operation is split so that each lane performs a few Fp2
// products on operands fetched from its group with __shfl (ds_bpermute):
//   Miller squaring   : complex squaring over Fp6 -- lanes 0-2 form t = c0 c1, lanes 3-5
//                       s = (c0 + c1)(c0 + v c1); 3 Fp2 products per lane
//   line multiplication: f_k c0 + xi^[k<2] f_{k-2} c1 + xi^[k<3] f_{k-3} c4; 3 products per lane
//   cyclotomic square : Granger-Scott; the 18 Fp products split 3 per lane (no redundancy)
//   generic product   : schoolbook, 6 Fp2 products per lane
// Per-lane state is one Fp2 (28 VGPRs) instead of one Fp12 (168), so the kernels keep a small
// register footprint and run several waves per SIMD; the wave scheduler, not the compiler, hides
// the MAD latency.  Stages communicate through HBM in a lane-major layout
// (word w of lane (check, k) at buf[w * lstride + check * 6 + k]: a wave reads 256 contiguous bytes).
// Same formulas and verdict as pairing.hpp (miller loop + final_exp_x3); line tables come from
// k_g2_prepare.
#include <hip/hip_runtime.h>

#include "launch.hpp"
#include "sfp.hpp"

// Minimum waves per SIMD requested from the register allocator (tuned).
#ifndef HBS_LB_MILLER
#define HBS_LB_MILLER 1
#endif
#ifndef HBS_LB_EXP
#define HBS_LB_EXP 1
#endif

namespace hbs {

constexpr int GL = 6;            // lanes per check
constexpr int CPW = 10;          // checks per wave
constexpr int F2W = 2 * NL;      // 28 words per Fp2
constexpr int LINE_WORDS = 84;   // c0, c1, c4 (Fp2 each) per line, 14-limb words
constexpr uint64_t X_ABS = 0xd201000000010000ull;

struct Lane {
  int k;      // coefficient index 0..5
  int base;   // first lane of the group in the wave
  int check;  // check index
  bool valid;
};

__device__ __forceinline__ Lane lane_ids(int n) {
  const int lane = threadIdx.x & 63;
  const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int g = lane / GL;
  Lane L;
  L.k = lane - g * GL;
  L.base = g * GL;
  L.check = wave * CPW + g;
  L.valid = g < CPW && L.check < n;
  return L;
}

__device__ __forceinline__ Fp shfl_fp(const Fp& a, int src) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = __shfl(a.l[i], src, 64);
  return r;
}
__device__ __forceinline__ Fp2 shfl2(const Fp2& a, int src) { return {shfl_fp(a.c0, src), shfl_fp(a.c1, src)}; }

// lane-major state I/O
__device__ __forceinline__ Fp2 ld2(const int32_t* __restrict__ b, size_t lstride, size_t gl) {
  Fp2 r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.c0.l[i] = b[(size_t)i * lstride + gl];
#pragma unroll
  for (int i = 0; i < NL; i++) r.c1.l[i] = b[(size_t)(NL + i) * lstride + gl];
  return r;
}
__device__ __forceinline__ void st2(int32_t* __restrict__ b, size_t lstride, size_t gl, const Fp2& v) {
#pragma unroll
  for (int i = 0; i < NL; i++) b[(size_t)i * lstride + gl] = v.c0.l[i];
#pragma unroll
  for (int i = 0; i < NL; i++) b[(size_t)(NL + i) * lstride + gl] = v.c1.l[i];
}

// ------------------------------------------------------------------ lane-cooperative Fp12 ops
// All take / return the lane's reduced coefficient (|.| < 2p).

// f^2 by complex squaring over Fp6 = Fp2[v]/(v^3 - xi): c0 = (f0, f2, f4), c1 = (f1, f3, f5).
__device__ __forceinline__ Fp2 lc_sqr(const Fp2& f, const Lane& L) {
  const bool sl = L.k >= 3;          // lanes 3-5 form s, lanes 0-2 form t
  const int m = sl ? L.k - 3 : L.k;  // output coefficient of the Fp6 product
  Fp2 acc = f2_zero();
#pragma unroll 1
  for (int i = 0; i < 3; i++) {
    const int j = (m - i + 3) % 3;
    const Fp2 c0i = shfl2(f, L.base + 2 * i);
    const Fp2 c1i = shfl2(f, L.base + 2 * i + 1);
    const Fp2 c0j = shfl2(f, L.base + 2 * j);
    const Fp2 c1j = shfl2(f, L.base + 2 * j + 1);
    Fp2 vc1j = shfl2(f, L.base + (j == 0 ? 5 : 2 * j - 1));  // (v c1)_j = xi c1_2, c1_0, c1_1
    if (j == 0) vc1j = f2_mul_xi(vc1j);
    const Fp2 x = sl ? f2_add(c0i, c1i) : c0i;               // A_i = c0_i + c1_i  |  c0_i
    const Fp2 y = sl ? f2_add(c0j, vc1j) : c1j;              // B_j = c0_j + (v c1)_j  |  c1_j
    Fp2 p = f2_mul(x, y);
    if (i > m) p = f2_mul_xi(p);
    acc = f2_add(acc, p);
  }
  // t_m at lane m, s_m at lane 3 + m.  c0'_m = s_m - t_m - (v t)_m ; c1'_m = 2 t_m
  const bool even = (L.k & 1) == 0;
  const int mo = even ? L.k >> 1 : (L.k - 1) >> 1;
  const Fp2 s_m = shfl2(acc, L.base + 3 + mo);
  const Fp2 t_m = shfl2(acc, L.base + mo);
  Fp2 vt = shfl2(acc, L.base + (mo + 2) % 3);  // (v t)_m = xi t_2 (m = 0), t_{m-1}
  if (mo == 0) vt = f2_mul_xi(vt);
  const Fp2 r = even ? f2_sub(f2_sub(s_m, t_m), vt) : f2_add(t_m, t_m);
  return f2_red(r);
}

// f * (c0 + c1 w^2 + c4 w^3)
__device__ __forceinline__ Fp2 lc_mul014(const Fp2& f, const Lane& L, const Fp2& c0, const Fp2& c1, const Fp2& c4) {
  const Fp2 b = shfl2(f, L.base + (L.k + 4) % 6);  // f_{k-2}
  const Fp2 c = shfl2(f, L.base + (L.k + 3) % 6);  // f_{k-3}
  const Fp2 t0 = f2_mul(f, c0);
  Fp2 t1 = f2_mul(b, c1);
  Fp2 t2 = f2_mul(c, c4);
  if (L.k < 2) t1 = f2_mul_xi(t1);
  if (L.k < 3) t2 = f2_mul_xi(t2);
  return f2_red(f2_add(f2_add(t0, t1), t2));
}

// general product a * b (schoolbook over the w-basis)
__device__ __forceinline__ Fp2 lc_mul(const Fp2& a, const Fp2& b, const Lane& L) {
  Fp2 acc = f2_zero();
#pragma unroll 1
  for (int j = 0; j < 6; j++) {
    const Fp2 x = shfl2(a, L.base + (L.k - j + 6) % 6);
    const Fp2 y = shfl2(b, L.base + j);
    Fp2 p = f2_mul(x, y);
    if (j > L.k) p = f2_mul_xi(p);
    acc = f2_add(acc, p);
  }
  return f2_red(acc);
}

__device__ __forceinline__ Fp2 lc_conj(const Fp2& f, const Lane& L) { return (L.k & 1) ? f2_neg(f) : f; }

// Granger-Scott cyclotomic squaring: pairs q = k mod 3 (f_q, f_{q+3}) form Fp4 = Fp2[t]/(t^2 - xi)
// elements A, B, C; lane q computes the (c0+c1)(c0-c1) halves of the 3 Fp2 squarings of its pair,
// lane q+3 the c0*c1 halves.
__device__ __forceinline__ Fp2 lc_cyclo_sqr(const Fp2& f, const Lane& L) {
  const int q = L.k % 3;
  const bool lo = L.k < 3;
  const Fp2 x0 = shfl2(f, L.base + q);
  const Fp2 x1 = shfl2(f, L.base + q + 3);
  const Fp2 x01 = f2_add(x0, x1);
  Fp own[3];
  own[0] = lo ? fp_mul(fp_addl(x0.c0, x0.c1), fp_subl(x0.c0, x0.c1)) : fp_mul(x0.c0, x0.c1);
  own[1] = lo ? fp_mul(fp_addl(x1.c0, x1.c1), fp_subl(x1.c0, x1.c1)) : fp_mul(x1.c0, x1.c1);
  own[2] = lo ? fp_mul(fp_addl(x01.c0, x01.c1), fp_subl(x01.c0, x01.c1)) : fp_mul(x01.c0, x01.c1);
  const int partner = lo ? L.k + 3 : L.k - 3;
  Fp2 S[3];
#pragma unroll
  for (int z = 0; z < 3; z++) {
    const Fp other = shfl_fp(own[z], L.base + partner);
    const Fp c0 = lo ? own[z] : other;
    const Fp c1h = lo ? other : own[z];
    S[z] = {c0, fp_add(c1h, c1h)};
  }
  // (x0 + x1 t)^2 = (S0 + xi S1) + (S01 - S0 - S1) t
  const Fp2 r0 = f2_add(S[0], f2_mul_xi(S[1]));
  const Fp2 r1 = f2_sub(f2_sub(S[2], S[0]), S[1]);
  // A' = 3A^2 - 2conj(A) -> k 0, 3 ; B' = 3tC^2 + 2conj(B) -> k 1, 4 ; C' = 3B^2 - 2conj(C) -> k 2, 5
  const Fp2 e = (L.k == 2 || L.k == 4) ? r1 : r0;     // exported: lane 1 B0, 2 C1, 4 B1, 5 C0
  const int src_tab = 0x453120;                        // k -> source lane: 0,2,1,3,5,4 (nibbles)
  const int src = (src_tab >> (4 * L.k)) & 0xf;
  const Fp2 got = shfl2(e, L.base + src);
  Fp2 val = (L.k == 0) ? r0 : ((L.k == 3) ? r1 : got);
  if (L.k == 1) val = f2_mul_xi(val);
  const int sgn = (L.k == 0 || L.k == 2 || L.k == 4) ? -2 : 2;
  return f2_red(f2_lin(3, val, sgn, f));
}

// Frobenius f -> f^(p^e), e in {1, 2}: f_k -> (conj^e f_k) gamma_{e,k}
__constant__ uint32_t FROB_TAB[2][6][2][NL];

__device__ __forceinline__ Fp2 lc_frob(const Fp2& f, const Lane& L, int e) {
  Fp2 g;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    g.c0.l[i] = (int32_t)FROB_TAB[e - 1][L.k][0][i];
    g.c1.l[i] = (int32_t)FROB_TAB[e - 1][L.k][1][i];
  }
  const Fp2 x = (e & 1) ? f2_conj(f) : f;
  return f2_red(f2_mul(x, g));
}

// ------------------------------------------------------------------ kernels
struct LineC {
  Fp2 c0, c1, c4;
};
// line words: c0.c0 c0.c1 c1.c0 c1.c1 c4.c0 c4.c1 (14 each), int4 chunks strided by point
__device__ __forceinline__ LineC load_line(const int4* __restrict__ coef, int stride, int step, int pt) {
  int32_t w[LINE_WORDS];
#pragma unroll
  for (int q = 0; q < LINE_WORDS / 4; q++) {
    const int4 v = coef[((size_t)step * (LINE_WORDS / 4) + q) * stride + pt];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
  LineC l;
#pragma unroll
  for (int j = 0; j < NL; j++) {
    l.c0.c0.l[j] = w[0 * NL + j];
    l.c0.c1.l[j] = w[1 * NL + j];
    l.c1.c0.l[j] = w[2 * NL + j];
    l.c1.c1.l[j] = w[3 * NL + j];
    l.c4.c0.l[j] = w[4 * NL + j];
    l.c4.c1.l[j] = w[5 * NL + j];
  }
  return l;
}

struct MillerPair {
  Fp x, y;
  bool act;
  const int4* coef;
  int stride;
  int q;
};

__device__ __forceinline__ Fp2 lc_line(const Fp2& f, const Lane& L, const MillerPair& P, int step) {
  const LineC l = load_line(P.coef, P.stride, step, P.q);
  const Fp2& c0 = l.c0;
  const Fp2& c1 = l.c1;
  const Fp2& c4 = l.c4;
  // c1 * xP, c4 * yP: the 4 Fp products split over lanes 0..3, broadcast to the group
  const Fp& a = (L.k == 0) ? c1.c0 : (L.k == 1) ? c1.c1 : (L.k == 2) ? c4.c0 : c4.c1;
  const Fp& s = (L.k < 2) ? P.x : P.y;
  const Fp pr = fp_mul(a, s);
  const Fp2 c1x = {shfl_fp(pr, L.base + 0), shfl_fp(pr, L.base + 1)};
  const Fp2 c4y = {shfl_fp(pr, L.base + 2), shfl_fp(pr, L.base + 3)};
  return lc_mul014(f, L, f2_sel(P.act, c0, f2_one()), f2_sel(P.act, c1x, f2_zero()), f2_sel(P.act, c4y, f2_zero()));
}

__global__ void __launch_bounds__(256, HBS_LB_MILLER) k_lc_miller(int n, const uint32_t* __restrict__ p1, const int4* __restrict__ coef1,
                                                   int stride1, const uint8_t* __restrict__ inf1,
                                                   const uint32_t* __restrict__ idx1, const uint32_t* __restrict__ p2,
                                                   const int4* __restrict__ coef2, int stride2,
                                                   const uint8_t* __restrict__ inf2, const uint32_t* __restrict__ idx2,
                                                   int flags, int32_t* __restrict__ fout, size_t lstride) {
  const Lane L = lane_ids(n);
  const int c = L.valid ? L.check : 0;  // idle lanes shadow check 0 and never store
  MillerPair A, B;
  A.x = fp_from_words(p1 + (size_t)c * 24);
  A.y = fp_from_words(p1 + (size_t)c * 24 + 12);
  B.x = fp_from_words(p2 + (size_t)c * 24);
  B.y = fp_from_words(p2 + (size_t)c * 24 + 12);
  bool pinf1 = true, pinf2 = true;
  for (int w = 0; w < 24; w++) {
    pinf1 &= p1[(size_t)c * 24 + w] == 0;
    pinf2 &= p2[(size_t)c * 24 + w] == 0;
  }
  if (flags & 1) B.y = fp_neg(B.y);
  A.q = idx1 ? (int)idx1[c] : c;
  B.q = idx2 ? (int)idx2[c] : c;
  A.act = !pinf1 && !inf1[A.q];
  B.act = !pinf2 && !inf2[B.q];
  A.coef = coef1;
  A.stride = stride1;
  B.coef = coef2;
  B.stride = stride2;
  Fp2 f = (L.k == 0) ? f2_one() : f2_zero();
  int step = 0;
  for (int b = 62; b >= 0; b--) {
    if (b != 62) f = lc_sqr(f, L);
    f = lc_line(f, L, A, step);
    f = lc_line(f, L, B, step);
    step++;
    if ((X_ABS >> b) & 1) {
      f = lc_line(f, L, A, step);
      f = lc_line(f, L, B, step);
      step++;
    }
  }
  if (flags & 2) f = lc_conj(f, L);
  if (L.valid) st2(fout, lstride, (size_t)L.check * GL + L.k, f);
}

// f2 = f^((p^6 - 1)(p^2 + 1)); f^-1 = (a - b w) / (a^2 - v b^2) with a = (f0, f2, f4), b = (f1, f3, f5)
__global__ void __launch_bounds__(256) k_lc_easy(int n, const int32_t* __restrict__ fin, int32_t* __restrict__ fout,
                                                 size_t lstride) {
  const Lane L = lane_ids(n);
  const size_t gl = (size_t)(L.valid ? L.check : 0) * GL + L.k;
  const Fp2 f = ld2(fin, lstride, gl);
  // lanes 0-2: (a^2)_m, lanes 3-5: (b^2)_m
  const int par = L.k >= 3 ? 1 : 0;
  const int m = L.k - 3 * par;
  Fp2 acc = f2_zero();
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const int j = (m - i + 3) % 3;
    const Fp2 x = shfl2(f, L.base + 2 * i + par);
    const Fp2 y = shfl2(f, L.base + 2 * j + par);
    Fp2 p = f2_mul(x, y);
    if (i > m) p = f2_mul_xi(p);
    acc = f2_add(acc, p);
  }
  acc = f2_red(acc);
  // N = a^2 - v b^2, every lane gets N0..N2 (v b^2 = (xi B2, B0, B1))
  Fp2 N[3];
#pragma unroll
  for (int t = 0; t < 3; t++) {
    Fp2 vb = shfl2(acc, L.base + (t == 0 ? 5 : 3 + t - 1));
    if (t == 0) vb = f2_mul_xi(vb);
    N[t] = f2_red(f2_sub(shfl2(acc, L.base + t), vb));
  }
  // Fp6 inverse of N (redundantly in every lane)
  const Fp2 i0 = f2_red(f2_sub(f2_sqr(N[0]), f2_mul_xi(f2_mul(N[1], N[2]))));
  const Fp2 i1 = f2_red(f2_sub(f2_mul_xi(f2_sqr(N[2])), f2_mul(N[0], N[1])));
  const Fp2 i2 = f2_red(f2_sub(f2_sqr(N[1]), f2_mul(N[0], N[2])));
  const Fp2 tt = f2_red(f2_add(f2_mul(N[0], i0), f2_mul_xi(f2_add(f2_mul(N[2], i1), f2_mul(N[1], i2)))));
  const Fp2 ti = f2_red(f2_inv(tt));
  const Fp2 inv[3] = {f2_red(f2_mul(i0, ti)), f2_red(f2_mul(i1, ti)), f2_red(f2_mul(i2, ti))};
  // f^-1: even k = 2m: (a N^-1)_m ; odd k = 2m+1: -(b N^-1)_m
  const int pk = L.k & 1;
  const int mk = L.k >> 1;
  Fp2 fi = f2_zero();
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const int j = (mk - i + 3) % 3;
    const Fp2 x = shfl2(f, L.base + 2 * i + pk);
    const Fp2& y = (j == 0) ? inv[0] : (j == 1) ? inv[1] : inv[2];
    Fp2 p = f2_mul(x, y);
    if (i > mk) p = f2_mul_xi(p);
    fi = f2_add(fi, p);
  }
  fi = f2_red(pk ? f2_neg(fi) : fi);
  const Fp2 f1 = lc_mul(lc_conj(f, L), fi, L);      // f^(p^6 - 1)
  const Fp2 r = lc_mul(lc_frob(f1, L, 2), f1, L);   // ^(p^2 + 1)
  if (L.valid) st2(fout, lstride, gl, r);
}

// out = conj(in^|x|) = in^x   or   conj(in^(|x|+1)) = in^(x-1)
__global__ void __launch_bounds__(256, HBS_LB_EXP) k_lc_exp(int n, const int32_t* __restrict__ fin, int32_t* __restrict__ fout,
                                                size_t lstride, int plus1) {
  const Lane L = lane_ids(n);
  const size_t gl = (size_t)(L.valid ? L.check : 0) * GL + L.k;
  const Fp2 base = ld2(fin, lstride, gl);
  const uint64_t e = plus1 ? X_ABS + 1 : X_ABS;
  Fp2 r = base;
  for (int i = 62; i >= 0; i--) {
    r = lc_cyclo_sqr(r, L);
    if ((e >> i) & 1) r = lc_mul(r, base, L);
  }
  r = lc_conj(r, L);
  if (L.valid) st2(fout, lstride, gl, r);
}

// mode 1: out = t * frob1(a) ; mode 2: out = t * frob2(a) * conj(a)
__global__ void __launch_bounds__(256) k_lc_glue(int n, const int32_t* __restrict__ t, const int32_t* __restrict__ a,
                                                 int32_t* __restrict__ fout, size_t lstride, int mode) {
  const Lane L = lane_ids(n);
  const size_t gl = (size_t)(L.valid ? L.check : 0) * GL + L.k;
  const Fp2 av = ld2(a, lstride, gl);
  Fp2 r = lc_mul(ld2(t, lstride, gl), lc_frob(av, L, mode), L);
  if (mode == 2) r = lc_mul(r, lc_conj(av, L), L);
  if (L.valid) st2(fout, lstride, gl, r);
}

// e = c * f2^3 ; verdict = (e == 1) or the canonical value words (debug)
__global__ void __launch_bounds__(256) k_lc_verdict(int n, const int32_t* __restrict__ c, const int32_t* __restrict__ f2,
                                                    size_t lstride, uint8_t* __restrict__ verdict,
                                                    uint32_t* __restrict__ value_out) {
  const Lane L = lane_ids(n);
  const size_t gl = (size_t)(L.valid ? L.check : 0) * GL + L.k;
  const Fp2 g = ld2(f2, lstride, gl);
  const Fp2 e = lc_mul(ld2(c, lstride, gl), lc_mul(lc_cyclo_sqr(g, L), g, L), L);
  if (value_out) {
    // tower storage order: c0.c0 (k0), c0.c1 (k2), c0.c2 (k4), c1.c0 (k1), c1.c1 (k3), c1.c2 (k5)
    const int slot = (L.k & 1) ? 3 + (L.k >> 1) : (L.k >> 1);
    if (L.valid) {
      uint32_t* o = value_out + (size_t)L.check * 144 + 24 * slot;
      fp_to_words(e.c0, o);
      fp_to_words(e.c1, o + 12);
    }
    return;
  }
  const bool ok = (L.k == 0) ? (fp_is_zero(fp_sub(e.c0, fp_one())) && fp_is_zero(e.c1)) : f2_is_zero(e);
  int all = ok ? 1 : 0;
#pragma unroll
  for (int j = 0; j < GL; j++) all &= __shfl(ok ? 1 : 0, L.base + j, 64);
  if (L.valid && L.k == 0) verdict[L.check] = (uint8_t)all;
}

}  // namespace hbs

// ------------------------------------------------------------------ host launchers
namespace hbl {

static inline dim3 lc_grid(int n) {
  const int waves = (n + hbs::CPW - 1) / hbs::CPW;
  return dim3((unsigned)((waves + 3) / 4));  // 4 waves (256 threads) per block
}
size_t lc_lstride(int n) { return (size_t)((n + 63) / 64 * 64) * hbs::GL; }
size_t lc_state_words(int n) { return (size_t)hbs::F2W * lc_lstride(n); }

hipError_t lc_init_constants() {
  static bool done = false;
  if (done) return hipSuccess;
  uint32_t tab[2][6][2][hb::NL];
  const uint32_t* c1[6][2] = {{hb::FROB1_0_C0, hb::FROB1_0_C1}, {hb::FROB1_1_C0, hb::FROB1_1_C1},
                              {hb::FROB1_2_C0, hb::FROB1_2_C1}, {hb::FROB1_3_C0, hb::FROB1_3_C1},
                              {hb::FROB1_4_C0, hb::FROB1_4_C1}, {hb::FROB1_5_C0, hb::FROB1_5_C1}};
  const uint32_t* c2[6][2] = {{hb::FROB2_0_C0, hb::FROB2_0_C1}, {hb::FROB2_1_C0, hb::FROB2_1_C1},
                              {hb::FROB2_2_C0, hb::FROB2_2_C1}, {hb::FROB2_3_C0, hb::FROB2_3_C1},
                              {hb::FROB2_4_C0, hb::FROB2_4_C1}, {hb::FROB2_5_C0, hb::FROB2_5_C1}};
  for (int k = 0; k < 6; k++)
    for (int h = 0; h < 2; h++)
      for (int i = 0; i < hb::NL; i++) {
        tab[0][k][h][i] = c1[k][h][i];
        tab[1][k][h][i] = c2[k][h][i];
      }
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(hbs::FROB_TAB), tab, sizeof(tab));
  if (e == hipSuccess) done = true;
  return e;
}

hipError_t lc_pairing(hipStream_t s, int n, const void* p1, const void* coef1, int nq1, const uint8_t* inf1,
                      const uint32_t* idx1, const void* p2, const void* coef2, int nq2, const uint8_t* inf2,
                      const uint32_t* idx2, int flags, int32_t* w0, int32_t* w1, int32_t* w2, int32_t* w3,
                      uint8_t* verdict, uint32_t* value_out) {
  if (n <= 0) return hipSuccess;
  hipError_t e = lc_init_constants();
  if (e != hipSuccess) return e;
  const dim3 g = lc_grid(n), b(256);
  const size_t ls = lc_lstride(n);
  hipLaunchKernelGGL(hbs::k_lc_miller, g, b, 0, s, n, (const uint32_t*)p1, (const int4*)coef1, pad64(nq1), inf1, idx1,
                     (const uint32_t*)p2, (const int4*)coef2, pad64(nq2), inf2, idx2, flags, w0, ls);
  hipLaunchKernelGGL(hbs::k_lc_easy, g, b, 0, s, n, (const int32_t*)w0, w1, ls);                    // f2 -> w1
  hipLaunchKernelGGL(hbs::k_lc_exp, g, b, 0, s, n, (const int32_t*)w1, w2, ls, 1);                  // t = f2^(x-1)
  hipLaunchKernelGGL(hbs::k_lc_exp, g, b, 0, s, n, (const int32_t*)w2, w3, ls, 1);                  // a = t^(x-1)
  hipLaunchKernelGGL(hbs::k_lc_exp, g, b, 0, s, n, (const int32_t*)w3, w2, ls, 0);                  // t = a^x
  hipLaunchKernelGGL(hbs::k_lc_glue, g, b, 0, s, n, (const int32_t*)w2, (const int32_t*)w3, w0, ls, 1);  // b
  hipLaunchKernelGGL(hbs::k_lc_exp, g, b, 0, s, n, (const int32_t*)w0, w2, ls, 0);                  // t = b^x
  hipLaunchKernelGGL(hbs::k_lc_exp, g, b, 0, s, n, (const int32_t*)w2, w3, ls, 0);                  // t = t^x
  hipLaunchKernelGGL(hbs::k_lc_glue, g, b, 0, s, n, (const int32_t*)w3, (const int32_t*)w0, w2, ls, 2);  // c
  hipLaunchKernelGGL(hbs::k_lc_verdict, g, b, 0, s, n, (const int32_t*)w2, (const int32_t*)w1, ls, verdict, value_out);
  return hipGetLastError();
}

}  // namespace hbl
