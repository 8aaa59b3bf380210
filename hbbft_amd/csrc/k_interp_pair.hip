// Latency form of the G2 Lagrange combine (PublicKeySet::combine_signatures,
// src/threshold_sign.rs:249-259, for the one document of combine_and_verify_sig): the curve work of
// k_interp_endo on LANE QUADS.  Two lanes hold the c0 / c1 components of every Fp2 coordinate
// (pfp.hpp), so each Fp2 product is one lane-pair product; two lane pairs (a quad) hold the same
// point and split each group operation's independent products between them, trading results with
// one DPP quad permute per limb: a doubling is 4 product rounds instead of 7 serial products, a
// mixed addition 6 instead of 11, a general addition 9 instead of 16.  The work split is the one
// of k_interp_endo: term (k, j) = digit chunk s of GLS digit j of lambda_k(0) times psi^j(P_k)
// (sign (-1)^j), 32-bit chunks, one quad per (chunk, term).  One workgroup per (combine, chunk,
// half of the terms): an LDS tree sums its terms, the chunk-1 workgroups scale their sums by 2^32
// (Horner), and k_interp_join adds the four partial sums and writes the affine result.  Formulas:
// dbl-2009-l, add-2007-bl, madd-2007-bl (curve.hpp) -- the same group law, so the affine output is
// byte-identical to the C oracle's.  Digits come from the host or k_interp_digits (k_curve.hip).
#define HS_MULFN static __device__ __noinline__
#include "interp_pair.hpp"
#include "launch.hpp"
#include "pfp.hpp"
#include "words.hpp"

namespace hbs {

constexpr int IP_THREADS = 256;          // one workgroup per (combine, chunk, half): 64 lane quads
constexpr int IP_NCHUNK = 2;             // 32-bit chunks of the 64-bit digits
constexpr int IP_NHALF = 2;              // workgroups per chunk (terms interleaved between them)
constexpr int IP_WG = IP_NCHUNK * IP_NHALF;
constexpr int IP_Q = IP_THREADS / 4;     // lane quads per workgroup (power of two)
constexpr int IP_WORDS = 3 * NL;         // one lane's Jacobian point (x, y, z own components)
constexpr int DPP_XQ = 0x4E;             // quad_perm [2,3,0,1]: the other lane pair, same component

HP_D bool hj_is_zero(const HJac& p) { return h_is_zero(p.z); }
HP_D HJac hj_zero() { return {h_one(), h_one(), h_zero()}; }
HP_D HJac hj_reduce(const HJac& p) { return {fp_reduce(p.x), fp_reduce(p.y), fp_reduce(p.z)}; }

// dbl-2009-l; inputs |.| < 2p, outputs reduced
HP_D HJac hj_dbl(const HJac& p) {
  const Fp A = h_sqr(p.x);
  const Fp B = h_sqr(p.y);
  const Fp C = h_sqr(B);
  const Fp D = fp_reduce(fp_lin(2, fp_sub(fp_sub(h_sqr(fp_add(p.x, B)), A), C), 0, C));
  const Fp E = fp_lin(3, A, 0, A);
  const Fp F = h_sqr(E);
  HJac r;
  r.x = fp_reduce(fp_sub(F, fp_add(D, D)));
  r.y = fp_reduce(fp_sub(h_mul(E, fp_sub(D, r.x)), fp_lin(8, C, 0, C)));
  const Fp yz = h_mul(p.y, p.z);
  r.z = fp_reduce(fp_add(yz, yz));
  return r;
}

// add-2007-bl (general), exceptional cases as curve.hpp jac_add; conditions are pair-uniform
HP_D HJac hj_add(const HJac& p, const HJac& q) {
  if (hj_is_zero(p)) return q;
  if (hj_is_zero(q)) return p;
  const Fp Z1Z1 = h_sqr(p.z);
  const Fp Z2Z2 = h_sqr(q.z);
  const Fp U1 = h_mul(p.x, Z2Z2);
  const Fp U2 = h_mul(q.x, Z1Z1);
  const Fp S1 = h_mul(h_mul(p.y, q.z), Z2Z2);
  const Fp S2 = h_mul(h_mul(q.y, p.z), Z1Z1);
  const Fp H = fp_reduce(fp_sub(U2, U1));
  const Fp rr = fp_reduce(fp_lin(2, S2, -2, S1));
  if (h_is_zero(H)) {
    if (h_is_zero(rr)) return hj_dbl(p);
    return hj_zero();
  }
  const Fp I = h_sqr(fp_add(H, H));
  const Fp J = h_mul(H, I);
  const Fp V = h_mul(U1, I);
  HJac r;
  r.x = fp_reduce(fp_sub(fp_sub(h_sqr(rr), J), fp_add(V, V)));
  const Fp SJ = h_mul(S1, J);
  r.y = fp_reduce(fp_sub(h_mul(rr, fp_sub(V, r.x)), fp_add(SJ, SJ)));
  r.z = fp_reduce(h_mul(fp_sub(fp_sub(h_sqr(fp_add(p.z, q.z)), Z1Z1), Z2Z2), H));
  return r;
}

// madd-2007-bl: p + (x2, y2), the affine point not infinity
HP_D HJac hj_add_affine(const HJac& p, const Fp& x2, const Fp& y2) {
  if (hj_is_zero(p)) return {x2, y2, h_one()};
  const Fp Z1Z1 = h_sqr(p.z);
  const Fp U2 = h_mul(x2, Z1Z1);
  const Fp S2 = h_mul(h_mul(y2, p.z), Z1Z1);
  const Fp H = fp_reduce(fp_sub(U2, p.x));
  const Fp rr = fp_reduce(fp_lin(2, S2, -2, p.y));
  if (h_is_zero(H)) {
    if (h_is_zero(rr)) return hj_dbl(p);
    return hj_zero();
  }
  const Fp HH = h_sqr(H);
  const Fp I = fp_lin(4, HH, 0, HH);
  const Fp J = h_mul(H, I);
  const Fp V = h_mul(p.x, I);
  HJac r;
  r.x = fp_reduce(fp_sub(fp_sub(h_sqr(rr), J), fp_add(V, V)));
  const Fp YJ = h_mul(p.y, J);
  r.y = fp_reduce(fp_sub(h_mul(rr, fp_sub(V, r.x)), fp_add(YJ, YJ)));
  r.z = fp_reduce(fp_sub(fp_sub(h_sqr(fp_add(p.z, H)), Z1Z1), HH));
  return r;
}

// k * (x, y) for a 32-bit k, double-and-add from the top set bit (jac_mul_affine)
HP_D HJac hj_mul_affine(const Fp& x, const Fp& y, bool inf, uint32_t k) {
  HJac acc = hj_zero();
  if (inf || k == 0) return acc;
  const int top = 31 - __builtin_clz(k);
  acc = {x, y, h_one()};
#pragma unroll 1
  for (int i = top - 1; i >= 0; i--) {
    acc = hj_dbl(acc);
    if ((k >> i) & 1) acc = hj_add_affine(acc, x, y);
  }
  return acc;
}

// ---------------------------------------------------------------- lane quads
// A quad's two lane pairs hold the same values; in a round pair 0 forms a0 * b0 and pair 1 a1 * b1
// (or squares), and both end with both products.  Conditions below are quad-uniform.
HP_D bool q_hi() { return (threadIdx.x & 2) != 0; }
HP_D void q_mul(const Fp& a0, const Fp& b0, const Fp& a1, const Fp& b1, Fp& r0, Fp& r1) {
  const bool q = q_hi();
  const Fp r = h_mul(fp_sel(q, a1, a0), fp_sel(q, b1, b0));
  const Fp o = dpp_fp<DPP_XQ>(r);
  r0 = fp_sel(q, o, r);
  r1 = fp_sel(q, r, o);
}
HP_D void q_sqr(const Fp& a0, const Fp& a1, Fp& r0, Fp& r1) {
  const bool q = q_hi();
  const Fp r = h_sqr(fp_sel(q, a1, a0));
  const Fp o = dpp_fp<DPP_XQ>(r);
  r0 = fp_sel(q, o, r);
  r1 = fp_sel(q, r, o);
}

// hj_dbl in 4 rounds
HP_D HJac qj_dbl(const HJac& p) {
  Fp A, B, C, F, XB2, YZ;
  q_sqr(p.x, p.y, A, B);
  const Fp E = fp_lin(3, A, 0, A);
  q_sqr(B, E, C, F);
  q_mul(fp_add(p.x, B), fp_add(p.x, B), p.y, p.z, XB2, YZ);
  const Fp D = fp_reduce(fp_lin(2, fp_sub(fp_sub(XB2, A), C), 0, C));
  HJac r;
  r.x = fp_reduce(fp_sub(F, fp_add(D, D)));
  r.y = fp_reduce(fp_sub(h_mul(E, fp_sub(D, r.x)), fp_lin(8, C, 0, C)));
  r.z = fp_reduce(fp_add(YZ, YZ));
  return r;
}

// hj_add_affine in 6 rounds (Z3 = 2 Z1 H, the same value as (Z1 + H)^2 - Z1Z1 - HH)
HP_D HJac qj_add_affine(const HJac& p, const Fp& x2, const Fp& y2) {
  if (hj_is_zero(p)) return {x2, y2, h_one()};
  Fp Z1Z1, YZ, U2, S2;
  q_mul(p.z, p.z, y2, p.z, Z1Z1, YZ);
  q_mul(x2, Z1Z1, YZ, Z1Z1, U2, S2);
  const Fp H = fp_reduce(fp_sub(U2, p.x));
  const Fp rr = fp_reduce(fp_lin(2, S2, -2, p.y));
  if (h_is_zero(H)) {
    if (h_is_zero(rr)) return qj_dbl(p);
    return hj_zero();
  }
  Fp HH, RR, J, V, EV, YJ;
  q_sqr(H, rr, HH, RR);
  const Fp I = fp_lin(4, HH, 0, HH);
  q_mul(H, I, p.x, I, J, V);
  HJac r;
  r.x = fp_reduce(fp_sub(fp_sub(RR, J), fp_add(V, V)));
  q_mul(rr, fp_sub(V, r.x), p.y, J, EV, YJ);
  r.y = fp_reduce(fp_sub(EV, fp_add(YJ, YJ)));
  const Fp ZH = h_mul(p.z, H);
  r.z = fp_reduce(fp_add(ZH, ZH));
  return r;
}

// hj_add in 9 rounds (Z3 = 2 Z1 Z2 H)
HP_D HJac qj_add(const HJac& p, const HJac& q) {
  if (hj_is_zero(p)) return q;
  if (hj_is_zero(q)) return p;
  Fp Z1Z1, Z2Z2, U1, U2, YZ1, YZ2, S1, S2;
  q_sqr(p.z, q.z, Z1Z1, Z2Z2);
  q_mul(p.x, Z2Z2, q.x, Z1Z1, U1, U2);
  q_mul(p.y, q.z, q.y, p.z, YZ1, YZ2);
  q_mul(YZ1, Z2Z2, YZ2, Z1Z1, S1, S2);
  const Fp H = fp_reduce(fp_sub(U2, U1));
  const Fp rr = fp_reduce(fp_lin(2, S2, -2, S1));
  if (h_is_zero(H)) {
    if (h_is_zero(rr)) return qj_dbl(p);
    return hj_zero();
  }
  Fp I, RR, J, V, EV, SJ, Z12, ZH;
  q_sqr(fp_add(H, H), rr, I, RR);
  q_mul(H, I, U1, I, J, V);
  HJac r;
  r.x = fp_reduce(fp_sub(fp_sub(RR, J), fp_add(V, V)));
  q_mul(rr, fp_sub(V, r.x), S1, J, EV, SJ);
  r.y = fp_reduce(fp_sub(EV, fp_add(SJ, SJ)));
  Z12 = h_mul(p.z, q.z);
  ZH = h_mul(Z12, H);
  r.z = fp_reduce(fp_add(ZH, ZH));
  return r;
}

HP_D HJac qj_mul_affine(const Fp& x, const Fp& y, bool inf, uint32_t k) {
  HJac acc = hj_zero();
  if (inf || k == 0) return acc;
  const int top = 31 - __builtin_clz(k);
  acc = {x, y, h_one()};
#pragma unroll 1
  for (int i = top - 1; i >= 0; i--) {
    acc = qj_dbl(acc);
    if ((k >> i) & 1) acc = qj_add_affine(acc, x, y);
  }
  return acc;
}

// psi on own components: psi(x) = conj(x) * (0 + c u) -> (x1 c, x0 c); psi(y) = conj(y) * c2
HP_D Fp psi_xh(const Fp& x) { return fp_reduce(fp_mul(dpp_fp<DPP_SWAP>(x), fp_const(hb::PSI_C1_C1))); }
HP_D Fp psi_yh(const Fp& y) { return fp_reduce(h_mul(h_conj(y), h_const(hb::PSI_C2_C0, hb::PSI_C2_C1))); }

HP_D void lds_put(uint32_t* s, const HJac& p) {
#pragma unroll
  for (int i = 0; i < NL; i++) {
    s[i] = (uint32_t)p.x.l[i];
    s[NL + i] = (uint32_t)p.y.l[i];
    s[2 * NL + i] = (uint32_t)p.z.l[i];
  }
}
HP_D HJac lds_get(const uint32_t* s) {
  HJac p;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    p.x.l[i] = (int32_t)s[i];
    p.y.l[i] = (int32_t)s[NL + i];
    p.z.l[i] = (int32_t)s[2 * NL + i];
  }
  return p;
}

// Workgroup (c, chunk, half): every other term of the chunk on 64 lane quads (4 waves, one per
// SIMD), an LDS tree, then quad 0 scales a chunk-1 sum by 2^32 (Horner) and writes the partial sum.
__global__ void __launch_bounds__(IP_THREADS) k_interp_pair(int ncomb, int m, const uint64_t* __restrict__ digits,
                                                            const uint32_t* __restrict__ pts, int32_t* __restrict__ part) {
  extern __shared__ uint32_t sm[];  // IP_Q quads x 2 lanes x IP_WORDS
  const int c = blockIdx.x / IP_WG, chunk = (blockIdx.x / IP_NHALF) % IP_NCHUNK, half = blockIdx.x % IP_NHALF;
  if (c >= ncomb) return;  // uniform per workgroup
  const int g = threadIdx.x >> 2, h = threadIdx.x & 1;
  HJac acc = hj_zero();
  for (int t = half + IP_NHALF * g; t < m * 4; t += IP_NHALF * IP_Q) {
    const int k = t >> 2, j = t & 3;
    const uint32_t* w = pts + ((size_t)c * m + k) * 48;
    const bool inf = lp_both(words_zero(w + (lp_even() ? 0 : 12), 12) && words_zero(w + (lp_even() ? 24 : 36), 12));
    Fp x, y;
    h_g2_load(w, x, y);
    for (int s = 0; s < j; s++) {
      x = psi_xh(x);
      y = psi_yh(y);
    }
    if (j & 1) y = fp_neg(y);
    const uint64_t d = digits[((size_t)c * m + k) * 4 + j];
    const uint32_t kc = (uint32_t)(d >> (32 * chunk));
    acc = qj_add(acc, qj_mul_affine(x, y, inf, kc));
  }
  uint32_t* mine = sm + (size_t)(g * 2 + h) * IP_WORDS;
  if (!q_hi()) lds_put(mine, acc);
  __syncthreads();
  for (int s = IP_Q / 2; s > 0; s >>= 1) {
    if (g < s) {
      acc = qj_add(lds_get(mine), lds_get(sm + (size_t)((g + s) * 2 + h) * IP_WORDS));
    }
    __syncthreads();
    if (g < s && !q_hi()) lds_put(mine, acc);
    __syncthreads();
  }
  if (g != 0) return;
  HJac r = lds_get(sm + (size_t)h * IP_WORDS);
  if (chunk == 1) {
#pragma unroll 1
    for (int b = 0; b < 32; b++) r = qj_dbl(r);
  }
  if (!q_hi()) lds_put((uint32_t*)part + ((size_t)blockIdx.x * 2 + h) * IP_WORDS, r);
}

// out[c] = affine(sum of the four partial sums): one lane quad per combine
__global__ void __launch_bounds__(64) k_interp_join(int ncomb, const int32_t* __restrict__ part,
                                                    uint32_t* __restrict__ out) {
  const int c = (int)((blockIdx.x * 64u + threadIdx.x) >> 2);
  if (c >= ncomb) return;
  const int h = threadIdx.x & 1;
  const uint32_t* p = (const uint32_t*)part + (size_t)c * IP_WG * 2 * IP_WORDS;
  HJac s1 = qj_add(lds_get(p + (size_t)(2 * 2 + h) * IP_WORDS), lds_get(p + (size_t)(3 * 2 + h) * IP_WORDS));
  HJac s0 = qj_add(lds_get(p + (size_t)(0 * 2 + h) * IP_WORDS), lds_get(p + (size_t)(1 * 2 + h) * IP_WORDS));
  HJac r = qj_add(s1, s0);
  uint32_t* o = out + (size_t)c * 48 + (lp_even() ? 0 : 12);
  if (hj_is_zero(r)) {
    if (!q_hi()) {
#pragma unroll
      for (int i = 0; i < 12; i++) {
        o[i] = 0u;
        o[24 + i] = 0u;
      }
    }
    return;
  }
  const Fp zi = h_inv_vartime(fp_reduce(r.z));
  const Fp zi2 = h_sqr(zi);
  Fp xa, zi3;
  q_mul(r.x, zi2, zi2, zi, xa, zi3);
  const Fp ya = h_mul(r.y, zi3);
  if (!q_hi()) {
    fp_to_words(xa, o);
    fp_to_words(ya, o + 24);
  }
}

}  // namespace hbs

namespace hbl {

bool interp_g2_pair_fits(int m) { return m >= 1 && m <= 512; }

size_t interp_g2_pair_part_bytes(int ncomb) { return (size_t)ncomb * hbs::IP_WG * 2 * hbs::IP_WORDS * 4; }

hipError_t interp_g2_pair(hipStream_t s, int ncomb, int m, const uint64_t* digits, const void* pts, void* part,
                          void* out) {
  if (ncomb <= 0) return hipSuccess;
  const size_t lds = (size_t)hbs::IP_Q * 2 * hbs::IP_WORDS * 4;
  hipLaunchKernelGGL(hbs::k_interp_pair, dim3((unsigned)ncomb * hbs::IP_WG), dim3(hbs::IP_THREADS), lds, s, ncomb, m,
                     digits, (const uint32_t*)pts, (int32_t*)part);
  hipLaunchKernelGGL(hbs::k_interp_join, dim3((unsigned)((4 * ncomb + 63) / 64)), dim3(64), 0, s, ncomb,
                     (const int32_t*)part, (uint32_t*)out);
  return hipGetLastError();
}

}  // namespace hbl
