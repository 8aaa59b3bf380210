// BivarCommitment::evaluate(x, y) == g1 * val for SyncKeyGen Ack checks (src/sync_key_gen.rs:542)
// on LANE QUADS (gfx950).
//
// One node checks ~N^2 acks at once, each a serial G1 chain: the Horner evaluation of the row
// polynomial at the small y (t + 1 steps of a 7-bit double-and-add plus a mixed addition) and g1 *
// val from the comb table.  10,000 acks are 0.15 waves per SIMD with one lane per ack, so the chain
// length is the time.  Here four lanes hold the same point and split every group operation's
// independent Fp products between them, one product per lane per round, exchanging results with DPP
// quad broadcasts: a doubling takes 3 rounds instead of 7 serial products, a mixed or general
// addition 5 instead of 11 / 16.  The rows R = row(x) come from k_bivar_row_quad in Jacobian form
// (no inversion per row element).  g1 * val: each lane adds its quarter of the 32 comb windows on
// its own, then the quad joins the four partial sums.  Formulas: dbl-2009-l, madd-2007-bl, add-2007-bl
// (the group law of curve.hpp) on the signed-limb Fp of sfp.hpp; the verdict is point equality, so
// it is the one of k_bivar_check.
#include "interp_pair.hpp"
#include "launch.hpp"
#include "sfp.hpp"
#include "words.hpp"

namespace hbs {

constexpr int Q_FB_WINDOWS = 32, Q_FB_ROW = 256, Q_G1_WORDS = 24;

struct QJ {
  Fp x, y, z;
};

__device__ __forceinline__ int q_lane() { return threadIdx.x & 3; }
template <int CTRL>
__device__ __forceinline__ Fp q_dpp(const Fp& a) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = __builtin_amdgcn_mov_dpp(a.l[i], CTRL, 0xF, 0xF, true);
  return r;
}
__device__ __forceinline__ Fp q_sel4(int q, const Fp& a0, const Fp& a1, const Fp& a2, const Fp& a3) {
  return fp_sel(q == 0, a0, fp_sel(q == 1, a1, fp_sel(q == 2, a2, a3)));
}
// one round: lane k of the quad forms a_k * b_k; every lane gets all four products
__device__ __forceinline__ void q4(const Fp& a0, const Fp& b0, const Fp& a1, const Fp& b1, const Fp& a2, const Fp& b2,
                                   const Fp& a3, const Fp& b3, Fp& r0, Fp& r1, Fp& r2, Fp& r3) {
  const int q = q_lane();
  const Fp r = fp_mul(q_sel4(q, a0, a1, a2, a3), q_sel4(q, b0, b1, b2, b3));
  r0 = q_dpp<0x00>(r);
  r1 = q_dpp<0x55>(r);
  r2 = q_dpp<0xAA>(r);
  r3 = q_dpp<0xFF>(r);
}
__device__ __forceinline__ void q3(const Fp& a0, const Fp& b0, const Fp& a1, const Fp& b1, const Fp& a2, const Fp& b2,
                                   Fp& r0, Fp& r1, Fp& r2) {
  const int q = q_lane();
  const Fp r = fp_mul(q_sel4(q, a0, a1, a2, a2), q_sel4(q, b0, b1, b2, b2));
  r0 = q_dpp<0x00>(r);
  r1 = q_dpp<0x55>(r);
  r2 = q_dpp<0xAA>(r);
}
__device__ __forceinline__ void q2(const Fp& a0, const Fp& b0, const Fp& a1, const Fp& b1, Fp& r0, Fp& r1) {
  const bool odd = (q_lane() & 1) != 0;
  const Fp r = fp_mul(fp_sel(odd, a1, a0), fp_sel(odd, b1, b0));
  r0 = q_dpp<0x00>(r);
  r1 = q_dpp<0x55>(r);
}

__device__ __forceinline__ bool qj_zero(const QJ& p) { return fp_is_zero(p.z); }
__device__ __forceinline__ QJ qj_inf() { return {fp_one(), fp_one(), fp_zero()}; }

// dbl-2009-l, 3 rounds; inputs reduced, outputs reduced
__device__ __forceinline__ QJ g1q_dbl(const QJ& p) {
  Fp A, B, YZ, C, XB2, F, u;
  q3(p.x, p.x, p.y, p.y, p.y, p.z, A, B, YZ);
  const Fp E = fp_lin(3, A, 0, A);
  const Fp XB = fp_add(p.x, B);
  q3(B, B, XB, XB, E, E, C, XB2, F);
  const Fp D = fp_reduce(fp_lin(2, fp_sub(fp_sub(XB2, A), C), 0, C));
  QJ r;
  r.x = fp_reduce(fp_sub(F, fp_add(D, D)));
  u = fp_mul(E, fp_sub(D, r.x));
  r.y = fp_reduce(fp_sub(u, fp_lin(8, C, 0, C)));
  r.z = fp_reduce(fp_add(YZ, YZ));
  return r;
}

// madd-2007-bl: p + (x2, y2) with (x2, y2) affine and not infinity, 5 rounds
__device__ __forceinline__ QJ g1q_add_affine(const QJ& p, const Fp& x2, const Fp& y2) {
  if (qj_zero(p)) return {x2, y2, fp_one()};
  Fp Z1Z1, YZ, U2, S2;
  q2(p.z, p.z, y2, p.z, Z1Z1, YZ);
  q2(x2, Z1Z1, YZ, Z1Z1, U2, S2);
  const Fp H = fp_reduce(fp_sub(U2, p.x));
  const Fp rr = fp_reduce(fp_lin(2, S2, -2, p.y));
  if (fp_is_zero(H)) {
    if (fp_is_zero(rr)) return g1q_dbl(p);
    return qj_inf();
  }
  Fp HH, RR, ZH, J, V, EV, YJ;
  q3(H, H, rr, rr, p.z, H, HH, RR, ZH);
  const Fp I = fp_lin(4, HH, 0, HH);
  q2(H, I, p.x, I, J, V);
  QJ r;
  r.x = fp_reduce(fp_sub(fp_sub(RR, J), fp_add(V, V)));
  q2(rr, fp_sub(V, r.x), p.y, J, EV, YJ);
  r.y = fp_reduce(fp_sub(EV, fp_add(YJ, YJ)));
  r.z = fp_reduce(fp_add(ZH, ZH));
  return r;
}

// add-2007-bl (general), 5 rounds
__device__ __forceinline__ QJ g1q_add(const QJ& p, const QJ& q) {
  if (qj_zero(p)) return q;
  if (qj_zero(q)) return p;
  Fp Z1Z1, Z2Z2, Y1Z2, Y2Z1, U1, U2, S1, S2;
  q4(p.z, p.z, q.z, q.z, p.y, q.z, q.y, p.z, Z1Z1, Z2Z2, Y1Z2, Y2Z1);
  q4(p.x, Z2Z2, q.x, Z1Z1, Y1Z2, Z2Z2, Y2Z1, Z1Z1, U1, U2, S1, S2);
  const Fp H = fp_reduce(fp_sub(U2, U1));
  const Fp rr = fp_reduce(fp_lin(2, S2, -2, S1));
  if (fp_is_zero(H)) {
    if (fp_is_zero(rr)) return g1q_dbl(p);
    return qj_inf();
  }
  Fp I, RR, Z12, J, V, Z12H, EV, SJ;
  const Fp H2 = fp_add(H, H);
  q3(H2, H2, rr, rr, p.z, q.z, I, RR, Z12);
  q3(H, I, U1, I, Z12, H, J, V, Z12H);
  QJ r;
  r.x = fp_reduce(fp_sub(fp_sub(RR, J), fp_add(V, V)));
  q2(rr, fp_sub(V, r.x), S1, J, EV, SJ);
  r.y = fp_reduce(fp_sub(EV, fp_add(SJ, SJ)));
  r.z = fp_reduce(fp_add(Z12H, Z12H));
  return r;
}

// k * p for a small k (double-and-add from the top bit)
__device__ __forceinline__ QJ g1q_mul_small(const QJ& p, uint32_t k) {
  if (k == 0) return qj_inf();
  const int top = 31 - __builtin_clz(k);
  QJ acc = p;
#pragma unroll 1
  for (int i = top - 1; i >= 0; i--) {
    acc = g1q_dbl(acc);
    if ((k >> i) & 1) acc = g1q_add(acc, p);
  }
  return acc;
}

// P == Q as group elements, 2 rounds
__device__ __forceinline__ bool g1q_eq(const QJ& p, const QJ& q) {
  const bool pz = qj_zero(p), qz = qj_zero(q);
  if (pz || qz) return pz && qz;
  Fp Z1Z1, Z2Z2, Y1Z2, Y2Z1, a, b, c, d;
  q4(p.z, p.z, q.z, q.z, p.y, q.z, q.y, p.z, Z1Z1, Z2Z2, Y1Z2, Y2Z1);
  q4(p.x, Z2Z2, q.x, Z1Z1, Y1Z2, Z2Z2, Y2Z1, Z1Z1, a, b, c, d);
  return fp_is_zero(fp_sub(a, b)) && fp_is_zero(fp_sub(c, d));
}

__device__ __forceinline__ bool load_aff(const uint32_t* __restrict__ w, Fp& x, Fp& y) {
  uint32_t o = 0;
#pragma unroll
  for (int k = 0; k < Q_G1_WORDS; k++) o |= w[k];
  x = fp_from_words(w);
  y = fp_from_words(w + 12);
  return o == 0;
}

// single-lane mixed addition (this lane's own comb windows)
__device__ __forceinline__ QJ g1_madd_lane(const QJ& p, const Fp& x2, const Fp& y2);
__device__ __forceinline__ QJ g1_dbl_lane(const QJ& p) {
  const Fp A = fp_sqr(p.x);
  const Fp B = fp_sqr(p.y);
  const Fp C = fp_sqr(B);
  const Fp D = fp_reduce(fp_lin(2, fp_sub(fp_sub(fp_sqr(fp_add(p.x, B)), A), C), 0, C));
  const Fp E = fp_lin(3, A, 0, A);
  QJ r;
  r.x = fp_reduce(fp_sub(fp_sqr(E), fp_add(D, D)));
  r.y = fp_reduce(fp_sub(fp_mul(E, fp_sub(D, r.x)), fp_lin(8, C, 0, C)));
  const Fp yz = fp_mul(p.y, p.z);
  r.z = fp_reduce(fp_add(yz, yz));
  return r;
}
__device__ __forceinline__ QJ g1_madd_lane(const QJ& p, const Fp& x2, const Fp& y2) {
  if (qj_zero(p)) return {x2, y2, fp_one()};
  const Fp Z1Z1 = fp_sqr(p.z);
  const Fp U2 = fp_mul(x2, Z1Z1);
  const Fp S2 = fp_mul(fp_mul(y2, p.z), Z1Z1);
  const Fp H = fp_reduce(fp_sub(U2, p.x));
  const Fp rr = fp_reduce(fp_lin(2, S2, -2, p.y));
  if (fp_is_zero(H)) {
    if (fp_is_zero(rr)) return g1_dbl_lane(p);
    return qj_inf();
  }
  const Fp HH = fp_sqr(H);
  const Fp I = fp_lin(4, HH, 0, HH);
  const Fp J = fp_mul(H, I);
  const Fp V = fp_mul(p.x, I);
  QJ r;
  r.x = fp_reduce(fp_sub(fp_sub(fp_sqr(rr), J), fp_add(V, V)));
  const Fp YJ = fp_mul(p.y, J);
  r.y = fp_reduce(fp_sub(fp_mul(rr, fp_sub(V, r.x)), fp_add(YJ, YJ)));
  const Fp ZH = fp_mul(p.z, H);
  r.z = fp_reduce(fp_add(ZH, ZH));
  return r;
}

// Jacobian row points in the engine's workspace: 3 x 14 signed limbs (Montgomery), z = 0 at infinity
constexpr int Q_JROW_WORDS = 3 * NL;
__device__ __forceinline__ void qj_store(int32_t* __restrict__ o, const QJ& p) {
#pragma unroll
  for (int i = 0; i < NL; i++) {
    o[i] = p.x.l[i];
    o[NL + i] = p.y.l[i];
    o[2 * NL + i] = p.z.l[i];
  }
}
__device__ __forceinline__ QJ qj_load(const int32_t* __restrict__ o) {
  QJ p;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    p.x.l[i] = o[i];
    p.y.l[i] = o[NL + i];
    p.z.l[i] = o[2 * NL + i];
  }
  return p;
}
__device__ __forceinline__ int q_coeff_pos(int i, int j) {  // BivarCommitment's symmetric index
  return i <= j ? j * (j + 1) / 2 + i : i * (i + 1) / 2 + j;
}

// BivarCommitment::row(x)[i] = sum_j C[coeff_pos(i, j)] x^j (src/sync_key_gen.rs:496) by Horner
// with the small x, one quad per (row, i); the result stays Jacobian (no inversion): the ack check
// adds it with the general addition, which costs the quad the same 5 rounds as a mixed one.
__global__ void __launch_bounds__(256) k_bivar_row_quad(int nrow, int t, const uint32_t* __restrict__ commits,
                                                        const uint32_t* __restrict__ part_idx,
                                                        const uint32_t* __restrict__ xs, int32_t* __restrict__ out) {
  const int g = (int)((blockIdx.x * 256u + threadIdx.x) >> 2);
  if (g >= nrow * (t + 1)) return;
  const int r = g / (t + 1), i = g % (t + 1);
  const int ncoef = (t + 1) * (t + 2) / 2;
  const uint32_t* C = commits + (size_t)part_idx[r] * ncoef * Q_G1_WORDS;
  const uint32_t x = xs[r];
  QJ acc = qj_inf();
#pragma unroll 1
  for (int j = t; j >= 0; j--) {
    acc = g1q_mul_small(acc, x);
    Fp cx, cy;
    if (!load_aff(C + (size_t)q_coeff_pos(i, j) * Q_G1_WORDS, cx, cy)) acc = g1q_add_affine(acc, cx, cy);
  }
  if (q_lane() == 0) qj_store(out + (size_t)g * Q_JROW_WORDS, acc);
}

// thread k of quad-group checks ack order[k] (order may be null); rows: Jacobian (k_bivar_row_quad)
__global__ void __launch_bounds__(256) k_bivar_check_quad(int nack, int t, const uint32_t* __restrict__ rows,
                                                          const uint32_t* __restrict__ row_idx,
                                                          const uint32_t* __restrict__ ys,
                                                          const uint32_t* __restrict__ vals,
                                                          const uint32_t* __restrict__ fbtab,
                                                          const uint32_t* __restrict__ order,
                                                          uint8_t* __restrict__ verdict) {
  const int k = (int)((blockIdx.x * 256u + threadIdx.x) >> 2);
  if (k >= nack) return;  // the four lanes of a quad leave together
  const int a = order ? (int)order[k] : k;
  const int32_t* R = (const int32_t*)rows + (size_t)row_idx[a] * (t + 1) * Q_JROW_WORDS;
  const uint32_t y = ys[a];
  // sum_j R_j y^j by Horner
  QJ acc = qj_inf();
#pragma unroll 1
  for (int j = t; j >= 0; j--) {
    acc = g1q_mul_small(acc, y);
    acc = g1q_add(acc, qj_load(R + (size_t)j * Q_JROW_WORDS));
  }
  // g1 * val: lane q adds comb windows q, q + 4, ..., then the quad joins the four partial sums
  const int q = q_lane();
  QJ part = qj_inf();
#pragma unroll 1
  for (int w = q; w < Q_FB_WINDOWS; w += 4) {
    const uint32_t d = (vals[(size_t)a * 8 + (w >> 2)] >> (8 * (w & 3))) & 0xffu;
    if (d == 0) continue;
    Fp x, yy;
    if (!load_aff(fbtab + ((size_t)w * Q_FB_ROW + d) * Q_G1_WORDS, x, yy)) part = g1_madd_lane(part, x, yy);
  }
  QJ p0{q_dpp<0x00>(part.x), q_dpp<0x00>(part.y), q_dpp<0x00>(part.z)};
  QJ p1{q_dpp<0x55>(part.x), q_dpp<0x55>(part.y), q_dpp<0x55>(part.z)};
  QJ p2{q_dpp<0xAA>(part.x), q_dpp<0xAA>(part.y), q_dpp<0xAA>(part.z)};
  QJ p3{q_dpp<0xFF>(part.x), q_dpp<0xFF>(part.y), q_dpp<0xFF>(part.z)};
  const QJ w = g1q_add(g1q_add(p0, p1), g1q_add(p2, p3));
  const bool ok = g1q_eq(acc, w);
  if (q == 0) verdict[a] = ok ? 1 : 0;
}

// ---------------------------------------------------------------- G1 Lagrange combine, latency form
// PublicKeySet::decrypt's interpolation (src/threshold_decrypt.rs:242-250) for a few ciphertexts: the
// GLV split lambda = d0 + d1 x^2 (phi(x, y) = (beta x, y) = [-x^2], so x^2 P = (beta x, -y)), each
// 128-bit digit in four 32-bit chunks; workgroup (c, s) sums chunk s of every term on 64 lane quads,
// an LDS tree joins them and quad 0 shifts the sum by 2^(32 s) (Horner); k_interp_g1_join adds the four
// partial sums and writes the affine point.  The group law of curve.hpp, so the affine bytes equal
// k_interp_endo<Fp>'s and the C oracle's.
constexpr int G1Q_NCHUNK = 4;
constexpr int G1Q_Q = 64;  // quads per workgroup

__device__ __forceinline__ QJ g1q_mul_affine(const Fp& x, const Fp& y, bool inf, uint32_t k) {
  if (inf || k == 0) return qj_inf();
  const int top = 31 - __builtin_clz(k);
  QJ acc{x, y, fp_one()};
#pragma unroll 1
  for (int i = top - 1; i >= 0; i--) {
    acc = g1q_dbl(acc);
    if ((k >> i) & 1) acc = g1q_add_affine(acc, x, y);
  }
  return acc;
}

__global__ void __launch_bounds__(256) k_interp_g1q(int ncomb, int m, const uint64_t* __restrict__ digits,
                                                    const uint32_t* __restrict__ pts, int32_t* __restrict__ part) {
  __shared__ int32_t sm[G1Q_Q * Q_JROW_WORDS];
  const int c = blockIdx.x / G1Q_NCHUNK, chunk = blockIdx.x % G1Q_NCHUNK;
  if (c >= ncomb) return;  // uniform per workgroup
  const int g = threadIdx.x >> 2;
  QJ acc = qj_inf();
  for (int t = g; t < m * 2; t += G1Q_Q) {
    const int k = t >> 1, j = t & 1;
    Fp x, y;
    const bool inf = load_aff(pts + ((size_t)c * m + k) * Q_G1_WORDS, x, y);
    if (j) {
      x = fp_reduce(fp_mul(x, fp_const(hb::BETA_M)));
      y = fp_neg(y);
    }
    const uint64_t d = digits[((size_t)c * m + k) * 4 + 2 * j + (chunk >> 1)];
    const uint32_t kc = (uint32_t)(d >> (32 * (chunk & 1)));
    acc = g1q_add(acc, g1q_mul_affine(x, y, inf, kc));
  }
  if (q_lane() == 0) qj_store(sm + g * Q_JROW_WORDS, acc);
  __syncthreads();
  for (int s = G1Q_Q / 2; s > 0; s >>= 1) {
    if (g < s) acc = g1q_add(qj_load(sm + g * Q_JROW_WORDS), qj_load(sm + (g + s) * Q_JROW_WORDS));
    __syncthreads();
    if (g < s && q_lane() == 0) qj_store(sm + g * Q_JROW_WORDS, acc);
    __syncthreads();
  }
  if (g != 0) return;
  QJ r = qj_load(sm);
#pragma unroll 1
  for (int b = 0; b < 32 * chunk; b++) r = g1q_dbl(r);
  if (q_lane() == 0) qj_store(part + (size_t)blockIdx.x * Q_JROW_WORDS, r);
}

__device__ __forceinline__ Fp fp_inv_vartime(const Fp& a) {
  uint32_t w[12], p[12], r[12];
  fp_to_words(a, w);
#pragma unroll
  for (int i = 0; i < 12; i++) p[i] = hb::PM2_W[i];
  p[0] += 2;  // p - 2 + 2
  hb::words_inv_vartime<12>(w, p, r);
  return fp_from_words(r);
}

// out[c] = affine(sum of the four chunk sums), one lane quad per combine
__global__ void __launch_bounds__(64) k_interp_g1_join(int ncomb, const int32_t* __restrict__ part,
                                                       uint32_t* __restrict__ out) {
  const int c = (int)((blockIdx.x * 64u + threadIdx.x) >> 2);
  if (c >= ncomb) return;
  const int32_t* p = part + (size_t)c * G1Q_NCHUNK * Q_JROW_WORDS;
  const QJ r = g1q_add(g1q_add(qj_load(p), qj_load(p + Q_JROW_WORDS)),
                       g1q_add(qj_load(p + 2 * Q_JROW_WORDS), qj_load(p + 3 * Q_JROW_WORDS)));
  uint32_t* o = out + (size_t)c * Q_G1_WORDS;
  if (qj_zero(r)) {
    if (q_lane() == 0)
      for (int i = 0; i < Q_G1_WORDS; i++) o[i] = 0u;
    return;
  }
  const Fp zi = fp_inv_vartime(fp_reduce(r.z));
  Fp zi2, u, xa, ya;
  zi2 = fp_sqr(zi);
  q2(r.x, zi2, zi2, zi, xa, u);
  ya = fp_mul(r.y, u);
  if (q_lane() == 0) {
    fp_to_words(xa, o);
    fp_to_words(ya, o + 12);
  }
}

// lambda_k g1 for the split master check of hbh_combine_verify_g2 (latency, not throughput): one
// 64-lane workgroup per scalar; quad g adds the comb-table points of scalar bytes 2g and 2g + 1 (a
// mixed addition), then four levels of general additions through LDS sum the 16 quads (depth 5 group
// operations of 5 product rounds each instead of 32 sequential additions); quad 0 writes the Jacobian
// sum (no inversion) as point p = (c, k) of combine c to side k & 1 of wave c * nw + k / 2 -- the P
// arrays the Miller-only k_wave launch reads (WAVE_JAC_P).
__global__ void __launch_bounds__(64) k_g1_gen_quad(int n, int m, int nw, int pairs, const uint32_t* __restrict__ tab,
                                                    const uint32_t* __restrict__ scalars, uint32_t* __restrict__ out0,
                                                    uint32_t* __restrict__ out1) {
  __shared__ int32_t sm[16 * Q_JROW_WORDS];
  const int p = blockIdx.x;
  if (p >= n) return;  // uniform per workgroup
  const int g = threadIdx.x >> 2;
  QJ acc = qj_inf();
#pragma unroll 1
  for (int h = 0; h < 2; h++) {
    const int w = 2 * g + h;
    const uint32_t d = (scalars[(size_t)p * 8 + (w >> 2)] >> (8 * (w & 3))) & 0xffu;
    if (d) {
      Fp x, y;
      load_aff(tab + ((size_t)w * Q_FB_ROW + d) * Q_G1_WORDS, x, y);
      acc = g1q_add_affine(acc, x, y);
    }
  }
  if (q_lane() == 0) qj_store(sm + g * Q_JROW_WORDS, acc);
  __syncthreads();
  for (int s = 8; s > 0; s >>= 1) {
    if (g < s) acc = g1q_add(qj_load(sm + g * Q_JROW_WORDS), qj_load(sm + (g + s) * Q_JROW_WORDS));
    __syncthreads();
    if (g < s && q_lane() == 0) qj_store(sm + g * Q_JROW_WORDS, acc);
    __syncthreads();
  }
  if (g != 0) return;
  const int c = p / m, k = p % m;
  uint32_t* o = pairs == 1 ? out0 + ((size_t)c * nw + k) * 36 : ((k & 1) ? out1 : out0) + ((size_t)c * nw + k / 2) * 36;
  if (qj_zero(acc)) {
    if (q_lane() == 0)
      for (int i = 0; i < 36; i++) o[i] = 0u;
    return;
  }
  // Jacobian out (the Miller kernel scales its lines by Z^3 instead of inverting Z); the quad's
  // lanes 0-2 convert one coordinate each
  const int q = q_lane();
  if (q < 3) fp_to_words(q == 0 ? acc.x : (q == 1 ? acc.y : acc.z), o + 12 * q);
}

}  // namespace hbs

namespace hbl {

hipError_t g1_gen_tree(hipStream_t s, int n, int m, int nw, int pairs, const void* tab, const uint32_t* scalars,
                       void* out0, void* out1) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hbs::k_g1_gen_quad, dim3((unsigned)n), dim3(64), 0, s, n, m, nw, pairs, (const uint32_t*)tab,
                     scalars, (uint32_t*)out0, (uint32_t*)out1);
  return hipGetLastError();
}

size_t interp_g1_quad_part_bytes(int ncomb) { return (size_t)ncomb * hbs::G1Q_NCHUNK * hbs::Q_JROW_WORDS * 4; }

hipError_t interp_g1_quad(hipStream_t s, int ncomb, int m, const uint64_t* digits, const void* pts, void* part,
                          void* out) {
  if (ncomb <= 0) return hipSuccess;
  hipLaunchKernelGGL(hbs::k_interp_g1q, dim3((unsigned)ncomb * hbs::G1Q_NCHUNK), dim3(256), 0, s, ncomb, m, digits,
                     (const uint32_t*)pts, (int32_t*)part);
  hipLaunchKernelGGL(hbs::k_interp_g1_join, dim3((unsigned)((4 * ncomb + 63) / 64)), dim3(64), 0, s, ncomb,
                     (const int32_t*)part, (uint32_t*)out);
  return hipGetLastError();
}


size_t bivar_rows_quad_bytes(int nrow, int t) { return (size_t)nrow * (t + 1) * hbs::Q_JROW_WORDS * 4; }

hipError_t bivar_row_quad(hipStream_t s, int nrow, int t, const void* commits, const uint32_t* part_idx,
                          const uint32_t* xs, void* rows) {
  if (nrow <= 0) return hipSuccess;
  const size_t lanes = 4 * (size_t)nrow * (t + 1);
  hipLaunchKernelGGL(hbs::k_bivar_row_quad, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, s, nrow, t,
                     (const uint32_t*)commits, part_idx, xs, (int32_t*)rows);
  return hipGetLastError();
}

hipError_t bivar_check_quad(hipStream_t s, int nack, int t, const void* rows, const uint32_t* row_idx,
                            const uint32_t* ys, const uint32_t* vals, const void* fbtab, uint8_t* verdict,
                            const uint32_t* order) {
  if (nack <= 0) return hipSuccess;
  hipLaunchKernelGGL(hbs::k_bivar_check_quad, dim3((unsigned)((4 * (size_t)nack + 255) / 256)), dim3(256), 0, s, nack, t,
                     (const uint32_t*)rows, row_idx, ys, vals, (const uint32_t*)fbtab, order, verdict);
  return hipGetLastError();
}

}  // namespace hbl
