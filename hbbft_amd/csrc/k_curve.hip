// Curve kernels (gfx950): batched scalar multiplication, threshold_crypto interpolate() (the
// Lagrange-at-0 MSMs behind combine_signatures and PublicKeySet::decrypt) and the SyncKeyGen
// bivariate-commitment checks.  Host launchers at the bottom (declared in launch.hpp).
// Variable-time Fp inverse (fp.hpp) for the single-thread affine outputs of this file's kernels.
#define HB_FP_LATENCY 1
#include <hip/hip_runtime.h>

#include "curve.hpp"
#include "fr.hpp"
#include "interp_pair.hpp"
#include "launch.hpp"

namespace hb {

HB_HD int coeff_pos(int i, int j) {  // threshold_crypto BivarPoly/BivarCommitment symmetric index
  return i <= j ? j * (j + 1) / 2 + i : i * (i + 1) / 2 + j;
}

__device__ __forceinline__ void load_g1(const uint32_t* w, Fp& x, Fp& y, bool& inf) {
  G1Aff a = g1_from_words(w);
  x = a.x;
  y = a.y;
  inf = a.inf;
}
__device__ __forceinline__ void load_g2(const uint32_t* w, Fp2& x, Fp2& y, bool& inf) {
  G2Aff a = g2_from_words(w);
  x = a.x;
  y = a.y;
  inf = a.inf;
}

// ------------------------------------------------------------------ batched k * P
__global__ void __launch_bounds__(256) k_g1_mul(int n, const uint32_t* __restrict__ pts,
                                                const uint32_t* __restrict__ scalars, uint32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fp x, y;
  bool inf;
  load_g1(pts + (size_t)i * G1_WORDS, x, y, inf);
  uint32_t k[8];
  for (int j = 0; j < 8; j++) k[j] = scalars[(size_t)i * 8 + j];
  g1_jac_to_words(jac_mul_affine(x, y, inf, k), out + (size_t)i * G1_WORDS);
}

__global__ void __launch_bounds__(256) k_g2_mul(int n, const uint32_t* __restrict__ pts,
                                                const uint32_t* __restrict__ scalars, uint32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fp2 x, y;
  bool inf;
  load_g2(pts + (size_t)i * G2_WORDS, x, y, inf);
  uint32_t k[8];
  for (int j = 0; j < 8; j++) k[j] = scalars[(size_t)i * 8 + j];
  g2_jac_to_words(jac_mul_affine(x, y, inf, k), out + (size_t)i * G2_WORDS);
}

// ------------------------------------------------------------------ fixed-base g1 * k
// Comb table of the G1 generator: FB_TAB[w][d] = d * 2^(8w) * g1 (affine words), w < 32, 1 <= d < 256
// (row d = 0 unused).  g1 * k is then 32 mixed additions of table points -- no doublings -- instead
// of ~255 doublings + ~128 additions: the public commitments of BivarPoly::commitment /
// Poly::commitment (src/sync_key_gen.rs:346-357, 508) and the g1 * val side of every Ack check
// (:542).  784 KiB per engine, built once on first use.
constexpr int FB_WINDOWS = 32;
constexpr int FB_ROW = 256;

__global__ void __launch_bounds__(256) k_fb_table(uint32_t* __restrict__ tab) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= FB_WINDOWS * FB_ROW) return;
  const int w = g / FB_ROW, d = g % FB_ROW;
  uint32_t k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int bit = 8 * w;
  k[bit >> 5] = (uint32_t)d << (bit & 31);
  g1_jac_to_words(jac_mul_affine(fp_const(G1X_M), fp_const(G1Y_M), false, k), tab + (size_t)g * G1_WORDS);
}

// acc + g1 * k from the comb table (k: 8 LE words)
__device__ __forceinline__ Jac<Fp> fb_mul(const uint32_t* __restrict__ tab, const uint32_t* k) {
  Jac<Fp> acc = jac_zero<Fp>();
#pragma unroll 1
  for (int w = 0; w < FB_WINDOWS; w++) {
    const uint32_t d = (k[w >> 2] >> (8 * (w & 3))) & 0xffu;
    if (d == 0) continue;
    Fp x, y;
    bool inf;
    load_g1(tab + ((size_t)w * FB_ROW + d) * G1_WORDS, x, y, inf);
    acc = jac_add_affine(acc, x, y);
  }
  return acc;
}

__global__ void __launch_bounds__(256) k_g1_mul_gen(int n, const uint32_t* __restrict__ tab,
                                                    const uint32_t* __restrict__ scalars, uint32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  for (int j = 0; j < 8; j++) k[j] = scalars[(size_t)i * 8 + j];
  g1_jac_to_words(fb_mul(tab, k), out + (size_t)i * G1_WORDS);
}

// ------------------------------------------------------------------ interpolate()
// lambda_k(0) = prod_{j != k} x_j / (x_j - x_k) over Fr (threshold_crypto interpolate, SURVEY
// Appendix B.6), then term_k = lambda_k * sample_k.  One thread per (combine, sample).
__device__ __forceinline__ bool lagrange(const uint32_t* __restrict__ xs, int m, int k, uint32_t* lam_canon) {
  Fr num = fr_raw(FR_ONE_M), den = fr_raw(FR_ONE_M);
  const Fr xk = fr_from_u32(xs[k]);
  for (int j = 0; j < m; j++) {
    if (j == k) continue;
    const Fr xj = fr_from_u32(xs[j]);
    num = fr_mul(num, xj);
    den = fr_mul(den, fr_sub(xj, xk));
  }
  if (fr_is_zero(den)) return false;  // duplicate x: threshold_crypto Error::DuplicateEntry
  const Fr lam = fr_to_canon(fr_mul(num, fr_inv(den)));
  for (int j = 0; j < FRL; j++) lam_canon[j] = lam.l[j];
  return true;
}

// Endomorphism split of a canonical scalar k < r (r < |x|^4, x the BLS parameter):
//   G2: k = d0 + d1|x| + d2|x|^2 + d3|x|^3 (digits < |x| < 2^64); psi = [x] on G2, so
//       |x|^j P = (-1)^j psi^j(P) and k P = sum_j d_j (-1)^j psi^j(P).
//   G1: k = d0 + d1 x^2 (digits < x^2 < 2^128); phi(x, y) = (beta x, y) = [-x^2] on G1, so
//       x^2 P = (beta x, -y) and k P = d0 P + d1 (beta x, -y).
// Digits by bit-serial long division (wave-uniform loops, no 128-bit types on the device).
// Valid for points of the prime-order subgroups, which the ABI requires of every sample.
HB_HD void k_to_u64(const uint32_t* k, uint64_t q[4]) {
  for (int w = 0; w < 4; w++) q[w] = (uint64_t)k[2 * w] | ((uint64_t)k[2 * w + 1] << 32);
}

// q <- q / D, returns q mod D; D = X_ABS (top bit set, so a shifted-out bit always means >= D)
HB_HD uint64_t div_x_abs(uint64_t q[4]) {
  uint64_t rem = 0;
  for (int w = 3; w >= 0; w--) {
    uint64_t qw = 0;
    for (int b = 63; b >= 0; b--) {
      const bool top = (rem >> 63) != 0;
      rem = (rem << 1) | ((q[w] >> b) & 1);
      const bool ge = top || rem >= X_ABS;
      if (ge) rem -= X_ABS;
      qw |= (uint64_t)ge << b;
    }
    q[w] = qw;
  }
  return rem;
}

// q <- q / x^2, rem <- q mod x^2 (128-bit divisor with its top bit set)
HB_HD void div_x2(uint64_t q[4], uint64_t rem[2]) {
  uint64_t r0 = 0, r1 = 0;
  for (int w = 3; w >= 0; w--) {
    uint64_t qw = 0;
    for (int b = 63; b >= 0; b--) {
      const bool top = (r1 >> 63) != 0;
      r1 = (r1 << 1) | (r0 >> 63);
      r0 = (r0 << 1) | ((q[w] >> b) & 1);
      const bool ge = top || r1 > X2_ABS[1] || (r1 == X2_ABS[1] && r0 >= X2_ABS[0]);
      if (ge) {
        const uint64_t nr0 = r0 - X2_ABS[0];
        r1 = r1 - X2_ABS[1] - (r0 < X2_ABS[0] ? 1 : 0);
        r0 = nr0;
      }
      qw |= (uint64_t)ge << b;
    }
    q[w] = qw;
  }
  rem[0] = r0;
  rem[1] = r1;
}

HB_HD Fp2 psi_x(const Fp2& x) {  // conj(x) * (0 + c u) = (x1 c) + (x0 c) u
  const Fp c = fp_const(PSI_C1_C1);
  return {fp_mul(x.c1, c), fp_mul(x.c0, c)};
}
HB_HD Fp2 psi_y(const Fp2& y) {
  const Fp2 c2 = {fp_const(PSI_C2_C0), fp_const(PSI_C2_C1)};
  return f2_mul(f2_conj(y), c2);
}

// term j of the split: digit_j * base_j(P) as a Jacobian point
// Keep 32-bit words [chunk * words / nchunk, (chunk + 1) * words / nchunk) of a digit of `words` words,
// shifted down to bit 0 (k_interp_endo's chunked chains: digit = sum_s chunk_s * 2^(s * bits)).
__device__ __forceinline__ void take_chunk(uint32_t kk[8], int words, int chunk, int nchunk) {
  const int wpc = words / nchunk, lo = chunk * wpc;
  const uint32_t t0 = kk[0], t1 = kk[1], t2 = kk[2], t3 = kk[3];
  for (int i = 0; i < 4; i++) {
    const int src = lo + i;
    const uint32_t v = src == 0 ? t0 : src == 1 ? t1 : src == 2 ? t2 : t3;
    kk[i] = (i < wpc && src < 4) ? v : 0u;
  }
}

__device__ __forceinline__ Jac<Fp2> endo_term(const uint32_t* w, const uint32_t* lam, int j, int chunk, int nchunk) {
  Fp2 x, y;
  bool inf;
  load_g2(w, x, y, inf);
  uint64_t q[4], dg[4];
  k_to_u64(lam, q);
  dg[0] = div_x_abs(q);
  dg[1] = div_x_abs(q);
  dg[2] = div_x_abs(q);
  dg[3] = q[0];  // the quotient after three divisions (< |x| since k < r < |x|^4)
  const uint64_t d = j == 0 ? dg[0] : j == 1 ? dg[1] : j == 2 ? dg[2] : dg[3];
  for (int s = 0; s < j; s++) {
    x = psi_x(x);
    y = psi_y(y);
  }
  if (j & 1) y = f2_neg(y);
  uint32_t kk[8] = {(uint32_t)d, (uint32_t)(d >> 32), 0, 0, 0, 0, 0, 0};
  take_chunk(kk, 2, chunk, nchunk);
  return jac_mul_affine(x, y, inf, kk);
}
__device__ __forceinline__ Jac<Fp> endo_term(const uint32_t* w, const uint32_t* lam, int j, int chunk, int nchunk,
                                             Fp /*tag*/) {
  Fp x, y;
  bool inf;
  load_g1(w, x, y, inf);
  uint64_t q[4], rem[2];
  k_to_u64(lam, q);
  div_x2(q, rem);
  uint64_t d0 = rem[0], d1 = rem[1];
  if (j == 1) {  // x^2 P = (beta x, -y); quotient < x^2 < 2^128
    d0 = q[0];
    d1 = q[1];
    x = fp_mul(x, fp_const(BETA_M));
    y = fp_neg(y);
  }
  uint32_t kk[8] = {(uint32_t)d0, (uint32_t)(d0 >> 32), (uint32_t)d1, (uint32_t)(d1 >> 32), 0, 0, 0, 0};
  take_chunk(kk, 4, chunk, nchunk);
  return jac_mul_affine(x, y, inf, kk);
}

template <class F>
struct EndoSplit;
template <>
struct EndoSplit<Fp2> {
  static constexpr int N = 4, WORDS = G2_WORDS, DIGIT_WORDS = 2;  // 64-bit digits
  __device__ static Jac<Fp2> term(const uint32_t* w, const uint32_t* lam, int j, int c, int nc) {
    return endo_term(w, lam, j, c, nc);
  }
  __device__ static void store(const Jac<Fp2>& p, uint32_t* out) { g2_jac_to_words(p, out); }
};
template <>
struct EndoSplit<Fp> {
  static constexpr int N = 2, WORDS = G1_WORDS, DIGIT_WORDS = 4;  // 128-bit digits
  __device__ static Jac<Fp> term(const uint32_t* w, const uint32_t* lam, int j, int c, int nc) {
    return endo_term(w, lam, j, c, nc, Fp{});
  }
  __device__ static void store(const Jac<Fp>& p, uint32_t* out) { g1_jac_to_words(p, out); }
};

// numerator / denominator of lambda_k(0) (Montgomery); false when some x_j == x_k (j != k)
__device__ __forceinline__ bool lagrange_parts(const uint32_t* __restrict__ xs, int m, int k, Fr& num, Fr& den) {
  num = fr_raw(FR_ONE_M);
  den = fr_raw(FR_ONE_M);
  const Fr xk = fr_from_u32(xs[k]);
  for (int j = 0; j < m; j++) {
    if (j == k) continue;
    const Fr xj = fr_from_u32(xs[j]);
    num = fr_mul(num, xj);
    den = fr_mul(den, fr_sub(xj, xk));
  }
  return !fr_is_zero(den);
}

// variable-time Fr inverse (one thread, public denominators)
__device__ __forceinline__ Fr fr_inv_vartime(const Fr& a) {
  const Fr c = fr_to_canon(a);
  uint32_t r[FRL];
  words_inv_vartime<FRL>(c.l, FR_W, r);
  Fr t;
  for (int j = 0; j < FRL; j++) t.l[j] = r[j];
  return fr_mul(t, fr_raw(FR_R2));  // canonical -> Montgomery
}

// One workgroup per combine.
//  Phase 1: thread k < m forms num_k and den_k of lambda_k(0) = prod x_j / prod (x_j - x_k); thread 0
//           inverts all den_k with one (variable-time) inversion (Montgomery's batch trick: 3m
//           products) and stages the canonical lambda_k in LDS.
//  Phase 2: each digit (64-bit on G2, 128-bit on G1) is cut into nchunk 32-bit-aligned chunks.
//           Thread (chunk s, slot t < m*N) computes term (k, j) = (t / N, t % N): chunk s of
//           endomorphism digit j of lambda_k(0), times base_j(P_k) -- a serial double-and-add chain of
//           64 / nchunk (G2) or 128 / nchunk (G1) steps instead of 255.
//  Phase 3: tree sum of each chunk's terms in LDS; thread 0 joins the chunk sums by Horner
//           (R = sum_s 2^(s*bits) S_s: the doublings run once, on the sum, without per-step adds)
//           and writes the affine result.  For m = 22: G2 chain 32 (dbl+add) + 32 dbl instead of
//           64 (dbl+add); G1 32 (dbl+add) + 96 dbl instead of 128 (dbl+add).
// Combines with m > LAM_LDS_MAX samples compute lambda per term instead (uniform Fermat inverse).
constexpr int LAM_LDS_MAX = 256;

template <class F>
__global__ void __launch_bounds__(256) k_interp_endo(int ncomb, int m, const uint32_t* __restrict__ xs,
                                                     const uint32_t* __restrict__ pts, uint32_t* __restrict__ out,
                                                     int* __restrict__ status, int nchunk) {
  extern __shared__ unsigned char smem_raw[];
  __shared__ int s_dup;
  Jac<F>* sm = reinterpret_cast<Jac<F>*>(smem_raw);
  Fr* snum = reinterpret_cast<Fr*>(smem_raw + blockDim.x * sizeof(Jac<F>));
  Fr* sden = snum + m;
  Fr* slam = sden + m;  // prefix products, then the canonical lambda_k
  using S = EndoSplit<F>;
  const int c = blockIdx.x;
  if (c >= ncomb) return;  // uniform per workgroup
  const uint32_t* cx = xs + (size_t)c * m;
  const bool staged = m <= LAM_LDS_MAX;
  if (staged) {
    if (threadIdx.x == 0) s_dup = 0;
    __syncthreads();
    for (int k = threadIdx.x; k < m; k += blockDim.x) {
      Fr num, den;
      if (!lagrange_parts(cx, m, k, num, den)) s_dup = 1;
      snum[k] = num;
      sden[k] = den;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      if (s_dup) {
        status[c] = hbl::HBL_DUPLICATE;  // the combine's output is void; its terms are O
        for (int k = 0; k < m; k++)
          for (int w = 0; w < FRL; w++) slam[k].l[w] = 0;
      } else {
        slam[0] = sden[0];
        for (int k = 1; k < m; k++) slam[k] = fr_mul(slam[k - 1], sden[k]);
        Fr inv = fr_inv_vartime(slam[m - 1]);
        for (int k = m - 1; k > 0; k--) {
          const Fr ik = fr_mul(inv, slam[k - 1]);
          inv = fr_mul(inv, sden[k]);
          slam[k] = fr_to_canon(fr_mul(snum[k], ik));
        }
        slam[0] = fr_to_canon(fr_mul(snum[0], inv));
      }
    }
    __syncthreads();
  }
  // thread -> (chunk, slot): group `chunk` of G = blockDim / nchunk threads sums chunk `chunk` of
  // every term's digit, so each chain is (digit bits / nchunk) steps instead of digit bits.
  const int G = blockDim.x / nchunk, chunk = threadIdx.x / G, g = threadIdx.x % G;
  Jac<F> acc = jac_zero<F>();
  for (int t = g; t < m * S::N; t += G) {
    const int k = t / S::N, j = t % S::N;
    uint32_t lam[8];
    if (staged) {
      for (int w = 0; w < 8; w++) lam[w] = slam[k].l[w];
    } else if (!lagrange(cx, m, k, lam)) {
      status[c] = hbl::HBL_DUPLICATE;
      continue;
    }
    acc = jac_add(acc, S::term(pts + ((size_t)c * m + k) * S::WORDS, lam, j, chunk, nchunk));
  }
  sm[threadIdx.x] = acc;
  __syncthreads();
  for (int s = G / 2; s > 0; s >>= 1) {
    if (g < s) sm[threadIdx.x] = jac_add(sm[threadIdx.x], sm[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    // Horner over the chunk sums: R = sum_s 2^(s * bits) * S_s, one shared doubling tail
    const int bits = 32 * S::DIGIT_WORDS / nchunk;
    Jac<F> r = sm[(nchunk - 1) * G];
    for (int s = nchunk - 2; s >= 0; s--) {
      for (int b = 0; b < bits; b++) r = jac_dbl(r);
      r = jac_add(r, sm[s * G]);
    }
    S::store(r, out + (size_t)c * S::WORDS);
  }
}

// ------------------------------------------------------------------ interpolate(), lane-pair form
// Stage 1 of the latency form of the G2 combine (k_interp_pair.hip does the curve work): the four
// 64-bit GLS digits of every lambda_k(0) (the endo_term split), digits[(c*m + k)*4 + j].  One
// workgroup per combine; a duplicate x sets status[c] = HBL_DUPLICATE and zero digits (terms = O).
// g1: the two 128-bit GLV digits instead (d[0..1] = lambda mod x^2, d[2..3] = lambda div x^2, low word first).
__global__ void __launch_bounds__(64) k_interp_digits(int ncomb, int m, const uint32_t* __restrict__ xs,
                                                      uint64_t* __restrict__ digits, int* __restrict__ status, int g1) {
  extern __shared__ unsigned char smem_raw[];
  __shared__ int s_dup;
  Fr* snum = reinterpret_cast<Fr*>(smem_raw);
  Fr* sden = snum + m;
  Fr* slam = sden + m;
  const int c = blockIdx.x;
  if (c >= ncomb) return;
  const uint32_t* cx = xs + (size_t)c * m;
  if (threadIdx.x == 0) s_dup = 0;
  __syncthreads();
  for (int k = threadIdx.x; k < m; k += blockDim.x) {
    Fr num, den;
    if (!lagrange_parts(cx, m, k, num, den)) s_dup = 1;
    snum[k] = num;
    sden[k] = den;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_dup) {
      status[c] = hbl::HBL_DUPLICATE;
      for (int k = 0; k < m; k++)
        for (int w = 0; w < FRL; w++) slam[k].l[w] = 0;
    } else {
      slam[0] = sden[0];
      for (int k = 1; k < m; k++) slam[k] = fr_mul(slam[k - 1], sden[k]);
      Fr inv = fr_inv_vartime(slam[m - 1]);
      for (int k = m - 1; k > 0; k--) {
        const Fr ik = fr_mul(inv, slam[k - 1]);
        inv = fr_mul(inv, sden[k]);
        slam[k] = fr_to_canon(fr_mul(snum[k], ik));
      }
      slam[0] = fr_to_canon(fr_mul(snum[0], inv));
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < m; k += blockDim.x) {
    uint64_t q[4];
    k_to_u64(slam[k].l, q);
    uint64_t* d = digits + ((size_t)c * m + k) * 4;
    if (g1) {
      uint64_t rem[2];
      div_x2(q, rem);
      d[0] = rem[0];
      d[1] = rem[1];
      d[2] = q[0];
      d[3] = q[1];
    } else {
      d[0] = div_x_abs(q);
      d[1] = div_x_abs(q);
      d[2] = div_x_abs(q);
      d[3] = q[0];
    }
  }
}

// ------------------------------------------------------------------ SyncKeyGen
// BivarCommitment::row(x)[i] = sum_j C[coeff_pos(i,j)] x^j, by Horner in G1 with the small
// integer x (src/sync_key_gen.rs:496): t steps of (x * acc + C) instead of (t+1) full scalar
// multiplications.  One thread per (row request, i).
__global__ void __launch_bounds__(256) k_bivar_row(int nrow, int t, const uint32_t* __restrict__ commits,
                                                   const uint32_t* __restrict__ part_idx, const uint32_t* __restrict__ xs,
                                                   uint32_t* __restrict__ out) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nrow * (t + 1)) return;
  const int r = g / (t + 1), i = g % (t + 1);
  const int ncoef = (t + 1) * (t + 2) / 2;
  const uint32_t* C = commits + (size_t)part_idx[r] * ncoef * G1_WORDS;
  const uint32_t x = xs[r];
  Jac<Fp> acc = jac_zero<Fp>();
  for (int j = t; j >= 0; j--) {
    acc = jac_mul_small(acc, x);
    Fp cx, cy;
    bool inf;
    load_g1(C + (size_t)coeff_pos(i, j) * G1_WORDS, cx, cy, inf);
    if (!inf) acc = jac_add_affine(acc, cx, cy);
  }
  g1_jac_to_words(acc, out + (size_t)g * G1_WORDS);
}

// x_k = idx_k + 1 (threshold_crypto into_fr_plus_1) for device-resident index arrays; an index of
// 0xffffffff (x would wrap to 0) sets the combine's status to HBL_BAD_INDEX (== HBH_ERR_ARG).
__global__ void __launch_bounds__(256) k_index_plus_one(int n, int m, const uint32_t* __restrict__ idx,
                                                        uint32_t* __restrict__ xs, int* __restrict__ status) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t v = idx[k];
  xs[k] = v + 1u;
  if (v == 0xffffffffu) status[k / m] = hbl::HBL_BAD_INDEX;
}

// BivarCommitment::evaluate(x, y) == G1::one() * val  (src/sync_key_gen.rs:542), from the rows
// R = row(x): evaluate(x, y) = sum_j R_j y^j (Horner with the small y).  One thread per ack.
// order (optional): thread k checks ack order[k] -- the host sorts acks by y so that the lanes of a
// wave share y and the small-scalar double-and-add of the Horner steps does not diverge.
__global__ void __launch_bounds__(256) k_bivar_check(int nack, int t, const uint32_t* __restrict__ rows,
                                                     const uint32_t* __restrict__ row_idx,
                                                     const uint32_t* __restrict__ ys, const uint32_t* __restrict__ vals,
                                                     const uint32_t* __restrict__ fbtab, const uint32_t* __restrict__ order,
                                                     uint8_t* __restrict__ verdict) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nack) return;
  const int a = order ? (int)order[k] : k;
  const uint32_t* R = rows + (size_t)row_idx[a] * (t + 1) * G1_WORDS;
  const uint32_t y = ys[a];
  Jac<Fp> acc = jac_zero<Fp>();
  for (int j = t; j >= 0; j--) {
    acc = jac_mul_small(acc, y);
    Fp rx, ry;
    bool inf;
    load_g1(R + (size_t)j * G1_WORDS, rx, ry, inf);
    if (!inf) acc = jac_add_affine(acc, rx, ry);
  }
  uint32_t ks[8];
  for (int j = 0; j < 8; j++) ks[j] = vals[(size_t)a * 8 + j];
  const Jac<Fp> w = fb_mul(fbtab, ks);
  verdict[a] = jac_eq(acc, w) ? 1 : 0;
}

// ------------------------------------------------------------------ Ack checks by finite differences
// The acks of one row R = row(x) (one Part, one checking node x) evaluate the same degree-t polynomial
// E(y) = sum_j R_j y^j at the senders' y = 1..N.  For a dense run of y (a row with many acks, as every
// node's Ack drain has: one Ack per sender per Part) E is evaluated at y0 .. y0 + L - 1 as
//   1. the forward-difference table D_k = Delta^k E(y0), k <= t, straight from the row: with the
//      Horner tails F_m(y) = R_m + y F_{m+1}(y) (F_t = R_t, F_0 = E) the product rule of differences
//      gives  Delta^k F_m(y0) = [k = 0] R_m + (y0 + k) Delta^k F_{m+1}(y0) + k Delta^{k-1} F_{m+1}(y0),
//      one level per m (k_bivar_fd_seed, one launch per level, lane (k, row) k-major so a wave's lanes
//      share the small multipliers); for y0 = 0 a level entry is one product k (D_k + D_{k-1}), so the
//      table costs (t+1)(t+2)/2 small products per row where Horner at t+1 points cost (t+1) t,
//   2. D_k += D_{k+1} (k < t) per step of y: every further E(y) costs t independent G1 additions
//      (k_bivar_fd_run: one lane per (row, k)),
// and each ack compares its E(y) with g1 * val (k_bivar_fd_check).  Exact group arithmetic throughout:
// the verdicts are the Horner kernel's bit for bit (tests/test_gpu_commit_set.py compares them).
// E values are stored as Jacobian points (FD_WORDS words each); a row's region of L >= 2 (t + 1) points
// holds the seed levels' two tables (level m in slots (m & 1) (t + 1) + k) before the run fills it.
constexpr int FD_WORDS = 3 * NL;

__device__ __forceinline__ void jac_store(uint32_t* __restrict__ w, const Jac<Fp>& p) {
#pragma unroll
  for (int i = 0; i < NL; i++) {
    w[i] = p.x.l[i];
    w[NL + i] = p.y.l[i];
    w[2 * NL + i] = p.z.l[i];
  }
}
__device__ __forceinline__ Jac<Fp> jac_load(const uint32_t* __restrict__ w) {
  Jac<Fp> p;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    p.x.l[i] = w[i];
    p.y.l[i] = w[NL + i];
    p.z.l[i] = w[2 * NL + i];
  }
  return p;
}

// step 1, level m: lane g = k * nfd + f (k <= t - m) writes Delta^k F_m(y0[f]) of FD row f; level t
// is F_t = R_t itself.
__global__ void __launch_bounds__(256) k_bivar_fd_seed(int nfd, int t, int m, const uint32_t* __restrict__ rows,
                                                       const uint32_t* __restrict__ fd_slot,
                                                       const uint32_t* __restrict__ fd_y0,
                                                       const uint32_t* __restrict__ fd_off, uint32_t* __restrict__ ebuf) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  const int deg = t - m;  // degree of F_m
  if (g >= nfd * (deg + 1)) return;
  const int k = g / nfd, f = g % nfd;
  const size_t T1 = (size_t)t + 1;
  uint32_t* E = ebuf + (size_t)fd_off[f] * FD_WORDS;
  const uint32_t* in = E + ((m + 1) & 1) * T1 * FD_WORDS;
  Jac<Fp> d = jac_zero<Fp>();
  if (m < t) {
    const Jac<Fp> a = k < deg ? jac_load(in + (size_t)k * FD_WORDS) : jac_zero<Fp>();
    const Jac<Fp> b = k > 0 ? jac_load(in + (size_t)(k - 1) * FD_WORDS) : jac_zero<Fp>();
    const uint32_t y0 = fd_y0[f];
    if (y0 == 0)
      d = jac_mul_small(jac_add(a, b), (uint32_t)k);
    else
      d = jac_add(jac_mul_small(a, y0 + (uint32_t)k), jac_mul_small(b, (uint32_t)k));
  }
  if (k == 0) {
    Fp rx, ry;
    bool inf;
    load_g1(rows + ((size_t)fd_slot[f] * T1 + m) * G1_WORDS, rx, ry, inf);
    if (!inf) d = jac_add_affine(d, rx, ry);
  }
  jac_store(E + ((m & 1) * T1 + k) * FD_WORDS, d);
}

// step 2: one workgroup per G = blockDim / (t + 1) FD rows, lane (r, k) holds D_k of row r; the
// neighbour's D crosses lanes through LDS (blockDim x FD_WORDS words).  Rows are sorted by length, so
// a workgroup's rows step together; a row stops at its own length.
__global__ void __launch_bounds__(256) k_bivar_fd_run(int nfd, int t, const uint32_t* __restrict__ fd_off,
                                                      const uint32_t* __restrict__ fd_len, uint32_t* __restrict__ ebuf) {
  extern __shared__ uint32_t fd_lds[];
  __shared__ int lmax;
  const int T1 = t + 1;
  const int G = blockDim.x / T1;
  const int r = threadIdx.x / T1, k = threadIdx.x % T1;
  const int f = blockIdx.x * G + r;
  const bool active = r < G && f < nfd;
  if (threadIdx.x == 0) lmax = 0;
  __syncthreads();
  int L = 0;
  size_t off = 0;
  Jac<Fp> D = jac_zero<Fp>();
  if (active) {
    L = (int)fd_len[f];
    off = fd_off[f];
    D = jac_load(ebuf + (off + k) * FD_WORDS);
    atomicMax(&lmax, L);
  }
  __syncthreads();
  uint32_t* mine = fd_lds + (size_t)threadIdx.x * FD_WORDS;
  // step s moves the table from y0 + s - 1 to y0 + s; D_0 = E(y0 + s) (E(y0) = D_0 is in slot 0)
  const int steps = lmax;
  for (int s = 1; s < steps; s++) {
    if (active) jac_store(mine, D);
    __syncthreads();
    if (active && k < t && s < L) D = jac_add(D, jac_load(mine + FD_WORDS));
    __syncthreads();
    if (active && k == 0 && s < L) jac_store(ebuf + (off + s) * FD_WORDS, D);
  }
}

// ------------------------------------------------------------------ 16-bit fixed-base comb of g1
// FB16[w][d] = d * 2^(16 w) * g1 (affine words), w < 16, 1 <= d < 65536 (d = 0 unused): g1 * k in 16
// mixed additions instead of the 8-bit comb's 32 -- the g1 * val side of the finite-difference Ack
// check, where it is a fifth of the work.  96 MiB per engine, built once on first use:
// k_fb16_base computes the 16 window bases, k_fb16_chunk one chunk of 256 consecutive d per thread
// (one multiplication by a 16-bit scalar, 255 mixed additions, then a batch normalisation with one
// inversion through the caller's scratch: FD_WORDS + NL words per entry).
constexpr int FB16_WINDOWS = 16;
constexpr int FB16_ROW = 65536;
constexpr int FB16_CHUNK = 256;

__global__ void __launch_bounds__(64) k_fb16_base(uint32_t* __restrict__ base) {
  const int w = threadIdx.x;
  if (w >= FB16_WINDOWS) return;
  uint32_t k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  k[w >> 1] = 1u << (16 * (w & 1));
  g1_jac_to_words(jac_mul_affine(fp_const(G1X_M), fp_const(G1Y_M), false, k), base + (size_t)w * G1_WORDS);
}

__global__ void __launch_bounds__(256) k_fb16_chunk(const uint32_t* __restrict__ base, uint32_t* __restrict__ scratch,
                                                    uint32_t* __restrict__ tab) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int NCH = FB16_ROW / FB16_CHUNK;
  if (g >= FB16_WINDOWS * NCH) return;
  const int w = g / NCH, c = g % NCH;
  Fp bx, by;
  bool binf;
  load_g1(base + (size_t)w * G1_WORDS, bx, by, binf);
  const int n = (c == NCH - 1) ? FB16_CHUNK - 1 : FB16_CHUNK;  // d = 65536 is not an entry
  uint32_t* J = scratch + (size_t)g * FB16_CHUNK * (FD_WORDS + NL);  // Jacobian entries
  uint32_t* Z = J + (size_t)FB16_CHUNK * FD_WORDS;                   // prefix products of Z
  Jac<Fp> p = jac_mul_small(jac_from_affine(bx, by, false), (uint32_t)(c * FB16_CHUNK + 1));
  Fp acc = fp_one();
  for (int j = 0; j < n; j++) {
    jac_store(J + (size_t)j * FD_WORDS, p);
    acc = fp_mul(acc, p.z);
    for (int i = 0; i < NL; i++) Z[(size_t)j * NL + i] = acc.l[i];
    p = jac_add_affine(p, bx, by);
  }
  Fp inv = fp_inv(acc);  // 1 / (z_0 ... z_{n-1})
  for (int j = n - 1; j >= 0; j--) {
    const Jac<Fp> q = jac_load(J + (size_t)j * FD_WORDS);
    Fp zi = inv;
    if (j > 0) {
      Fp prev;
      for (int i = 0; i < NL; i++) prev.l[i] = Z[(size_t)(j - 1) * NL + i];
      zi = fp_mul(inv, prev);  // 1 / z_j
    }
    inv = fp_mul(inv, q.z);    // 1 / (z_0 ... z_{j-1})
    const Fp zi2 = fp_sqr(zi);
    uint32_t* out = tab + ((size_t)w * FB16_ROW + (size_t)(c * FB16_CHUNK + 1 + j)) * G1_WORDS;
    fp_to_words(fp_mul(q.x, zi2), out);
    fp_to_words(fp_mul(q.y, fp_mul(zi2, zi)), out + 12);
  }
}

// g1 * k from the 16-bit comb (k: 8 LE words)
__device__ __forceinline__ Jac<Fp> fb16_mul(const uint32_t* __restrict__ tab, const uint32_t* k) {
  Jac<Fp> acc = jac_zero<Fp>();
#pragma unroll 1
  for (int w = 0; w < FB16_WINDOWS; w++) {
    const uint32_t d = (k[w >> 1] >> (16 * (w & 1))) & 0xffffu;
    if (d == 0) continue;
    Fp x, y;
    bool inf;
    load_g1(tab + ((size_t)w * FB16_ROW + d) * G1_WORDS, x, y, inf);
    acc = jac_add_affine(acc, x, y);
  }
  return acc;
}

// step 4: ack a = list[k] compares E at epos[a] with g1 * val (16-bit comb table)
__global__ void __launch_bounds__(256) k_bivar_fd_check(int n, const uint32_t* __restrict__ ebuf,
                                                        const uint32_t* __restrict__ epos,
                                                        const uint32_t* __restrict__ vals,
                                                        const uint32_t* __restrict__ fbtab,
                                                        const uint32_t* __restrict__ list, uint8_t* __restrict__ verdict) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int a = (int)list[k];
  const Jac<Fp> e = jac_load(ebuf + (size_t)epos[a] * FD_WORDS);
  uint32_t ks[8];
  for (int j = 0; j < 8; j++) ks[j] = vals[(size_t)a * 8 + j];
  verdict[a] = jac_eq(e, fb16_mul(fbtab, ks)) ? 1 : 0;
}

// Commitment::evaluate(x) = sum_j C_j x^j (threshold_crypto poly.rs) by Horner in G1 with the small
// integer x -- PublicKeySet::public_key_share(i) = evaluate(i + 1), precomputed for every node by
// NetworkInfo::new (src/network_info.rs:59-62).  commits holds ncommit commitments of t+1 points;
// request r evaluates commitment commit_idx[r] at xs[r].  One thread per request.
__global__ void __launch_bounds__(256) k_commit_eval(int n, int t, const uint32_t* __restrict__ commits,
                                                     const uint32_t* __restrict__ commit_idx,
                                                     const uint32_t* __restrict__ xs, uint32_t* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint32_t* C = commits + (size_t)commit_idx[r] * (t + 1) * G1_WORDS;
  const uint32_t x = xs[r];
  Jac<Fp> acc = jac_zero<Fp>();
  for (int j = t; j >= 0; j--) {
    acc = jac_mul_small(acc, x);
    Fp cx, cy;
    bool inf;
    load_g1(C + (size_t)j * G1_WORDS, cx, cy, inf);
    if (!inf) acc = jac_add_affine(acc, cx, cy);
  }
  g1_jac_to_words(acc, out + (size_t)r * G1_WORDS);
}

}  // namespace hb

// ------------------------------------------------------------------ host launchers
namespace hbl {

static inline dim3 grid_for(int n, int b = 256) { return dim3((unsigned)((n + b - 1) / b)); }

hipError_t g1_mul(hipStream_t s, int n, const void* pts, const uint32_t* scalars, void* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_g1_mul, grid_for(n), dim3(256), 0, s, n, (const uint32_t*)pts, scalars, (uint32_t*)out);
  return hipGetLastError();
}
hipError_t g2_mul(hipStream_t s, int n, const void* pts, const uint32_t* scalars, void* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_g2_mul, grid_for(n), dim3(256), 0, s, n, (const uint32_t*)pts, scalars, (uint32_t*)out);
  return hipGetLastError();
}

template <class F>
static hipError_t combine(hipStream_t s, int ncomb, int m, const uint32_t* xs, const void* pts, void* out,
                          int* status) {
  if (ncomb <= 0) return hipSuccess;
  using S = hb::EndoSplit<F>;
  int g = 64;  // group: power of two >= m * N (tree reduction), 64..256
  while (g < 256 && g < m * S::N) g *= 2;
  // Latency mode (few combines: the chip is mostly idle, the serial chain is the time): split each
  // digit into nchunk word-aligned chunks while the workgroup stays <= 256 threads.  Throughput
  // mode (>= COMBINE_CHUNK_MAX combines fill the CUs): unsplit chains do the least total work
  // (MI355X, 22 G2 shares: one combine 6.36 -> 5.37 ms chunked; 1,024 combines 83 k/s unsplit vs
  // 49 k/s chunked).
  constexpr int COMBINE_CHUNK_MAX = 128;
  int nchunk = 1;
  while (ncomb < COMBINE_CHUNK_MAX && nchunk < S::DIGIT_WORDS && g * nchunk * 2 <= 256) nchunk *= 2;
  const int b = g * nchunk;
  const size_t lds = b * sizeof(hb::Jac<F>) + (m <= hb::LAM_LDS_MAX ? (size_t)m * 3 * sizeof(hb::Fr) : 0);
  hipLaunchKernelGGL(hb::k_interp_endo<F>, dim3((unsigned)ncomb), dim3(b), lds, s, ncomb, m, xs,
                     (const uint32_t*)pts, (uint32_t*)out, status, nchunk);
  return hipGetLastError();
}
hipError_t combine_g1(hipStream_t s, int ncomb, int m, const uint32_t* xs, const void* pts, void* out, int* status) {
  return combine<hb::Fp>(s, ncomb, m, xs, pts, out, status);
}
hipError_t combine_g2(hipStream_t s, int ncomb, int m, const uint32_t* xs, const void* pts, void* out, int* status) {
  return combine<hb::Fp2>(s, ncomb, m, xs, pts, out, status);
}

hipError_t bivar_row(hipStream_t s, int nrow, int t, const void* commits, const uint32_t* part_idx, const uint32_t* xs,
                     void* out) {
  if (nrow <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_bivar_row, grid_for(nrow * (t + 1)), dim3(256), 0, s, nrow, t, (const uint32_t*)commits,
                     part_idx, xs, (uint32_t*)out);
  return hipGetLastError();
}
hipError_t bivar_check(hipStream_t s, int nack, int t, const void* rows, const uint32_t* row_idx, const uint32_t* ys,
                       const uint32_t* vals, const void* fbtab, uint8_t* verdict, const uint32_t* order) {
  if (nack <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_bivar_check, grid_for(nack), dim3(256), 0, s, nack, t, (const uint32_t*)rows, row_idx, ys,
                     vals, (const uint32_t*)fbtab, order, verdict);
  return hipGetLastError();
}

size_t fd_point_bytes() { return (size_t)hb::FD_WORDS * 4; }
hipError_t bivar_fd(hipStream_t s, int nfd, int t, const void* rows, const uint32_t* fd_slot, const uint32_t* fd_y0,
                    const uint32_t* fd_off, const uint32_t* fd_len, void* ebuf) {
  if (nfd <= 0) return hipSuccess;
  for (int m = t; m >= 0; m--)
    hipLaunchKernelGGL(hb::k_bivar_fd_seed, grid_for(nfd * (t - m + 1)), dim3(256), 0, s, nfd, t, m,
                       (const uint32_t*)rows, fd_slot, fd_y0, fd_off, (uint32_t*)ebuf);
  const int G = 256 / (t + 1);
  const size_t lds = (size_t)256 * hb::FD_WORDS * 4;
  hipLaunchKernelGGL(hb::k_bivar_fd_run, dim3((unsigned)((nfd + G - 1) / G)), dim3(256), lds, s, nfd, t, fd_off, fd_len,
                     (uint32_t*)ebuf);
  return hipGetLastError();
}
hipError_t bivar_fd_check(hipStream_t s, int n, const void* ebuf, const uint32_t* epos, const uint32_t* vals,
                          const void* fbtab, const uint32_t* list, uint8_t* verdict) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_bivar_fd_check, grid_for(n), dim3(256), 0, s, n, (const uint32_t*)ebuf, epos, vals,
                     (const uint32_t*)fbtab, list, verdict);
  return hipGetLastError();
}

size_t fb16_table_bytes() { return (size_t)hb::FB16_WINDOWS * hb::FB16_ROW * hb::G1_WORDS * 4; }
size_t fb16_scratch_bytes() {
  return (size_t)hb::FB16_WINDOWS * hb::FB16_ROW * (hb::FD_WORDS + hb::NL) * 4 + (size_t)hb::FB16_WINDOWS * hb::G1_WORDS * 4;
}
hipError_t fb16_table(hipStream_t s, void* tab, void* scratch) {
  uint32_t* base = (uint32_t*)scratch;
  uint32_t* rest = base + (size_t)hb::FB16_WINDOWS * hb::G1_WORDS;
  hipLaunchKernelGGL(hb::k_fb16_base, dim3(1), dim3(64), 0, s, base);
  const int n = hb::FB16_WINDOWS * (hb::FB16_ROW / hb::FB16_CHUNK);
  hipLaunchKernelGGL(hb::k_fb16_chunk, grid_for(n), dim3(256), 0, s, (const uint32_t*)base, rest, (uint32_t*)tab);
  return hipGetLastError();
}

size_t fb_table_bytes() { return (size_t)hb::FB_WINDOWS * hb::FB_ROW * hb::G1_WORDS * 4; }
hipError_t fb_table(hipStream_t s, void* tab) {
  hipLaunchKernelGGL(hb::k_fb_table, grid_for(hb::FB_WINDOWS * hb::FB_ROW), dim3(256), 0, s, (uint32_t*)tab);
  return hipGetLastError();
}
hipError_t g1_mul_gen(hipStream_t s, int n, const void* tab, const uint32_t* scalars, void* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_g1_mul_gen, grid_for(n), dim3(256), 0, s, n, (const uint32_t*)tab, scalars, (uint32_t*)out);
  return hipGetLastError();
}

hipError_t index_plus_one(hipStream_t s, int n, int m, const uint32_t* idx, uint32_t* xs, int* status) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_index_plus_one, grid_for(n), dim3(256), 0, s, n, m, idx, xs, status);
  return hipGetLastError();
}

hipError_t interp_digits(hipStream_t s, int ncomb, int m, const uint32_t* xs, uint64_t* digits, int* status, bool g1) {
  if (ncomb <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_interp_digits, dim3((unsigned)ncomb), dim3(64), (size_t)3 * m * sizeof(hb::Fr), s, ncomb, m,
                     xs, digits, status, g1 ? 1 : 0);
  return hipGetLastError();
}

hipError_t commit_eval(hipStream_t s, int n, int t, const void* commits, const uint32_t* commit_idx, const uint32_t* xs,
                       void* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_commit_eval, grid_for(n), dim3(256), 0, s, n, t, (const uint32_t*)commits, commit_idx, xs,
                     (uint32_t*)out);
  return hipGetLastError();
}

}  // namespace hbl
