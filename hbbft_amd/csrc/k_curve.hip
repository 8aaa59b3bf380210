// Curve kernels (gfx950): batched scalar multiplication, threshold_crypto interpolate() (the
// Lagrange-at-0 MSMs behind combine_signatures and PublicKeySet::decrypt) and the SyncKeyGen
// bivariate-commitment checks.  Host launchers at the bottom (declared in launch.hpp).
#include <hip/hip_runtime.h>

#include "curve.hpp"
#include "fr.hpp"
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

template <class F>
__device__ __forceinline__ void store_jac(void* work, size_t idx, const Jac<F>& p) {
  reinterpret_cast<Jac<F>*>(work)[idx] = p;
}
template <class F>
__device__ __forceinline__ Jac<F> load_jac(const void* work, size_t idx) {
  return reinterpret_cast<const Jac<F>*>(work)[idx];
}

__global__ void __launch_bounds__(256) k_g1_interp_terms(int ncomb, int m, const uint32_t* __restrict__ xs,
                                                         const uint32_t* __restrict__ pts, void* __restrict__ work,
                                                         int* __restrict__ status) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ncomb * m) return;
  const int c = t / m, k = t % m;
  uint32_t lam[8];
  if (!lagrange(xs + (size_t)c * m, m, k, lam)) {
    status[c] = hbl::HBL_DUPLICATE;
    store_jac(work, t, jac_zero<Fp>());
    return;
  }
  Fp x, y;
  bool inf;
  load_g1(pts + (size_t)t * G1_WORDS, x, y, inf);
  store_jac(work, t, jac_mul_affine(x, y, inf, lam));
}

__global__ void __launch_bounds__(256) k_g2_interp_terms(int ncomb, int m, const uint32_t* __restrict__ xs,
                                                         const uint32_t* __restrict__ pts, void* __restrict__ work,
                                                         int* __restrict__ status) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ncomb * m) return;
  const int c = t / m, k = t % m;
  uint32_t lam[8];
  if (!lagrange(xs + (size_t)c * m, m, k, lam)) {
    status[c] = hbl::HBL_DUPLICATE;
    store_jac(work, t, jac_zero<Fp2>());
    return;
  }
  Fp2 x, y;
  bool inf;
  load_g2(pts + (size_t)t * G2_WORDS, x, y, inf);
  store_jac(work, t, jac_mul_affine(x, y, inf, lam));
}

__global__ void __launch_bounds__(64) k_g1_interp_sum(int ncomb, int m, const void* __restrict__ work,
                                                      uint32_t* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncomb) return;
  Jac<Fp> acc = load_jac<Fp>(work, (size_t)c * m);
  for (int k = 1; k < m; k++) acc = jac_add(acc, load_jac<Fp>(work, (size_t)c * m + k));
  g1_jac_to_words(acc, out + (size_t)c * G1_WORDS);
}

__global__ void __launch_bounds__(64) k_g2_interp_sum(int ncomb, int m, const void* __restrict__ work,
                                                      uint32_t* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncomb) return;
  Jac<Fp2> acc = load_jac<Fp2>(work, (size_t)c * m);
  for (int k = 1; k < m; k++) acc = jac_add(acc, load_jac<Fp2>(work, (size_t)c * m + k));
  g2_jac_to_words(acc, out + (size_t)c * G2_WORDS);
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

// BivarCommitment::evaluate(x, y) == G1::one() * val  (src/sync_key_gen.rs:542), from the rows
// R = row(x): evaluate(x, y) = sum_j R_j y^j (Horner with the small y).  One thread per ack.
__global__ void __launch_bounds__(256) k_bivar_check(int nack, int t, const uint32_t* __restrict__ rows,
                                                     const uint32_t* __restrict__ row_idx,
                                                     const uint32_t* __restrict__ ys, const uint32_t* __restrict__ vals,
                                                     uint8_t* __restrict__ verdict) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= nack) return;
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
  uint32_t k[8];
  for (int j = 0; j < 8; j++) k[j] = vals[(size_t)a * 8 + j];
  const Jac<Fp> w = jac_mul_affine(fp_const(G1X_M), fp_const(G1Y_M), false, k);
  verdict[a] = jac_eq(acc, w) ? 1 : 0;
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

size_t combine_work_bytes(int ncomb, int m, int g2) {
  return (size_t)ncomb * m * (g2 ? sizeof(hb::Jac<hb::Fp2>) : sizeof(hb::Jac<hb::Fp>));
}

hipError_t combine_g1(hipStream_t s, int ncomb, int m, const uint32_t* xs, const void* pts, void* work, void* out,
                      int* status) {
  if (ncomb <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_g1_interp_terms, grid_for(ncomb * m), dim3(256), 0, s, ncomb, m, xs, (const uint32_t*)pts,
                     work, status);
  hipLaunchKernelGGL(hb::k_g1_interp_sum, grid_for(ncomb, 64), dim3(64), 0, s, ncomb, m, (const void*)work,
                     (uint32_t*)out);
  return hipGetLastError();
}
hipError_t combine_g2(hipStream_t s, int ncomb, int m, const uint32_t* xs, const void* pts, void* work, void* out,
                      int* status) {
  if (ncomb <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_g2_interp_terms, grid_for(ncomb * m), dim3(256), 0, s, ncomb, m, xs, (const uint32_t*)pts,
                     work, status);
  hipLaunchKernelGGL(hb::k_g2_interp_sum, grid_for(ncomb, 64), dim3(64), 0, s, ncomb, m, (const void*)work,
                     (uint32_t*)out);
  return hipGetLastError();
}

hipError_t bivar_row(hipStream_t s, int nrow, int t, const void* commits, const uint32_t* part_idx, const uint32_t* xs,
                     void* out) {
  if (nrow <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_bivar_row, grid_for(nrow * (t + 1)), dim3(256), 0, s, nrow, t, (const uint32_t*)commits,
                     part_idx, xs, (uint32_t*)out);
  return hipGetLastError();
}
hipError_t bivar_check(hipStream_t s, int nack, int t, const void* rows, const uint32_t* row_idx, const uint32_t* ys,
                       const uint32_t* vals, uint8_t* verdict) {
  if (nack <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_bivar_check, grid_for(nack), dim3(256), 0, s, nack, t, (const uint32_t*)rows, row_idx, ys,
                     vals, verdict);
  return hipGetLastError();
}

}  // namespace hbl
