// Wire-format parsing on the GPU: pairing 0.14 G1Compressed / G2Compressed
// ::into_affine for batches of compressed points (public keys, decryption shares, ciphertext U in
// G1; signature shares, signatures, ciphertext W in G2) -- the square root that recovers y, the
// sign choice and the prime-order-subgroup check (round 6: norm-method square root over one
// windowed exponentiation chain, endomorphism subgroup tests).  The host does
// the byte-level flag checks and the big-endian -> little-endian word reversal (wire.hpp).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "curve.hpp"
#include "wire.hpp"
#include "sqrt_chain.inc"

#ifndef HBH_G1_WAVES_PER_SIMD
#define HBH_G1_WAVES_PER_SIMD 2  // A/B: 1 (512 registers, no spills, half the waves in flight)
#endif

namespace hb {

// canonical words a > b
__device__ __forceinline__ bool words_gt(const uint32_t* a, const uint32_t* b, int n) {
  for (int i = n - 1; i >= 0; i--)
    if (a[i] != b[i]) return a[i] > b[i];
  return false;
}

// ---------------------------------------------------------------------------- subgroup membership
// Endomorphism tests instead of r * P == O (255-bit double-and-add):
//   G1: P in G1  <=>  phi(P) == [-x^2] P,  phi(x, y) = (beta x, y)            (Scott, eprint 2021/1130)
//   G2: P in G2  <=>  psi(P) == [x] P,     psi the untwist-Frobenius-twist map  (same note)
// with x = -|x| = -0xd201000000010000.  Exact on the whole curve, not only on likely inputs: on the
// l-power torsion of any prime l != r, phi + [x^2] has determinant x^4 - x^2 + 1 = r (phi^2 + phi +
// 1 = 0) and psi - [x] has x^2 - t x + p = p - x = h1 r (psi^2 - t psi + p = 0, t = x + 1), units mod
// every prime of h1 and h2, so neither map vanishes on a point outside the r-torsion
// (tests/test_subgroup_criteria.py).  [|x|] is 63 doublings + 5 additions (|x| has 6 set bits), so
// G2 pays 68 group operations instead of ~383 and G1 two such chains.  Both criteria are
// equalities of points, so a non-subgroup point whose chain hits an exceptional addition (P = +-Q,
// O) is handled by the group law's explicit cases (curve.hpp).  tests/test_gpu_wire_subgroup.py
// pins accept / reject against the oracle's r * P test on random on-curve points and on points of
// every prime order dividing the cofactors.

// [|x|] P for an affine P (not infinity): double-and-add over the constant |x|, one mixed addition
// per set bit.  Not unrolled: the loop control is uniform and one copy stays in the I-cache.
template <class F>
__device__ __forceinline__ Jac<F> mul_absx_affine(const F& x, const F& y) {
  Jac<F> acc = jac_from_affine(x, y, false);
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    acc = jac_dbl(acc);
    if ((X_ABS >> i) & 1) acc = jac_add_affine(acc, x, y);
  }
  return acc;
}

template <class F>
__device__ __forceinline__ Jac<F> mul_absx_jac(const Jac<F>& p) {
  Jac<F> acc = p;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    acc = jac_dbl(acc);
    if ((X_ABS >> i) & 1) acc = jac_add(acc, p);
  }
  return acc;
}

// Jacobian q == affine (x, y) (not infinity)
template <class F>
__device__ __forceinline__ bool jac_eq_affine(const Jac<F>& q, const F& x, const F& y) {
  if (jac_is_zero(q)) return false;
  const F z2 = fsqr(q.z);
  if (!fisz(fsub(q.x, fmul(x, z2)))) return false;
  return fisz(fsub(q.y, fmul(y, fmul(z2, q.z))));
}

// [-x^2] P == phi(P)  <=>  [|x|]([|x|] P) == -phi(P) = (beta x, -y)
__device__ __forceinline__ bool g1_in_subgroup(const Fp& x, const Fp& y) {
  const Jac<Fp> q = mul_absx_jac(mul_absx_affine(x, y));
  return jac_eq_affine(q, fp_mul(x, fp_const(BETA_M)), fp_neg(y));
}

// ---------------------------------------------------------------------------- decompression
// G1: two waves per 64 points (k_g1_decompress, 128 threads).  The subgroup test does not need y:
// (x, y) -> (u^2 x, u^3 y) with u = y maps E: y^2 = x^3 + 4 isomorphically onto E_u: Y^2 = X^3 + 4 rhs^3
// (rhs = x^3 + 4 = y^2) and sends (x, y) to P' = (rhs x, rhs^2) -- known from x alone.  The map
// commutes with scalar multiplication and with phi (beta scales X by the same u^2), and the a = 0
// Jacobian formulas never read b, so phi(P') == [-x^2] P'  <=>  phi(P) == [-x^2] P.  Wave 0 takes the
// square root (375 squarings + 86 products) while wave 1 runs the subgroup test on P' (two [|x|]
// chains): each point's serial chain is the longer of the two instead of their sum, and 65,536
// points are two waves per SIMD instead of one (the decoder is issue-bound at one wave per SIMD:
// profiles/r06/c3_wire/decode_pmc_sq.csv, ~5.1 cycles per VALU instruction).  When rhs is not a
// square, P' lies on a twist and wave 1's answer is discarded with the point.
__global__ void __launch_bounds__(128, HBH_G1_WAVES_PER_SIMD) k_g1_decompress(int n, const uint32_t* __restrict__ xw,
                                                       const uint8_t* __restrict__ flags, uint32_t* __restrict__ out,
                                                       uint8_t* __restrict__ ok) {
  __shared__ uint8_t in_group[64];
  const int lane = threadIdx.x & 63, role = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const bool live = i < n;
  const uint8_t f = live ? flags[i] : hbl::WIRE_REJECT;
  uint32_t x[12];
  for (int k = 0; k < 12; k++) x[k] = live ? xw[(size_t)i * 12 + k] : 0u;
  uint32_t p[12];
  for (int k = 0; k < 12; k++) p[k] = PM2_W[k];
  p[0] += 2;
  const bool try_point = !(f & hbl::WIRE_INFINITY) && !(f & hbl::WIRE_REJECT) && words_gt(p, x, 12);  // x < p
  Fp xm = fp_zero(), rhs = fp_zero();
  if (try_point) {
    xm = fp_from_words(x);
    rhs = fp_add(fp_mul(fp_sqr(xm), xm), fp_const(B1_M));
  }
  bool valid = false;
  uint32_t y[12];
  for (int k = 0; k < 12; k++) y[k] = 0;
  if (role == 1) {  // the subgroup test on P' = (rhs x, rhs^2)
    bool g = false;
    if (try_point) g = g1_in_subgroup(fp_mul(rhs, xm), fp_sqr(rhs));
    in_group[lane] = g ? 1 : 0;
  } else if (f & hbl::WIRE_INFINITY) {
    valid = true;  // the point at infinity (all-zero ABI words)
    for (int k = 0; k < 12; k++) x[k] = 0;
  } else if (try_point) {  // the square root, beside the other wave's subgroup test
    Fp ym = fp_mul(rhs, fp_pow_pm3d4(rhs));  // rhs^((p+1)/4)
    if (fp_eq(fp_sqr(ym), rhs)) {
      // "greatest" = y > p - y, i.e. y > (p - 1) / 2
      fp_to_words(ym, y);
      uint32_t half[12];
      for (int k = 0; k < 12; k++) half[k] = (p[k] >> 1) | (k < 11 ? (p[k + 1] << 31) : 0u);
      const bool greatest = words_gt(y, half, 12);
      if (greatest != ((f & hbl::WIRE_GREATEST) != 0)) {
        ym = fp_neg(ym);
        fp_to_words(ym, y);
      }
      valid = true;  // on the curve; the subgroup verdict joins after the barrier
    }
  }
  __syncthreads();
  if (role == 1 || !live) return;
  if (try_point) valid = valid && in_group[lane] != 0;
  uint32_t* o = out + (size_t)i * G1_WORDS;
  for (int k = 0; k < 12; k++) {
    o[k] = valid ? x[k] : 0u;
    o[12 + k] = valid ? y[k] : 0u;
  }
  ok[i] = valid ? 1 : 0;
}

// pairing 0.14 Ord for Fq2: c1 first, then c0 (canonical integers)
__device__ __forceinline__ bool f2_gt_canon(const Fp2& a, const Fp2& b) {
  uint32_t a0[12], a1[12], b0[12], b1[12];
  fp_to_words(a.c0, a0);
  fp_to_words(a.c1, a1);
  fp_to_words(b.c0, b0);
  fp_to_words(b.c1, b1);
  bool eq1 = true;
  for (int k = 0; k < 12; k++) eq1 = eq1 && a1[k] == b1[k];
  return eq1 ? words_gt(a0, b0, 12) : words_gt(a1, b1, 12);
}

// Square root in Fp2 by the norm (two Fp exponentiations by (p-3)/4 instead of two Fp2 ones):
// a = a0 + a1 u is a square iff N = a0^2 + a1^2 is a square in Fp; with s = sqrt(N) and
// t = (a0 + s) / 2 (or (a0 - s) / 2 when that is 0), w = t^((p-3)/4):
//   t w^2 ==  1 (t a square):      y = t w + (a1 w / 2) u
//   t w^2 == -1 (-t a square; p = 3 mod 8 makes (-1)^((p-3)/4) = 1, so w serves -t too):
//                                  y = a1 w / 2 - (t w) u
// (t (a0 - s)/2 = -a1^2 / 4 is a non-square for a1 != 0, so exactly one case holds.)  Any root:
// the caller picks the sign.  false when a is not a square.
__device__ __forceinline__ bool f2_sqrt_norm(const Fp2& a, Fp2& out) {
  out = f2_zero();
  if (f2_is_zero(a)) return true;
  const Fp nrm = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  const Fp s = fp_mul(nrm, fp_pow_pm3d4(nrm));
  if (!fp_eq(fp_sqr(s), nrm)) return false;
  const Fp half = fp_const(INV2_M);
  Fp t = fp_mul(fp_add(a.c0, s), half);
  if (fp_is_zero(t)) t = fp_mul(fp_sub(a.c0, s), half);
  const Fp w = fp_pow_pm3d4(t);
  const Fp tw = fp_mul(t, w);
  const Fp aw = fp_mul(fp_mul(a.c1, half), w);
  const bool qr = fp_eq(fp_mul(tw, w), fp_one());
  const Fp2 y = qr ? Fp2{tw, aw} : Fp2{aw, fp_neg(tw)};
  out = y;
  return f2_is_zero(f2_sub(f2_sqr(y), a));
}

// G2: two waves per 64 points, as G1.  The subgroup test needs y only through its norm: with
// rhs = x^3 + b = y^2, iota(X, Y) = (y^2 X, y^3 Y) maps E' isomorphically onto Y^2 = X^3 + b rhs^3 and
// sends P to P' = (rhs x, rhs^2) -- known from x alone -- and psi(P) = (C1 conj(x), C2 conj(y)) to
// (C1 rhs conj(x), C2 rhs N(y)) with N(y) = y conj(y) in Fp (the same for both roots).  iota commutes
// with [k] and the a = 0 formulas never read b, so psi(P) == -[|x|] P  <=>  [|x|] P' == (C1 rhs conj(x),
// -C2 rhs N(y)) (tests/test_subgroup_criteria.py checks the equivalence on every cofactor torsion).
// Wave 1 runs [|x|] P' (68 group operations over Fp2) while wave 0 takes the square root (two
// (p - 3) / 4 chains); wave 0 then publishes N(y) through LDS and wave 1 finishes the comparison.
// #E'(Fp2) = h2 r is odd, so no point has rhs = 0 (where iota would degenerate).
template <int WPS>
__global__ void __launch_bounds__(128, WPS) k_g2_decompress(int n, const uint32_t* __restrict__ xw,
                                                       const uint8_t* __restrict__ flags, uint32_t* __restrict__ out,
                                                       uint8_t* __restrict__ ok) {
  __shared__ uint32_t nrm[NL * 64];
  __shared__ uint8_t in_group[64];
  const int lane = threadIdx.x & 63, role = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const bool live = i < n;
  const uint8_t f = live ? flags[i] : hbl::WIRE_REJECT;
  const uint32_t* xi = xw + (size_t)(live ? i : 0) * 24;
  uint32_t* o = out + (size_t)(live ? i : 0) * G2_WORDS;
  bool try_point;
  {
    uint32_t x[24], p[12];
    for (int k = 0; k < 24; k++) x[k] = xi[k];
    for (int k = 0; k < 12; k++) p[k] = PM2_W[k];
    p[0] += 2;
    try_point = !(f & hbl::WIRE_INFINITY) && !(f & hbl::WIRE_REJECT) && words_gt(p, x, 12) && words_gt(p, x + 12, 12);
  }
  const Fp2 b2 = {fp_const(B1_M), fp_const(B1_M)};  // 4 (1 + u)
  bool valid = false, gx = false;
  Fp2 qy, w;  // wave 1 only, across the barrier: [|x|] P' .y and the Y target before its factor N(y)
  if (role == 1) {
    if (try_point) {
      Fp2 xm = {fp_from_words(xi), fp_from_words(xi + 12)};
      Fp2 rhs = f2_add(f2_mul(f2_sqr(xm), xm), b2);
      const Jac<Fp2> q = mul_absx_affine(f2_mul(rhs, xm), f2_sqr(rhs));
      xm = {fp_from_words(xi), fp_from_words(xi + 12)};  // reloaded: not live across the chain
      rhs = f2_add(f2_mul(f2_sqr(xm), xm), b2);
      // target iota(-psi(P)) = (C1 rhs conj(x), -C2 rhs N(y)); C1 = c1 u, so C1 conj(x) = (x1 c1, x0 c1)
      const Fp c1 = fp_const(PSI_C1_C1);
      const Fp2 tx = f2_mul(rhs, Fp2{fp_mul(xm.c1, c1), fp_mul(xm.c0, c1)});
      const Fp2 z2 = f2_sqr(q.z);
      gx = !jac_is_zero(q) && f2_is_zero(f2_sub(q.x, f2_mul(tx, z2)));
      w = f2_neg(f2_mul(f2_mul(rhs, Fp2{fp_const(PSI_C2_C0), fp_const(PSI_C2_C1)}), f2_mul(z2, q.z)));
      qy = q.y;
    }
  } else if (f & hbl::WIRE_INFINITY) {
    valid = live;  // the point at infinity (all-zero ABI words)
    if (live)
      for (int k = 0; k < G2_WORDS; k++) o[k] = 0u;
  } else if (try_point) {
    const Fp2 xm = {fp_from_words(xi), fp_from_words(xi + 12)};
    const Fp2 rhs = f2_add(f2_mul(f2_sqr(xm), xm), b2);
    Fp2 ym;
    if (f2_sqrt_norm(rhs, ym)) {
      const Fp2 ny = f2_neg(ym);
      if (f2_gt_canon(ym, ny) != ((f & hbl::WIRE_GREATEST) != 0)) ym = ny;
      const Fp nm = fp_add(fp_sqr(ym.c0), fp_sqr(ym.c1));
      for (int k = 0; k < NL; k++) nrm[k * 64 + lane] = nm.l[k];
      // on the curve: written now, zeroed after the second barrier when not in the subgroup
      for (int k = 0; k < 24; k++) o[k] = xi[k];
      fp_to_words(ym.c0, o + 24);
      fp_to_words(ym.c1, o + 36);
      valid = true;
    }
  }
  __syncthreads();
  if (role == 1) {
    bool g = false;
    if (try_point && gx) {
      Fp nm;
      for (int k = 0; k < NL; k++) nm.l[k] = nrm[k * 64 + lane];
      g = f2_is_zero(f2_sub(qy, Fp2{fp_mul(w.c0, nm), fp_mul(w.c1, nm)}));
    }
    in_group[lane] = g ? 1 : 0;
  }
  __syncthreads();
  if (role == 1 || !live) return;
  if (try_point) valid = valid && in_group[lane] != 0;
  if (!valid)
    for (int k = 0; k < G2_WORDS; k++) o[k] = 0u;
  ok[i] = valid ? 1 : 0;
}

// Byte-level half of the decoding on the device, for encodings already in HBM (the _dev entry
// points): the same flag rules and word reversal as the host's parse_compressed (engine.hip).
// One thread per encoding of nfe 48-byte big-endian field elements.
__global__ void __launch_bounds__(256) k_wire_parse(int n, int nfe, const uint8_t* __restrict__ in,
                                                    uint32_t* __restrict__ xw, uint8_t* __restrict__ flags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* b = in + (size_t)i * 48 * nfe;
  const uint8_t b0 = b[0];
  uint8_t f = 0;
  if (!(b0 & 0x80)) {
    f = hbl::WIRE_REJECT;
  } else if (b0 & 0x40) {
    bool zero = (b0 & 0x3f) == 0;
    for (int k = 1; k < 48 * nfe; k++) zero = zero && b[k] == 0;
    f = zero ? hbl::WIRE_INFINITY : hbl::WIRE_REJECT;
  } else if (b0 & 0x20) {
    f = hbl::WIRE_GREATEST;
  }
  for (int c = 0; c < nfe; c++) {
    const uint8_t* e = b + 48 * (nfe - 1 - c);
    for (int w = 0; w < 12; w++) {
      uint32_t v = 0;
      for (int k = 0; k < 4; k++) {
        const int pos = 47 - (w * 4 + k);
        const uint8_t byte = (c == nfe - 1 && pos == 0) ? (uint8_t)(b0 & 0x1f) : e[pos];
        v |= (uint32_t)byte << (8 * k);
      }
      xw[((size_t)i * nfe + c) * 12 + w] = v;
    }
  }
  flags[i] = f;
}

}  // namespace hb

namespace hbl {

hipError_t wire_parse(hipStream_t s, int n, int nfe, const uint8_t* in, uint32_t* xw, uint8_t* flags) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_wire_parse, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, nfe, in, xw, flags);
  return hipGetLastError();
}

hipError_t g1_decompress(hipStream_t s, int n, const uint32_t* xw, const uint8_t* flags, void* out, uint8_t* ok) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_g1_decompress, dim3((unsigned)((n + 63) / 64)), dim3(128), 0, s, n, xw, flags,
                     (uint32_t*)out, ok);
  return hipGetLastError();
}

hipError_t g2_decompress(hipStream_t s, int n, const uint32_t* xw, const uint8_t* flags, void* out, uint8_t* ok) {
  if (n <= 0) return hipSuccess;
  // one wave per SIMD: 512 registers, no spills; two: 256 registers (spills) and twice the waves in flight
  static const int waves = [] {
    const char* v = std::getenv("HBH_G2_DEC_WAVES");
    return v ? std::atoi(v) : 2;
  }();
  if (waves == 1)
    hipLaunchKernelGGL(hb::k_g2_decompress<1>, dim3((unsigned)((n + 63) / 64)), dim3(128), 0, s, n, xw, flags,
                       (uint32_t*)out, ok);
  else
    hipLaunchKernelGGL(hb::k_g2_decompress<2>, dim3((unsigned)((n + 63) / 64)), dim3(128), 0, s, n, xw, flags,
                       (uint32_t*)out, ok);
  return hipGetLastError();
}

}  // namespace hbl
