// Wire-format parsing on the GPU: pairing 0.14 G1Compressed / G2Compressed
// ::into_affine for batches of compressed points (public keys, decryption shares, ciphertext U in
// G1; signature shares, signatures, ciphertext W in G2) -- the square root that recovers y, the
// sign choice and the prime-order-subgroup check.  The host does
// the byte-level flag checks and the big-endian -> little-endian word reversal (wire.hpp).
#include <hip/hip_runtime.h>

#include "curve.hpp"
#include "fr.hpp"
#include "wire.hpp"

namespace hb {

// (p + 1) / 4 as 32-bit words (p = 3 mod 4, so a^((p+1)/4) is a square root of a square a)
__device__ __forceinline__ void sqrt_exp_words(uint32_t e[12]) {
  uint32_t w[12];
  for (int i = 0; i < 12; i++) w[i] = PM2_W[i];
  w[0] += 3;  // p - 2 + 3 = p + 1 (no carry: the low word of p - 2 is 0xffffaaa9)
  for (int i = 0; i < 12; i++) e[i] = (w[i] >> 2) | (i < 11 ? (w[i + 1] << 30) : 0u);
}

__device__ __forceinline__ Fp fp_pow_words(const Fp& a, const uint32_t e[12]) {
  Fp r = fp_one();
  for (int i = 12 * 32 - 1; i >= 0; i--) {
    r = fp_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1) r = fp_mul(r, a);
  }
  return r;
}

// canonical words a > b
__device__ __forceinline__ bool words_gt(const uint32_t* a, const uint32_t* b, int n) {
  for (int i = n - 1; i >= 0; i--)
    if (a[i] != b[i]) return a[i] > b[i];
  return false;
}

__global__ void __launch_bounds__(256) k_g1_decompress(int n, const uint32_t* __restrict__ xw,
                                                       const uint8_t* __restrict__ flags, uint32_t* __restrict__ out,
                                                       uint8_t* __restrict__ ok) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t* o = out + (size_t)i * G1_WORDS;
  const uint8_t f = flags[i];
  bool valid = false;
  uint32_t x[12], y[12];
  for (int k = 0; k < 12; k++) x[k] = xw[(size_t)i * 12 + k], y[k] = 0;
  if (f & hbl::WIRE_INFINITY) {
    valid = true;  // the point at infinity (all-zero ABI words)
    for (int k = 0; k < 12; k++) x[k] = 0;
  } else if (!(f & hbl::WIRE_REJECT)) {
    uint32_t p[12];
    for (int k = 0; k < 12; k++) p[k] = PM2_W[k];
    p[0] += 2;
    if (words_gt(p, x, 12)) {  // x < p
      const Fp xm = fp_from_words(x);
      const Fp rhs = fp_add(fp_mul(fp_sqr(xm), xm), fp_const(B1_M));
      uint32_t e[12];
      sqrt_exp_words(e);
      Fp ym = fp_pow_words(rhs, e);
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
        // prime-order subgroup: r * P == O
        uint32_t r[8];
        for (int k = 0; k < 8; k++) r[k] = FR_W[k];
        valid = jac_is_zero(jac_mul_affine(xm, ym, false, r));
      }
    }
  }
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

__device__ __forceinline__ Fp2 f2_pow_words(const Fp2& a, const uint32_t e[12]) {
  Fp2 r = f2_one();
  for (int i = 12 * 32 - 1; i >= 0; i--) {
    r = f2_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1) r = f2_mul(r, a);
  }
  return r;
}

__device__ __forceinline__ bool f2_is_minus_one(const Fp2& a) {
  return fp_eq(a.c0, fp_neg(fp_one())) && fp_is_zero(a.c1);
}

// square root in Fp2 for p = 3 mod 4 (Adj / Rodriguez-Henriquez): false when a is not a square
__device__ __forceinline__ bool f2_sqrt(const Fp2& a, Fp2& out) {
  if (f2_is_zero(a)) {
    out = f2_zero();
    return true;
  }
  uint32_t e[12];
  for (int i = 0; i < 12; i++) e[i] = PM2_W[i];
  e[0] -= 1;  // p - 3 (no borrow: the low word of p - 2 is 0xffffaaa9)
  for (int i = 0; i < 12; i++) e[i] = (e[i] >> 2) | (i < 11 ? (e[i + 1] << 30) : 0u);  // (p - 3) / 4
  const Fp2 a1 = f2_pow_words(a, e);
  const Fp2 alpha = f2_mul(f2_sqr(a1), a);
  const Fp2 a0 = f2_mul(f2_conj(alpha), alpha);  // alpha^p * alpha
  if (f2_is_minus_one(a0)) return false;
  const Fp2 x0 = f2_mul(a1, a);
  Fp2 res;
  if (f2_is_minus_one(alpha)) {
    res = {fp_neg(x0.c1), x0.c0};  // x0 * u
  } else {
    uint32_t h[12];
    for (int i = 0; i < 12; i++) h[i] = PM2_W[i];
    h[0] += 1;  // p - 1
    for (int i = 0; i < 12; i++) h[i] = (h[i] >> 1) | (i < 11 ? (h[i + 1] << 31) : 0u);  // (p - 1) / 2
    res = f2_mul(f2_pow_words(f2_add(f2_one(), alpha), h), x0);
  }
  const Fp2 chk = f2_sub(f2_sqr(res), a);
  out = res;
  return f2_is_zero(chk);
}

__global__ void __launch_bounds__(256) k_g2_decompress(int n, const uint32_t* __restrict__ xw,
                                                       const uint8_t* __restrict__ flags, uint32_t* __restrict__ out,
                                                       uint8_t* __restrict__ ok) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t* o = out + (size_t)i * G2_WORDS;
  const uint8_t f = flags[i];
  bool valid = false;
  uint32_t x[24], y[24];
  for (int k = 0; k < 24; k++) x[k] = xw[(size_t)i * 24 + k], y[k] = 0;
  if (f & hbl::WIRE_INFINITY) {
    valid = true;
    for (int k = 0; k < 24; k++) x[k] = 0;
  } else if (!(f & hbl::WIRE_REJECT)) {
    uint32_t p[12];
    for (int k = 0; k < 12; k++) p[k] = PM2_W[k];
    p[0] += 2;
    if (words_gt(p, x, 12) && words_gt(p, x + 12, 12)) {
      const Fp2 xm = {fp_from_words(x), fp_from_words(x + 12)};
      const Fp2 b2 = {fp_const(B1_M), fp_const(B1_M)};  // 4 (1 + u)
      const Fp2 rhs = f2_add(f2_mul(f2_sqr(xm), xm), b2);
      Fp2 ym;
      if (f2_sqrt(rhs, ym)) {
        const Fp2 ny = f2_neg(ym);
        if (f2_gt_canon(ym, ny) != ((f & hbl::WIRE_GREATEST) != 0)) ym = ny;
        fp_to_words(ym.c0, y);
        fp_to_words(ym.c1, y + 12);
        uint32_t r[8];
        for (int k = 0; k < 8; k++) r[k] = FR_W[k];
        valid = jac_is_zero(jac_mul_affine(xm, ym, false, r));
      }
    }
  }
  for (int k = 0; k < 24; k++) {
    o[k] = valid ? x[k] : 0u;
    o[24 + k] = valid ? y[k] : 0u;
  }
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
  hipLaunchKernelGGL(hb::k_g1_decompress, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, xw, flags,
                     (uint32_t*)out, ok);
  return hipGetLastError();
}

hipError_t g2_decompress(hipStream_t s, int n, const uint32_t* xw, const uint8_t* flags, void* out, uint8_t* ok) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_g2_decompress, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, xw, flags,
                     (uint32_t*)out, ok);
  return hipGetLastError();
}

}  // namespace hbl
