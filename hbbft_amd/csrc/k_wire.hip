// Wire-format parsing on the GPU: pairing 0.14 G1Compressed::into_affine for
// batches of 48-byte compressed G1 points (public keys, decryption shares, ciphertext U) -- the
// square root that recovers y, the sign choice and the prime-order-subgroup check.  The host does
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

}  // namespace hb

namespace hbl {

hipError_t g1_decompress(hipStream_t s, int n, const uint32_t* xw, const uint8_t* flags, void* out, uint8_t* ok) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_g1_decompress, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, xw, flags,
                     (uint32_t*)out, ok);
  return hipGetLastError();
}

}  // namespace hbl
