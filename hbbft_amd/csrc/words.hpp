// Multi-word (32-bit limb) helpers shared by both field representations (fp.hpp, and the lane-pair
// kernels over sfp.hpp): canonical-word comparisons and the variable-time binary-Euclid inverse.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define HW_HD __host__ __device__ __forceinline__
#else
#define HW_HD inline
#endif

namespace hb {

// Variable-time inverse for public values (HB_FP_LATENCY kernels: the single-thread affine output of
// combines and scalar multiples, whose inputs and results are public): binary extended Euclid over
// canonical 32-bit words, ~2 x 381 shift/subtract steps instead of 381 squarings + 190 products.
// Divergent across lanes, so kernels where every lane inverts keep the uniform Fermat form.
template <int N>
HW_HD bool words_is_one(const uint32_t* x) {
  uint32_t o = x[0] ^ 1u;
  for (int i = 1; i < N; i++) o |= x[i];
  return o == 0;
}
template <int N>
HW_HD void words_shr1(uint32_t* x, uint32_t top) {
  for (int i = 0; i < N - 1; i++) x[i] = (x[i] >> 1) | (x[i + 1] << 31);
  x[N - 1] = (x[N - 1] >> 1) | (top << 31);
}
template <int N>
HW_HD uint32_t words_add(uint32_t* x, const uint32_t* y) {
  uint64_t c = 0;
  for (int i = 0; i < N; i++) {
    c += (uint64_t)x[i] + y[i];
    x[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)c;
}
template <int N>
HW_HD uint32_t words_sub(uint32_t* x, const uint32_t* y) {  // returns the borrow
  uint64_t br = 0;
  for (int i = 0; i < N; i++) {
    const uint64_t d = (uint64_t)x[i] - y[i] - br;
    x[i] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
  return (uint32_t)br;
}
template <int N>
HW_HD bool words_geq(const uint32_t* x, const uint32_t* y) {
  for (int i = N - 1; i >= 0; i--)
    if (x[i] != y[i]) return x[i] > y[i];
  return true;
}
// out = a^-1 mod `mod` (odd), a canonical and nonzero
template <int N>
HW_HD void words_inv_vartime(const uint32_t* a, const uint32_t* mod, uint32_t* out) {
  uint32_t u[N], v[N], x1[N], x2[N];
  for (int i = 0; i < N; i++) {
    u[i] = a[i];
    v[i] = mod[i];
    x1[i] = 0;
    x2[i] = 0;
  }
  x1[0] = 1;
  while (!words_is_one<N>(u) && !words_is_one<N>(v)) {
    while ((u[0] & 1) == 0) {
      words_shr1<N>(u, 0);
      const uint32_t c = (x1[0] & 1) ? words_add<N>(x1, mod) : 0;
      words_shr1<N>(x1, c);
    }
    while ((v[0] & 1) == 0) {
      words_shr1<N>(v, 0);
      const uint32_t c = (x2[0] & 1) ? words_add<N>(x2, mod) : 0;
      words_shr1<N>(x2, c);
    }
    if (words_geq<N>(u, v)) {
      words_sub<N>(u, v);
      if (words_sub<N>(x1, x2)) words_add<N>(x1, mod);
    } else {
      words_sub<N>(v, u);
      if (words_sub<N>(x2, x1)) words_add<N>(x2, mod);
    }
  }
  const bool one_u = words_is_one<N>(u);
  for (int i = 0; i < N; i++) out[i] = one_u ? x1[i] : x2[i];
}

}  // namespace hb
