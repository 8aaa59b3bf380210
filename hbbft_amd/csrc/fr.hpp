// BLS12-381 scalar field Fr (r = 0x73ed...0001, 255 bits) on gfx950: 8 x 32-bit limbs,
// Montgomery R = 2^256, CIOS with 64-bit products.  Only the Lagrange coefficients of
// threshold_crypto's interpolate() run in Fr (a few hundred products per coefficient), so this is
// the plain form; the hot multi-precision work is in Fp (fp.hpp).
// Constants derived by tools/gen_constants.py's arithmetic (r, -r^-1 mod 2^32, 2^512 mod r).
#pragma once
#include <stdint.h>

#include "fp.hpp"  // HB_HD

namespace hb {

constexpr int FRL = 8;
constexpr uint32_t FR_W[FRL] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
constexpr uint32_t FR_NP0 = 0xffffffffu;  // -r^-1 mod 2^32
constexpr uint32_t FR_R2[FRL] = {0xf3f29c6du, 0xc999e990u, 0x87925c23u, 0x2b6cedcbu,
                                 0x7254398fu, 0x05d31496u, 0x9f59ff11u, 0x0748d9d9u};  // 2^512 mod r
constexpr uint32_t FR_ONE_M[FRL] = {0xfffffffeu, 0x00000001u, 0x00034802u, 0x5884b7fau,
                                    0xecbc4ff5u, 0x998c4fefu, 0xacc5056fu, 0x1824b159u};  // 2^256 mod r
constexpr uint32_t FR_RM2[FRL] = {0xffffffffu, 0xfffffffeu, 0xfffe5bfeu, 0x53bda402u,
                                  0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};  // r - 2

struct Fr {
  uint32_t l[FRL];
};

HB_HD Fr fr_raw(const uint32_t (&c)[FRL]) {
  Fr r;
#pragma unroll
  for (int i = 0; i < FRL; i++) r.l[i] = c[i];
  return r;
}

// x < r  ->  x - r if x >= r else x  (with an explicit carry word `hi` from the caller)
HB_HD Fr fr_csub(const uint32_t* t, uint32_t hi) {
  uint32_t s[FRL];
  uint64_t br = 0;
#pragma unroll
  for (int j = 0; j < FRL; j++) {
    const uint64_t d = (uint64_t)t[j] - FR_W[j] - br;
    s[j] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
  const bool ge = hi || !br;
  Fr r;
#pragma unroll
  for (int j = 0; j < FRL; j++) r.l[j] = ge ? s[j] : t[j];
  return r;
}

// Montgomery product a b / 2^256 mod r (inputs < r, output < r)
HB_HD Fr fr_mul(const Fr& a, const Fr& b) {
  uint32_t t[FRL + 2];
#pragma unroll
  for (int j = 0; j < FRL + 2; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < FRL; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < FRL; j++) {
      c = (uint64_t)a.l[j] * b.l[i] + t[j] + (c >> 32);
      t[j] = (uint32_t)c;
    }
    c = (uint64_t)t[FRL] + (c >> 32);
    t[FRL] = (uint32_t)c;
    t[FRL + 1] = (uint32_t)(c >> 32);
    const uint32_t m = t[0] * FR_NP0;
    c = (uint64_t)m * FR_W[0] + t[0];
#pragma unroll
    for (int j = 1; j < FRL; j++) {
      c = (uint64_t)m * FR_W[j] + t[j] + (c >> 32);
      t[j - 1] = (uint32_t)c;
    }
    c = (uint64_t)t[FRL] + (c >> 32);
    t[FRL - 1] = (uint32_t)c;
    t[FRL] = t[FRL + 1] + (uint32_t)(c >> 32);
  }
  return fr_csub(t, t[FRL]);
}

HB_HD Fr fr_sub(const Fr& a, const Fr& b) {
  uint32_t t[FRL];
  uint64_t br = 0;
#pragma unroll
  for (int j = 0; j < FRL; j++) {
    const uint64_t d = (uint64_t)a.l[j] - b.l[j] - br;
    t[j] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
  if (br) {  // add r back
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < FRL; j++) {
      c = (uint64_t)t[j] + FR_W[j] + (c >> 32);
      t[j] = (uint32_t)c;
    }
  }
  Fr r;
#pragma unroll
  for (int j = 0; j < FRL; j++) r.l[j] = t[j];
  return r;
}

HB_HD bool fr_is_zero(const Fr& a) {
  uint32_t o = 0;
#pragma unroll
  for (int j = 0; j < FRL; j++) o |= a.l[j];
  return o == 0;
}

// small integer v (< 2^32) into Montgomery form
HB_HD Fr fr_from_u32(uint32_t v) {
  Fr a;
#pragma unroll
  for (int j = 0; j < FRL; j++) a.l[j] = 0;
  a.l[0] = v;
  return fr_mul(a, fr_raw(FR_R2));
}
// Montgomery -> canonical integer words
HB_HD Fr fr_to_canon(const Fr& a) {
  Fr one;
#pragma unroll
  for (int j = 0; j < FRL; j++) one.l[j] = 0;
  one.l[0] = 1;
  return fr_mul(a, one);
}
// a^(r-2) (a != 0)
HB_HD Fr fr_inv(const Fr& a) {
  Fr r = fr_raw(FR_ONE_M);
  for (int i = 254; i >= 0; i--) {
    r = fr_mul(r, r);
    if ((FR_RM2[i >> 5] >> (i & 31)) & 1) r = fr_mul(r, a);
  }
  return r;
}

}  // namespace hb
