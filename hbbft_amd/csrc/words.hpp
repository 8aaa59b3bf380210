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

// Variable-time inverse for public values (the affine outputs of combines and scalar multiples,
// the final exponentiation's one inversion in the wave kernel): a batched binary GCD over canonical
// 32-bit words.  Divergent across lanes, so kernels where every lane inverts keep the uniform
// Fermat form.
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
// Bit length of an N-word value (0 for zero); branch-free over the words so that x stays in VGPRs.
template <int N>
HW_HD int words_bitlen(const uint32_t* x) {
  int len = 0;
#pragma unroll
  for (int i = 0; i < N; i++)
    if (x[i]) len = 32 * i + 32 - __builtin_clz(x[i]);
  return len;
}
// 64 bits of x starting at bit s (bits beyond the top read as zero), selected without dynamic
// register indexing
template <int N>
HW_HD uint64_t words_bits64(const uint32_t* x, int s) {
  const int w = s >> 5, sh = s & 31;
  uint32_t lo = 0, mid = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    lo = (i == w) ? x[i] : lo;
    mid = (i == w + 1) ? x[i] : mid;
    hi = (i == w + 2) ? x[i] : hi;
  }
  const uint64_t v = (uint64_t)lo | ((uint64_t)mid << 32);
  return sh ? (v >> sh) | ((uint64_t)hi << (64 - sh)) : v;
}
// t = x * fx + y * fy (x, y < 2^(32N) unsigned; |fx|, |fy| <= 2^31) as an (N+2)-word two's-complement
// value, shifted right (arithmetically) by 31 bits into N+1 words
template <int N>
HW_HD void words_lincomb_shr31(const uint32_t* x, int64_t fx, const uint32_t* y, int64_t fy, uint32_t* out) {
  uint32_t t[N + 2];
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const int64_t p1 = (int64_t)x[i] * fx, p2 = (int64_t)y[i] * fy;
    const int64_t sw = (int64_t)(uint32_t)p1 + (int64_t)(uint32_t)p2 + c;
    t[i] = (uint32_t)sw;
    c = (sw >> 32) + (p1 >> 32) + (p2 >> 32);
  }
  t[N] = (uint32_t)c;
  t[N + 1] = (uint32_t)(c >> 32);
#pragma unroll
  for (int i = 0; i <= N; i++) out[i] = (t[i] >> 31) | (t[i + 1] << 1);
}
template <int N>
HW_HD bool words_neg_if(uint32_t* x, bool neg) {  // two's-complement negation of N words when neg
  if (!neg) return false;
  uint64_t c = 1;
#pragma unroll
  for (int i = 0; i < N; i++) {
    c += (uint64_t)(uint32_t)~x[i];
    x[i] = (uint32_t)c;
    c >>= 32;
  }
  return true;
}

// out = (x fx + y fy + q mod) / 2^31 for signed (N+1)-word x, y (two's complement, top word signed),
// |fx|, |fy| <= 2^31, q in [0, 2^31) chosen (minv = -mod^-1 mod 2^32) so the sum is divisible by 2^31;
// out has N+1 words, signed (the caller keeps |out| < 2^(32N+31))
template <int N>
HW_HD void words_lin_mont31(const uint32_t* x, int64_t fx, const uint32_t* y, int64_t fy, const uint32_t* mod,
                            uint32_t minv, uint32_t* out) {
  const uint32_t t0 = (uint32_t)((uint64_t)x[0] * (uint64_t)fx + (uint64_t)y[0] * (uint64_t)fy);
  const uint64_t q = (uint64_t)((t0 * minv) & 0x7fffffffu);
  uint32_t t[N + 2];
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i <= N; i++) {
    const int64_t xi = i < N ? (int64_t)x[i] : (int64_t)(int32_t)x[N];
    const int64_t yi = i < N ? (int64_t)y[i] : (int64_t)(int32_t)y[N];
    const int64_t p1 = xi * fx, p2 = yi * fy;
    const uint64_t p3 = i < N ? q * mod[i] : 0;
    const int64_t sw = (int64_t)(uint32_t)p1 + (int64_t)(uint32_t)p2 + (int64_t)(uint32_t)p3 + c;
    t[i] = (uint32_t)sw;
    c = (sw >> 32) + (p1 >> 32) + (p2 >> 32) + (int64_t)(p3 >> 32);
  }
  t[N + 1] = (uint32_t)c;
#pragma unroll
  for (int i = 0; i <= N; i++) out[i] = (t[i] >> 31) | (t[i + 1] << 1);
}

// out = a^-1 mod `mod` (odd modulus of at most 32N - 2 bits, a canonical); 0 when a is 0 or not
// invertible.  Variable time, for public values only.  T. Pornin's optimized binary GCD
// (eprint 2020/972, Algorithm 2): the binary GCD's 2 len(m) - 1 divsteps in rounds of 31, each round
// deciding on 64-bit approximations of (a, b) -- the low 31 bits and the top 33 bits -- and then
// applying the round's 2x2 update matrix to the full a, b and to the coefficients u, v (divided
// by 2^31 mod m, Montgomery style).  ~25 rounds for a 381-bit modulus instead of ~760 multiword
// shift / subtract steps.  Fixed round count: no data-dependent termination.
// MODE (for callers whose lanes invert the same value, the wave kernels' one inversion; divergent
// callers keep 0): bit 0 (INV_BATCH) takes a run of even divsteps at once (count trailing zeros,
// shift, double the coefficients) -- the same divsteps in ~1/3 of the loop iterations; bit 1
// (INV_LAZY) takes the bit length of a | b once and keeps the coefficients u, v signed and unreduced across the
// rounds (one reduction at the end) -- fewer instructions, but more live registers: the two-wave
// k_wave64 takes it, the 256-register k_wave does not (it spills there).
constexpr int INV_BATCH = 1, INV_LAZY = 2;
template <int N, int MODE = 0>
HW_HD void words_inv_vartime(const uint32_t* y, const uint32_t* mod, uint32_t* out) {
  constexpr bool BATCH = (MODE & INV_BATCH) != 0, LAZY = (MODE & INV_LAZY) != 0;
  uint32_t a[N + 1], b[N + 1], u[N + 1], v[N + 1];
#pragma unroll
  for (int i = 0; i < N; i++) {
    a[i] = y[i];
    b[i] = mod[i];
    u[i] = 0;
    v[i] = 0;
  }
  a[N] = b[N] = u[N] = v[N] = 0;
  u[0] = 1;
  // -mod^-1 mod 2^32 (Newton)
  uint32_t inv = mod[0];
  for (int k = 0; k < 5; k++) inv *= 2u - mod[0] * inv;
  const uint32_t minv = 0u - inv;
  const int rounds = (2 * words_bitlen<N>(mod) - 1 + 30) / 31;
  for (int r = 0; r < rounds; r++) {
    int n;
    if (LAZY) {  // max(len a, len b) = len(a | b) (in k_wave this form measured slower: kept to k_wave64)
      uint32_t o[N];
#pragma unroll
      for (int i = 0; i < N; i++) o[i] = a[i] | b[i];
      n = words_bitlen<N>(o);
    } else {
      n = words_bitlen<N>(a);
      const int nb = words_bitlen<N>(b);
      if (nb > n) n = nb;
    }
    if (n < 64) n = 64;
    uint64_t ab = ((uint64_t)a[0] & 0x7fffffffu) | (words_bits64<N>(a, n - 33) << 31);
    uint64_t bb = ((uint64_t)b[0] & 0x7fffffffu) | (words_bits64<N>(b, n - 33) << 31);
    int64_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
    if (BATCH) {
      int j = 0;
      while (true) {
        const int tz = ab ? __builtin_ctzll(ab) : 64;
        const int z = tz < 31 - j ? tz : 31 - j;  // even divsteps
        ab >>= z;
        f1 <<= z;
        g1 <<= z;
        j += z;
        if (j >= 31) break;
        if (ab < bb) {  // odd divstep
          const uint64_t t = ab;
          ab = bb;
          bb = t;
          int64_t q = f0;
          f0 = f1;
          f1 = q;
          q = g0;
          g0 = g1;
          g1 = q;
        }
        ab = (ab - bb) >> 1;
        f0 -= f1;
        g0 -= g1;
        f1 *= 2;
        g1 *= 2;
        if (++j >= 31) break;
      }
    }
    for (int j = 0; j < (BATCH ? 0 : 31); j++) {
      if (ab & 1) {
        if (ab < bb) {
          const uint64_t t = ab;
          ab = bb;
          bb = t;
          int64_t q = f0;
          f0 = f1;
          f1 = q;
          q = g0;
          g0 = g1;
          g1 = q;
        }
        ab = (ab - bb) >> 1;
        f0 -= f1;
        g0 -= g1;
      } else {
        ab >>= 1;
      }
      f1 *= 2;
      g1 *= 2;
    }
    uint32_t na[N + 1], nbw[N + 1];
    words_lincomb_shr31<N>(a, f0, b, g0, na);
    words_lincomb_shr31<N>(a, f1, b, g1, nbw);
    if (words_neg_if<N + 1>(na, (int32_t)na[N] < 0)) {
      f0 = -f0;
      g0 = -g0;
    }
    if (words_neg_if<N + 1>(nbw, (int32_t)nbw[N] < 0)) {
      f1 = -f1;
      g1 = -g1;
    }
#pragma unroll
    for (int i = 0; i <= N; i++) {
      a[i] = na[i];
      b[i] = nbw[i];
    }
    if (LAZY) {
      // (u, v) <- ((u f0 + v g0) / 2^31, (u f1 + v g1) / 2^31), signed and NOT reduced mod m: with
      // |f0| + |g0| <= 2^31 (and the same for f1, g1) each round adds at most m to the bound, so
      // |u|, |v| < 26 m < 2^386 after the 25 rounds of a 381-bit modulus; one reduction at the end
      uint32_t nu0[N + 1], nv0[N + 1];
      words_lin_mont31<N>(u, f0, v, g0, mod, minv, nu0);
      words_lin_mont31<N>(u, f1, v, g1, mod, minv, nv0);
#pragma unroll
      for (int i = 0; i <= N; i++) {
        u[i] = nu0[i];
        v[i] = nv0[i];
      }
      continue;
    }
    // (u, v) <- ((u f0 + v g0) / 2^31, (u f1 + v g1) / 2^31) mod m
    uint32_t nu[2][N + 1];
#pragma unroll
    for (int side = 0; side < 2; side++) {
      const int64_t fu = side ? f1 : f0, fv = side ? g1 : g0;
      uint32_t t[N + 2];
      int64_t c = 0;
#pragma unroll
      for (int i = 0; i < N; i++) {
        const int64_t p1 = (int64_t)u[i] * fu, p2 = (int64_t)v[i] * fv;
        const int64_t sw = (int64_t)(uint32_t)p1 + (int64_t)(uint32_t)p2 + c;
        t[i] = (uint32_t)sw;
        c = (sw >> 32) + (p1 >> 32) + (p2 >> 32);
      }
      t[N] = (uint32_t)c;
      t[N + 1] = (uint32_t)(c >> 32);
      // + q m with q = -t mod^-1 mod 2^31: the sum is divisible by 2^31
      const uint64_t q = (uint64_t)((t[0] * minv) & 0x7fffffffu);
      uint64_t cc = 0;
#pragma unroll
      for (int i = 0; i < N; i++) {
        cc += (uint64_t)t[i] + q * mod[i];
        t[i] = (uint32_t)cc;
        cc >>= 32;
      }
#pragma unroll
      for (int i = N; i < N + 2; i++) {
        cc += (uint64_t)t[i];
        t[i] = (uint32_t)cc;
        cc >>= 32;
      }
      uint32_t w[N + 1];
#pragma unroll
      for (int i = 0; i <= N; i++) w[i] = (t[i] >> 31) | (t[i + 1] << 1);
      // |w| < 3m: bring into [0, m)
      for (int k = 0; k < 3 && (int32_t)w[N] < 0; k++) {
        uint64_t ac = 0;
#pragma unroll
        for (int i = 0; i < N; i++) {
          ac += (uint64_t)w[i] + mod[i];
          w[i] = (uint32_t)ac;
          ac >>= 32;
        }
        w[N] += (uint32_t)ac;
      }
      for (int k = 0; k < 3 && (w[N] != 0 || words_geq<N>(w, mod)); k++) {
        const uint32_t br = words_sub<N>(w, mod);
        w[N] -= br;
      }
#pragma unroll
      for (int i = 0; i <= N; i++) nu[side][i] = w[i];
    }
#pragma unroll
    for (int i = 0; i <= N; i++) {
      u[i] = nu[0][i];
      v[i] = nu[1][i];
    }
  }
  bool one = b[N] == 0 && words_is_one<N>(b);
  if (LAZY && one) {  // v signed, |v| < 26 m: into [0, m)
    while ((int32_t)v[N] < 0) {
      const uint32_t c = words_add<N>(v, mod);
      v[N] += c;
    }
    while (v[N] != 0 || words_geq<N>(v, mod)) {
      const uint32_t br = words_sub<N>(v, mod);
      v[N] -= br;
    }
  }
#pragma unroll
  for (int i = 0; i < N; i++) out[i] = one ? v[i] : 0u;
}

}  // namespace hb
