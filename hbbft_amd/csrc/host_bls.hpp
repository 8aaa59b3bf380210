// Host-side BLS12-381 arithmetic for the parts of the path that stay on the CPU (north star:
// hashing to G2, transcript parsing and secret-key operations stay on the host): hash_g2 /
// hash_g1_g2 (ThresholdSign::set_document, Ciphertext checks), xor_with_hash, Signature::parity,
// the secret scalar multiplications sign_g2 / decrypt_share / encrypt_with_rng, and the point
// encodings.  Fq is 6 x 64-bit limbs in Montgomery form (R = 2^384), as pairing 0.14's Fq, so
// ff 0.4's Fq::rand (limbs read AS the Montgomery representation) is reproduced directly.
//
// Round 5: the product is a fully unrolled "no-carry" CIOS (p's top limb < 2^63 - 1, so the
// running sum never needs a seventh word), exponentiations use a 5-bit sliding window over odd
// powers, and the curve code has mixed (affine + Jacobian) additions and batch normalisation for
// the endomorphism / comb scalar multiplications of host_hash.cpp.
#pragma once
#include <stdint.h>
#include <string.h>

#include <vector>

namespace hh {

typedef unsigned __int128 u128;

struct Fq {
  uint64_t l[6];
};
struct Fq2 {
  Fq c0, c1;
};

constexpr uint64_t P[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                           0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
constexpr uint64_t PINV = 0x89f3fffcfffcfffdull;  // -p^-1 mod 2^64

inline bool geq_p(const uint64_t* a) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] != P[i]) return a[i] > P[i];
  }
  return true;
}
inline void sub_p(uint64_t* a) {
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    const u128 d = (u128)a[i] - P[i] - br;
    a[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
}
// a - p if a >= p (a < 2p): the subtraction is computed unconditionally and kept when it does not borrow
inline void reduce_once(uint64_t* a) {
  uint64_t d[6], br = 0;
  for (int i = 0; i < 6; i++) {
    const u128 x = (u128)a[i] - P[i] - br;
    d[i] = (uint64_t)x;
    br = (uint64_t)(x >> 64) & 1;
  }
  if (!br) memcpy(a, d, sizeof(d));
}
inline Fq fq_add_portable(const Fq& a, const Fq& b) {
  Fq r;
  uint64_t c = 0;
  for (int i = 0; i < 6; i++) {
    const u128 s = (u128)a.l[i] + b.l[i] + c;
    r.l[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  reduce_once(r.l);  // a + b < 2p < 2^384: no carry out
  return r;
}
inline Fq fq_sub_portable(const Fq& a, const Fq& b) {
  Fq r;
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    const u128 d = (u128)a.l[i] - b.l[i] - br;
    r.l[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 6; i++) {
      const u128 s = (u128)r.l[i] + P[i] + c;
      r.l[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  return r;
}
inline bool fq_is_zero(const Fq& a) {
  uint64_t o = 0;
  for (int i = 0; i < 6; i++) o |= a.l[i];
  return o == 0;
}
inline bool fq_eq(const Fq& a, const Fq& b) { return memcmp(a.l, b.l, sizeof(a.l)) == 0; }
inline Fq fq_zero() {
  Fq r;
  memset(r.l, 0, sizeof(r.l));
  return r;
}

#if defined(__x86_64__)
// BMI2 + ADX (every x86-64 server core since Broadwell / Zen 1): the same no-carry CIOS with MULX and
// two independent carry chains (ADCX on CF for the low halves, ADOX on OF for the high halves), the
// seven running words rotating through registers round by round.  Dispatched at run time.
inline const bool g_adx = [] {
  __builtin_cpu_init();
  return __builtin_cpu_supports("bmi2") && __builtin_cpu_supports("adx");
}();
constexpr uint64_t P_PINV[7] = {P[0], P[1], P[2], P[3], P[4], P[5], PINV};
inline void fq_mul_adx(uint64_t* r, const uint64_t* a, const uint64_t* b) {
  uint64_t t0, t1, t2, t3, t4, t5, t6, lo, hi;
  __asm__(
      "xorq %[t0], %[t0]\n\t"
      "xorq %[t1], %[t1]\n\t"
      "xorq %[t2], %[t2]\n\t"
      "xorq %[t3], %[t3]\n\t"
      "xorq %[t4], %[t4]\n\t"
      "xorq %[t5], %[t5]\n\t"
      "xorq %[t6], %[t6]\n\t"
      "movq 0(%[b]), %%rdx\n\t"
      "xorq %[lo], %[lo]\n\t"
      "mulxq 0(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t0]\n\t"
      "adoxq %[hi], %[t1]\n\t"
      "mulxq 8(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t1]\n\t"
      "adoxq %[hi], %[t2]\n\t"
      "mulxq 16(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t2]\n\t"
      "adoxq %[hi], %[t3]\n\t"
      "mulxq 24(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t3]\n\t"
      "adoxq %[hi], %[t4]\n\t"
      "mulxq 32(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t4]\n\t"
      "adoxq %[hi], %[t5]\n\t"
      "mulxq 40(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t5]\n\t"
      "adoxq %[hi], %[t6]\n\t"
      "movq $0, %[lo]\n\t"
      "adcxq %[lo], %[t6]\n\t"
      "movq %[t0], %%rdx\n\t"
      "imulq 48(%[p]), %%rdx\n\t"
      "xorq %[lo], %[lo]\n\t"
      "mulxq 0(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t0]\n\t"
      "adoxq %[hi], %[t1]\n\t"
      "mulxq 8(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t1]\n\t"
      "adoxq %[hi], %[t2]\n\t"
      "mulxq 16(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t2]\n\t"
      "adoxq %[hi], %[t3]\n\t"
      "mulxq 24(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t3]\n\t"
      "adoxq %[hi], %[t4]\n\t"
      "mulxq 32(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t4]\n\t"
      "adoxq %[hi], %[t5]\n\t"
      "mulxq 40(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t5]\n\t"
      "adoxq %[hi], %[t6]\n\t"
      "movq $0, %[lo]\n\t"
      "adcxq %[lo], %[t6]\n\t"
      "movq 8(%[b]), %%rdx\n\t"
      "xorq %[lo], %[lo]\n\t"
      "mulxq 0(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t1]\n\t"
      "adoxq %[hi], %[t2]\n\t"
      "mulxq 8(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t2]\n\t"
      "adoxq %[hi], %[t3]\n\t"
      "mulxq 16(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t3]\n\t"
      "adoxq %[hi], %[t4]\n\t"
      "mulxq 24(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t4]\n\t"
      "adoxq %[hi], %[t5]\n\t"
      "mulxq 32(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t5]\n\t"
      "adoxq %[hi], %[t6]\n\t"
      "mulxq 40(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t6]\n\t"
      "adoxq %[hi], %[t0]\n\t"
      "movq $0, %[lo]\n\t"
      "adcxq %[lo], %[t0]\n\t"
      "movq %[t1], %%rdx\n\t"
      "imulq 48(%[p]), %%rdx\n\t"
      "xorq %[lo], %[lo]\n\t"
      "mulxq 0(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t1]\n\t"
      "adoxq %[hi], %[t2]\n\t"
      "mulxq 8(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t2]\n\t"
      "adoxq %[hi], %[t3]\n\t"
      "mulxq 16(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t3]\n\t"
      "adoxq %[hi], %[t4]\n\t"
      "mulxq 24(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t4]\n\t"
      "adoxq %[hi], %[t5]\n\t"
      "mulxq 32(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t5]\n\t"
      "adoxq %[hi], %[t6]\n\t"
      "mulxq 40(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t6]\n\t"
      "adoxq %[hi], %[t0]\n\t"
      "movq $0, %[lo]\n\t"
      "adcxq %[lo], %[t0]\n\t"
      "movq 16(%[b]), %%rdx\n\t"
      "xorq %[lo], %[lo]\n\t"
      "mulxq 0(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t2]\n\t"
      "adoxq %[hi], %[t3]\n\t"
      "mulxq 8(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t3]\n\t"
      "adoxq %[hi], %[t4]\n\t"
      "mulxq 16(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t4]\n\t"
      "adoxq %[hi], %[t5]\n\t"
      "mulxq 24(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t5]\n\t"
      "adoxq %[hi], %[t6]\n\t"
      "mulxq 32(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t6]\n\t"
      "adoxq %[hi], %[t0]\n\t"
      "mulxq 40(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t0]\n\t"
      "adoxq %[hi], %[t1]\n\t"
      "movq $0, %[lo]\n\t"
      "adcxq %[lo], %[t1]\n\t"
      "movq %[t2], %%rdx\n\t"
      "imulq 48(%[p]), %%rdx\n\t"
      "xorq %[lo], %[lo]\n\t"
      "mulxq 0(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t2]\n\t"
      "adoxq %[hi], %[t3]\n\t"
      "mulxq 8(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t3]\n\t"
      "adoxq %[hi], %[t4]\n\t"
      "mulxq 16(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t4]\n\t"
      "adoxq %[hi], %[t5]\n\t"
      "mulxq 24(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t5]\n\t"
      "adoxq %[hi], %[t6]\n\t"
      "mulxq 32(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t6]\n\t"
      "adoxq %[hi], %[t0]\n\t"
      "mulxq 40(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t0]\n\t"
      "adoxq %[hi], %[t1]\n\t"
      "movq $0, %[lo]\n\t"
      "adcxq %[lo], %[t1]\n\t"
      "movq 24(%[b]), %%rdx\n\t"
      "xorq %[lo], %[lo]\n\t"
      "mulxq 0(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t3]\n\t"
      "adoxq %[hi], %[t4]\n\t"
      "mulxq 8(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t4]\n\t"
      "adoxq %[hi], %[t5]\n\t"
      "mulxq 16(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t5]\n\t"
      "adoxq %[hi], %[t6]\n\t"
      "mulxq 24(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t6]\n\t"
      "adoxq %[hi], %[t0]\n\t"
      "mulxq 32(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t0]\n\t"
      "adoxq %[hi], %[t1]\n\t"
      "mulxq 40(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t1]\n\t"
      "adoxq %[hi], %[t2]\n\t"
      "movq $0, %[lo]\n\t"
      "adcxq %[lo], %[t2]\n\t"
      "movq %[t3], %%rdx\n\t"
      "imulq 48(%[p]), %%rdx\n\t"
      "xorq %[lo], %[lo]\n\t"
      "mulxq 0(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t3]\n\t"
      "adoxq %[hi], %[t4]\n\t"
      "mulxq 8(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t4]\n\t"
      "adoxq %[hi], %[t5]\n\t"
      "mulxq 16(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t5]\n\t"
      "adoxq %[hi], %[t6]\n\t"
      "mulxq 24(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t6]\n\t"
      "adoxq %[hi], %[t0]\n\t"
      "mulxq 32(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t0]\n\t"
      "adoxq %[hi], %[t1]\n\t"
      "mulxq 40(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t1]\n\t"
      "adoxq %[hi], %[t2]\n\t"
      "movq $0, %[lo]\n\t"
      "adcxq %[lo], %[t2]\n\t"
      "movq 32(%[b]), %%rdx\n\t"
      "xorq %[lo], %[lo]\n\t"
      "mulxq 0(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t4]\n\t"
      "adoxq %[hi], %[t5]\n\t"
      "mulxq 8(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t5]\n\t"
      "adoxq %[hi], %[t6]\n\t"
      "mulxq 16(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t6]\n\t"
      "adoxq %[hi], %[t0]\n\t"
      "mulxq 24(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t0]\n\t"
      "adoxq %[hi], %[t1]\n\t"
      "mulxq 32(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t1]\n\t"
      "adoxq %[hi], %[t2]\n\t"
      "mulxq 40(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t2]\n\t"
      "adoxq %[hi], %[t3]\n\t"
      "movq $0, %[lo]\n\t"
      "adcxq %[lo], %[t3]\n\t"
      "movq %[t4], %%rdx\n\t"
      "imulq 48(%[p]), %%rdx\n\t"
      "xorq %[lo], %[lo]\n\t"
      "mulxq 0(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t4]\n\t"
      "adoxq %[hi], %[t5]\n\t"
      "mulxq 8(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t5]\n\t"
      "adoxq %[hi], %[t6]\n\t"
      "mulxq 16(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t6]\n\t"
      "adoxq %[hi], %[t0]\n\t"
      "mulxq 24(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t0]\n\t"
      "adoxq %[hi], %[t1]\n\t"
      "mulxq 32(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t1]\n\t"
      "adoxq %[hi], %[t2]\n\t"
      "mulxq 40(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t2]\n\t"
      "adoxq %[hi], %[t3]\n\t"
      "movq $0, %[lo]\n\t"
      "adcxq %[lo], %[t3]\n\t"
      "movq 40(%[b]), %%rdx\n\t"
      "xorq %[lo], %[lo]\n\t"
      "mulxq 0(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t5]\n\t"
      "adoxq %[hi], %[t6]\n\t"
      "mulxq 8(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t6]\n\t"
      "adoxq %[hi], %[t0]\n\t"
      "mulxq 16(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t0]\n\t"
      "adoxq %[hi], %[t1]\n\t"
      "mulxq 24(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t1]\n\t"
      "adoxq %[hi], %[t2]\n\t"
      "mulxq 32(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t2]\n\t"
      "adoxq %[hi], %[t3]\n\t"
      "mulxq 40(%[a]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t3]\n\t"
      "adoxq %[hi], %[t4]\n\t"
      "movq $0, %[lo]\n\t"
      "adcxq %[lo], %[t4]\n\t"
      "movq %[t5], %%rdx\n\t"
      "imulq 48(%[p]), %%rdx\n\t"
      "xorq %[lo], %[lo]\n\t"
      "mulxq 0(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t5]\n\t"
      "adoxq %[hi], %[t6]\n\t"
      "mulxq 8(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t6]\n\t"
      "adoxq %[hi], %[t0]\n\t"
      "mulxq 16(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t0]\n\t"
      "adoxq %[hi], %[t1]\n\t"
      "mulxq 24(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t1]\n\t"
      "adoxq %[hi], %[t2]\n\t"
      "mulxq 32(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t2]\n\t"
      "adoxq %[hi], %[t3]\n\t"
      "mulxq 40(%[p]), %[lo], %[hi]\n\t"
      "adcxq %[lo], %[t3]\n\t"
      "adoxq %[hi], %[t4]\n\t"
      "movq $0, %[lo]\n\t"
      "adcxq %[lo], %[t4]\n\t"
      : [t0] "=&r"(t0), [t1] "=&r"(t1), [t2] "=&r"(t2), [t3] "=&r"(t3), [t4] "=&r"(t4), [t5] "=&r"(t5),
        [t6] "=&r"(t6), [lo] "=&r"(lo), [hi] "=&r"(hi)
      : [a] "r"(a), [b] "r"(b), [p] "r"(P_PINV), "m"(*(const uint64_t(*)[6])a), "m"(*(const uint64_t(*)[6])b),
        "m"(*(const uint64_t(*)[7])P_PINV)
      : "rdx", "cc");
  // result limb j sits in the register round 6 names t_j: t6, t0, t1, t2, t3, t4
  r[0] = t6;
  r[1] = t0;
  r[2] = t1;
  r[3] = t2;
  r[4] = t3;
  r[5] = t4;
  (void)t5;
  (void)lo;
  (void)hi;
}
#endif

#if defined(__x86_64__)
// a + b mod p (a, b < p): an add/adc chain, a sub/sbb chain of p, and a conditional move of the
// difference when it did not borrow -- no branch (plain x86-64).  The pointers a, b are dead after the
// first chain and hold two of the difference limbs.
inline void fq_add_asm(uint64_t* r, const uint64_t* a, const uint64_t* b) {
  uint64_t r0, r1, r2, r3, r4, r5, s0, s1, s2, s3;
  uint64_t pa = (uint64_t)a, pb = (uint64_t)b;
  __asm__(
      "movq 0(%[a]), %[r0]\n\t"
      "addq 0(%[b]), %[r0]\n\t"
      "movq 8(%[a]), %[r1]\n\t"
      "adcq 8(%[b]), %[r1]\n\t"
      "movq 16(%[a]), %[r2]\n\t"
      "adcq 16(%[b]), %[r2]\n\t"
      "movq 24(%[a]), %[r3]\n\t"
      "adcq 24(%[b]), %[r3]\n\t"
      "movq 32(%[a]), %[r4]\n\t"
      "adcq 32(%[b]), %[r4]\n\t"
      "movq 40(%[a]), %[r5]\n\t"
      "adcq 40(%[b]), %[r5]\n\t"
      "movq %[r0], %[s0]\n\t"
      "subq %[p0], %[s0]\n\t"
      "movq %[r1], %[s1]\n\t"
      "sbbq %[p1], %[s1]\n\t"
      "movq %[r2], %[s2]\n\t"
      "sbbq %[p2], %[s2]\n\t"
      "movq %[r3], %[s3]\n\t"
      "sbbq %[p3], %[s3]\n\t"
      "movq %[r4], %[a]\n\t"
      "sbbq %[p4], %[a]\n\t"
      "movq %[r5], %[b]\n\t"
      "sbbq %[p5], %[b]\n\t"
      "cmovncq %[s0], %[r0]\n\t"
      "cmovncq %[s1], %[r1]\n\t"
      "cmovncq %[s2], %[r2]\n\t"
      "cmovncq %[s3], %[r3]\n\t"
      "cmovncq %[a], %[r4]\n\t"
      "cmovncq %[b], %[r5]\n\t"
      : [r0] "=&r"(r0), [r1] "=&r"(r1), [r2] "=&r"(r2), [r3] "=&r"(r3), [r4] "=&r"(r4), [r5] "=&r"(r5),
        [s0] "=&r"(s0), [s1] "=&r"(s1), [s2] "=&r"(s2), [s3] "=&r"(s3), [a] "+&r"(pa), [b] "+&r"(pb)
      : [p0] "m"(P_PINV[0]), [p1] "m"(P_PINV[1]), [p2] "m"(P_PINV[2]), [p3] "m"(P_PINV[3]), [p4] "m"(P_PINV[4]),
        [p5] "m"(P_PINV[5]), "m"(*(const uint64_t(*)[6])a), "m"(*(const uint64_t(*)[6])b)
      : "cc");
  r[0] = r0;
  r[1] = r1;
  r[2] = r2;
  r[3] = r3;
  r[4] = r4;
  r[5] = r5;
}
#endif

// Montgomery product a b / 2^384 mod p: CIOS without the carry word (p[5] < 2^63 - 1 keeps every
// round's running value below 2p < 2^384), six rounds unrolled.
inline Fq fq_mul_portable(const Fq& a, const Fq& b) {
  const uint64_t a0 = a.l[0], a1 = a.l[1], a2 = a.l[2], a3 = a.l[3], a4 = a.l[4], a5 = a.l[5];
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
#define HH_ROUND(bi)                                                 \
  {                                                                  \
    const uint64_t b_ = (bi);                                        \
    u128 s;                                                          \
    uint64_t A, C, m;                                                \
    s = (u128)a0 * b_ + t0;                                          \
    t0 = (uint64_t)s;                                                \
    A = (uint64_t)(s >> 64);                                         \
    m = t0 * PINV;                                                   \
    s = (u128)m * P[0] + t0;                                         \
    C = (uint64_t)(s >> 64);                                         \
    s = (u128)a1 * b_ + t1 + A;                                      \
    t1 = (uint64_t)s;                                                \
    A = (uint64_t)(s >> 64);                                         \
    s = (u128)m * P[1] + t1 + C;                                     \
    t0 = (uint64_t)s;                                                \
    C = (uint64_t)(s >> 64);                                         \
    s = (u128)a2 * b_ + t2 + A;                                      \
    t2 = (uint64_t)s;                                                \
    A = (uint64_t)(s >> 64);                                         \
    s = (u128)m * P[2] + t2 + C;                                     \
    t1 = (uint64_t)s;                                                \
    C = (uint64_t)(s >> 64);                                         \
    s = (u128)a3 * b_ + t3 + A;                                      \
    t3 = (uint64_t)s;                                                \
    A = (uint64_t)(s >> 64);                                         \
    s = (u128)m * P[3] + t3 + C;                                     \
    t2 = (uint64_t)s;                                                \
    C = (uint64_t)(s >> 64);                                         \
    s = (u128)a4 * b_ + t4 + A;                                      \
    t4 = (uint64_t)s;                                                \
    A = (uint64_t)(s >> 64);                                         \
    s = (u128)m * P[4] + t4 + C;                                     \
    t3 = (uint64_t)s;                                                \
    C = (uint64_t)(s >> 64);                                         \
    s = (u128)a5 * b_ + t5 + A;                                      \
    t5 = (uint64_t)s;                                                \
    A = (uint64_t)(s >> 64);                                         \
    s = (u128)m * P[5] + t5 + C;                                     \
    t4 = (uint64_t)s;                                                \
    C = (uint64_t)(s >> 64);                                         \
    t5 = C + A;                                                      \
  }
  HH_ROUND(b.l[0])
  HH_ROUND(b.l[1])
  HH_ROUND(b.l[2])
  HH_ROUND(b.l[3])
  HH_ROUND(b.l[4])
  HH_ROUND(b.l[5])
#undef HH_ROUND
  Fq r;
  r.l[0] = t0;
  r.l[1] = t1;
  r.l[2] = t2;
  r.l[3] = t3;
  r.l[4] = t4;
  r.l[5] = t5;
  reduce_once(r.l);
  return r;
}
inline Fq fq_add(const Fq& a, const Fq& b) {
#if defined(__x86_64__)
  Fq r;
  fq_add_asm(r.l, a.l, b.l);
  return r;
#else
  return fq_add_portable(a, b);
#endif
}
// a - b = a + (p - b): p - b <= p, so the sum is < 2p and fq_add's single correction applies
inline Fq fq_sub(const Fq& a, const Fq& b) {
#if defined(__x86_64__)
  Fq nb;
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    const u128 d = (u128)P[i] - b.l[i] - br;
    nb.l[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  Fq r;
  fq_add_asm(r.l, a.l, nb.l);
  return r;
#else
  return fq_sub_portable(a, b);
#endif
}
inline Fq fq_dbl(const Fq& a) { return fq_add(a, a); }
inline Fq fq_neg(const Fq& a) { return fq_is_zero(a) ? a : fq_sub(fq_zero(), a); }
inline Fq fq_mul(const Fq& a, const Fq& b) {
#if defined(__x86_64__)
  if (__builtin_expect(g_adx, 1)) {
    Fq r;
    fq_mul_adx(r.l, a.l, b.l);
    reduce_once(r.l);
    return r;
  }
#endif
  return fq_mul_portable(a, b);
}
inline Fq fq_sqr(const Fq& a) { return fq_mul(a, a); }

struct Consts {
  Fq one;     // R mod p
  Fq r2;      // R^2 mod p
  Fq b1;      // 4 (G1 curve constant), Montgomery
  Fq inv2;    // 1/2, Montgomery
  uint64_t pm2[6], pm3d4[6], pm1d2[6];  // p - 2, (p - 3) / 4, (p - 1) / 2
};
const Consts& consts();

inline Fq fq_one() { return consts().one; }
// canonical little-endian 64-bit limbs (< p) <-> Montgomery
inline Fq fq_from_canon(const uint64_t* c) {
  Fq a;
  memcpy(a.l, c, sizeof(a.l));
  return fq_mul(a, consts().r2);
}
inline void fq_to_canon(const Fq& a, uint64_t* c) {
  Fq one = fq_zero();
  one.l[0] = 1;
  const Fq r = fq_mul(a, one);
  memcpy(c, r.l, sizeof(r.l));
}
// canonical big-endian 48 bytes
inline void fq_to_be(const Fq& a, uint8_t* out) {
  uint64_t c[6];
  fq_to_canon(a, c);
  for (int i = 0; i < 48; i++) out[i] = (uint8_t)(c[5 - i / 8] >> (8 * (7 - i % 8)));
}
// ABI little-endian 48 bytes
inline void fq_to_le(const Fq& a, uint8_t* out) {
  uint64_t c[6];
  fq_to_canon(a, c);
  memcpy(out, c, 48);
}
inline bool fq_from_le(const uint8_t* in, Fq& a) {
  uint64_t c[6];
  memcpy(c, in, 48);
  if (geq_p(c)) {
    a = fq_zero();
    return false;
  }
  a = fq_from_canon(c);
  return true;
}
// canonical integer comparison a > b
inline bool fq_gt(const Fq& a, const Fq& b) {
  uint64_t x[6], y[6];
  fq_to_canon(a, x);
  fq_to_canon(b, y);
  for (int i = 5; i >= 0; i--)
    if (x[i] != y[i]) return x[i] > y[i];
  return false;
}
// a^e for a public exponent e (nlimbs little-endian words): 5-bit sliding window over the odd
// powers a, a^3, ..., a^31 (15 products of precomputation, then one product per window)
inline Fq fq_pow(const Fq& a, const uint64_t* e, int nlimbs) {
  Fq odd[16];
  odd[0] = a;
  const Fq a2 = fq_sqr(a);
  for (int i = 1; i < 16; i++) odd[i] = fq_mul(odd[i - 1], a2);
  auto bit = [&](int i) { return (int)((e[i >> 6] >> (i & 63)) & 1); };
  int i = nlimbs * 64 - 1;
  while (i >= 0 && !bit(i)) i--;
  if (i < 0) return fq_one();
  Fq r = fq_one();
  bool started = false;
  while (i >= 0) {
    if (!bit(i)) {
      r = fq_sqr(r);
      i--;
      continue;
    }
    int j = i - 4 < 0 ? 0 : i - 4;
    while (!bit(j)) j++;
    int val = 0;
    for (int k = i; k >= j; k--) val = (val << 1) | bit(k);
    if (started) {
      for (int k = i; k >= j; k--) r = fq_sqr(r);
      r = fq_mul(r, odd[val >> 1]);
    } else {
      r = odd[val >> 1];
      started = true;
    }
    i = j - 1;
  }
  return r;
}
inline Fq fq_inv(const Fq& a) { return fq_pow(a, consts().pm2, 6); }

// ---------------------------------------------------------------- Fq2 = Fq[u]/(u^2 + 1)
inline Fq2 f2_add(const Fq2& a, const Fq2& b) { return {fq_add(a.c0, b.c0), fq_add(a.c1, b.c1)}; }
inline Fq2 f2_sub(const Fq2& a, const Fq2& b) { return {fq_sub(a.c0, b.c0), fq_sub(a.c1, b.c1)}; }
inline Fq2 f2_neg(const Fq2& a) { return {fq_neg(a.c0), fq_neg(a.c1)}; }
inline Fq2 f2_conj(const Fq2& a) { return {a.c0, fq_neg(a.c1)}; }
inline Fq2 f2_mul(const Fq2& a, const Fq2& b) {
  const Fq t0 = fq_mul(a.c0, b.c0), t1 = fq_mul(a.c1, b.c1);
  const Fq t2 = fq_mul(fq_add(a.c0, a.c1), fq_add(b.c0, b.c1));
  return {fq_sub(t0, t1), fq_sub(fq_sub(t2, t0), t1)};
}
inline Fq2 f2_sqr(const Fq2& a) {
  const Fq s = fq_mul(fq_add(a.c0, a.c1), fq_sub(a.c0, a.c1));
  const Fq m = fq_mul(a.c0, a.c1);
  return {s, fq_add(m, m)};
}
inline Fq2 f2_mul_fq(const Fq2& a, const Fq& s) { return {fq_mul(a.c0, s), fq_mul(a.c1, s)}; }
inline bool f2_is_zero(const Fq2& a) { return fq_is_zero(a.c0) && fq_is_zero(a.c1); }
inline bool f2_eq(const Fq2& a, const Fq2& b) { return fq_eq(a.c0, b.c0) && fq_eq(a.c1, b.c1); }
inline Fq2 f2_zero() { return {fq_zero(), fq_zero()}; }
inline Fq2 f2_one() { return {fq_one(), fq_zero()}; }
inline Fq2 f2_inv(const Fq2& a) {
  const Fq t = fq_inv(fq_add(fq_sqr(a.c0), fq_sqr(a.c1)));
  return {fq_mul(a.c0, t), fq_neg(fq_mul(a.c1, t))};
}
// pairing 0.14 Ord for Fq2: c1 first, then c0 (canonical integers)
inline bool f2_gt(const Fq2& a, const Fq2& b) {
  if (!fq_eq(a.c1, b.c1)) return fq_gt(a.c1, b.c1);
  return fq_gt(a.c0, b.c0);
}
// a square root of a in Fq2, false if a is not a square (host_hash.cpp: the norm method)
bool f2_sqrt(const Fq2& a, Fq2& out);

// ---------------------------------------------------------------- curve points (Jacobian)
template <class F>
struct Ops;
template <>
struct Ops<Fq> {
  static Fq add(const Fq& a, const Fq& b) { return fq_add(a, b); }
  static Fq sub(const Fq& a, const Fq& b) { return fq_sub(a, b); }
  static Fq mul(const Fq& a, const Fq& b) { return fq_mul(a, b); }
  static Fq sqr(const Fq& a) { return fq_sqr(a); }
  static bool zero(const Fq& a) { return fq_is_zero(a); }
  static Fq one() { return fq_one(); }
  static Fq zero_v() { return fq_zero(); }
  static Fq inv(const Fq& a) { return fq_inv(a); }
  static Fq neg(const Fq& a) { return fq_neg(a); }
};
template <>
struct Ops<Fq2> {
  static Fq2 add(const Fq2& a, const Fq2& b) { return f2_add(a, b); }
  static Fq2 sub(const Fq2& a, const Fq2& b) { return f2_sub(a, b); }
  static Fq2 mul(const Fq2& a, const Fq2& b) { return f2_mul(a, b); }
  static Fq2 sqr(const Fq2& a) { return f2_sqr(a); }
  static bool zero(const Fq2& a) { return f2_is_zero(a); }
  static Fq2 one() { return f2_one(); }
  static Fq2 zero_v() { return f2_zero(); }
  static Fq2 inv(const Fq2& a) { return f2_inv(a); }
  static Fq2 neg(const Fq2& a) { return f2_neg(a); }
};

// Jacobian point over F (y^2 = x^3 + b, a = 0); z = 0 is the point at infinity
template <class F>
struct Jac {
  F x, y, z;
};
// affine point; inf marks the point at infinity
template <class F>
struct Aff {
  F x, y;
  bool inf;
};
template <class F>
inline Jac<F> jac_inf() {
  return {Ops<F>::one(), Ops<F>::one(), Ops<F>::zero_v()};
}
template <class F>
inline Jac<F> jac_from_aff(const Aff<F>& a) {
  return a.inf ? jac_inf<F>() : Jac<F>{a.x, a.y, Ops<F>::one()};
}
template <class F>
inline Jac<F> jac_dbl(const Jac<F>& p) {  // dbl-2009-l
  typedef Ops<F> O;
  if (O::zero(p.z)) return p;
  const F A = O::sqr(p.x), B = O::sqr(p.y), C = O::sqr(B);
  F D = O::sub(O::sub(O::sqr(O::add(p.x, B)), A), C);
  D = O::add(D, D);
  const F E = O::add(O::add(A, A), A);
  const F Fv = O::sqr(E);
  Jac<F> r;
  r.x = O::sub(Fv, O::add(D, D));
  F C8 = O::add(C, C);
  C8 = O::add(C8, C8);
  C8 = O::add(C8, C8);
  r.y = O::sub(O::mul(E, O::sub(D, r.x)), C8);
  const F yz = O::mul(p.y, p.z);
  r.z = O::add(yz, yz);
  return r;
}
template <class F>
inline Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) {  // add-2007-bl
  typedef Ops<F> O;
  if (O::zero(p.z)) return q;
  if (O::zero(q.z)) return p;
  const F Z1Z1 = O::sqr(p.z), Z2Z2 = O::sqr(q.z);
  const F U1 = O::mul(p.x, Z2Z2), U2 = O::mul(q.x, Z1Z1);
  const F S1 = O::mul(O::mul(p.y, q.z), Z2Z2), S2 = O::mul(O::mul(q.y, p.z), Z1Z1);
  const F H = O::sub(U2, U1);
  F rr = O::sub(S2, S1);
  if (O::zero(H)) {
    if (O::zero(rr)) return jac_dbl(p);
    return jac_inf<F>();
  }
  const F H2 = O::add(H, H);
  const F I = O::sqr(H2);
  const F J = O::mul(H, I);
  rr = O::add(rr, rr);
  const F V = O::mul(U1, I);
  Jac<F> r;
  r.x = O::sub(O::sub(O::sqr(rr), J), O::add(V, V));
  const F S1J = O::mul(S1, J);
  r.y = O::sub(O::mul(rr, O::sub(V, r.x)), O::add(S1J, S1J));
  r.z = O::mul(O::sub(O::sub(O::sqr(O::add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return r;
}
// p + (qx, qy) for an affine q (madd-2007-bl)
template <class F>
inline Jac<F> jac_add_aff(const Jac<F>& p, const F& qx, const F& qy) {
  typedef Ops<F> O;
  if (O::zero(p.z)) return Jac<F>{qx, qy, O::one()};
  const F Z1Z1 = O::sqr(p.z);
  const F U2 = O::mul(qx, Z1Z1);
  const F S2 = O::mul(O::mul(qy, p.z), Z1Z1);
  const F H = O::sub(U2, p.x);
  F rr = O::sub(S2, p.y);
  if (O::zero(H)) {
    if (O::zero(rr)) return jac_dbl(Jac<F>{qx, qy, O::one()});
    return jac_inf<F>();
  }
  const F HH = O::sqr(H);
  F I = O::add(HH, HH);
  I = O::add(I, I);
  const F J = O::mul(H, I);
  rr = O::add(rr, rr);
  const F V = O::mul(p.x, I);
  Jac<F> r;
  r.x = O::sub(O::sub(O::sqr(rr), J), O::add(V, V));
  const F YJ = O::mul(p.y, J);
  r.y = O::sub(O::mul(rr, O::sub(V, r.x)), O::add(YJ, YJ));
  r.z = O::sub(O::sub(O::sqr(O::add(p.z, H)), Z1Z1), HH);
  return r;
}
template <class F>
inline Jac<F> jac_neg(const Jac<F>& p) {
  Jac<F> r = p;
  r.y = Ops<F>::neg(p.y);
  return r;
}
// affine (x, y); false for the point at infinity
template <class F>
inline bool jac_affine(const Jac<F>& p, F& x, F& y) {
  typedef Ops<F> O;
  if (O::zero(p.z)) return false;
  const F zi = O::inv(p.z), zi2 = O::sqr(zi);
  x = O::mul(p.x, zi2);
  y = O::mul(p.y, O::mul(zi2, zi));
  return true;
}
// affine forms of n points with one inversion (Montgomery's trick); points at infinity allowed
template <class F>
inline void jac_batch_affine(const Jac<F>* p, Aff<F>* out, size_t n) {
  typedef Ops<F> O;
  std::vector<F> pre(n);
  F acc = O::one();
  for (size_t i = 0; i < n; i++) {
    pre[i] = acc;
    if (!O::zero(p[i].z)) acc = O::mul(acc, p[i].z);
  }
  F inv = O::inv(acc);
  for (size_t i = n; i-- > 0;) {
    if (O::zero(p[i].z)) {
      out[i].inf = true;
      out[i].x = O::zero_v();
      out[i].y = O::zero_v();
      continue;
    }
    const F zi = O::mul(inv, pre[i]);
    inv = O::mul(inv, p[i].z);
    const F zi2 = O::sqr(zi);
    out[i].x = O::mul(p[i].x, zi2);
    out[i].y = O::mul(p[i].y, O::mul(zi2, zi));
    out[i].inf = false;
  }
}

// ---------------------------------------------------------------- ABI encodings (include/hbbft_hip.h)
// G1 = x || y (48-byte LE canonical each), G2 = x.c0 || x.c1 || y.c0 || y.c1; infinity = all zero
void g1_to_abi(const Jac<Fq>& p, uint8_t* out);
void g2_to_abi(const Jac<Fq2>& p, uint8_t* out);
void g1_aff_to_abi(const Aff<Fq>& p, uint8_t* out);
void g2_aff_to_abi(const Aff<Fq2>& p, uint8_t* out);
bool g1_from_abi(const uint8_t* in, Jac<Fq>& p);  // false: a coordinate >= p
bool g2_from_abi(const uint8_t* in, Jac<Fq2>& p);

}  // namespace hh
