/* bls_cpu.c -- ORACLE / CPU BASELINE.  TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's CPU path for hbbft's threshold-crypto hot path:
 * threshold_crypto 0.3 -> pairing 0.14 -> ff 0.4 (not vendored in /root/reference, SURVEY.md §8c;
 * restated from the crates' published algorithms).  It keeps the reference's
 * data representation and algorithms so that its timing stands in for the reference (which cannot
 * be built here: no Rust toolchain, crates absent):
 *   - Fq: 6 x u64 Montgomery (R = 2^384), schoolbook product + Montgomery reduction with u128
 *     (ff 0.4 derive: mul_assign / square / mont_reduce); inverse by binary extended Euclid
 *     (ff's Algorithm 16 of Guajardo-Kumar-Paar-Pelzl).
 *   - Fq2/Fq6/Fq12 tower with the pairing-0.14 formulas (Karatsuba mul, complex square,
 *     CH-SQR2 Fq6 square, mul_by_014 / mul_by_01 / mul_by_1, Frobenius tables).
 *   - G2Prepared: homogeneous-projective doubling/addition steps (Algorithms 26/27 of
 *     eprint 2010/354) over the bits of |x| >> 1, one ell() per pair per step, Fq12 square per bit.
 *   - final exponentiation: easy part + the Fuentes-Castaneda et al. hard-part chain with
 *     exp_by_x = Fq12::pow (full squarings) + conjugate.
 *   - PublicKey::verify_g2 = pairing(pk, H) == pairing(g1, sig): two separate pairings
 *     (threshold_crypto; call site src/threshold_sign.rs:223,264).
 *   - verify_decryption_share = pairing(D, hash_g1_g2(U,V)) == pairing(pk, W)
 *     (src/threshold_decrypt.rs:227); Ciphertext::verify (src/threshold_decrypt.rs:142).
 *   - scalar multiplication = double-and-add over the 256 scalar bits (pairing 0.14 mul);
 *     interpolate() = threshold_crypto's Lagrange-at-0 with one Fr inversion per sample,
 *     Sum sample_k * l_k (src/threshold_sign.rs:249-259, src/threshold_decrypt.rs:242-250);
 *   - BivarCommitment::evaluate = Sum_{i,j} C_ij * x^i * y^j with two scalar mults per term
 *     (src/sync_key_gen.rs:542), BivarCommitment::row (src/sync_key_gen.rs:496).
 * Only tests/ and bench.py's cpu_baseline leg load this library.
 *
 * Boundary format (same as include/hbbft_hip.h): affine points as canonical little-endian 48-byte
 * integers, G1 = x||y (96 B), G2 = x.c0||x.c1||y.c0||y.c1 (192 B), infinity = all-zero bytes;
 * Fr scalars 32-byte little-endian.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "bls_consts.h"

typedef unsigned __int128 u128;
typedef struct { uint64_t l[6]; } fq;
typedef struct { fq c0, c1; } fq2;
typedef struct { fq2 c0, c1, c2; } fq6;
typedef struct { fq6 c0, c1; } fq12;
typedef struct { fq x, y, z; } g1p;  /* Jacobian */
typedef struct { fq2 x, y, z; } g2p;
typedef struct { fq x, y; int inf; } g1a;
typedef struct { fq2 x, y; int inf; } g2a;

/* ------------------------------------------------------------------ Fq (ff 0.4 semantics) */
static inline int fq_geq_p(const uint64_t* a) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] > FQ_P[i]) return 1;
    if (a[i] < FQ_P[i]) return 0;
  }
  return 1;
}
static inline void sub_p(uint64_t* a) {
  u128 br = 0;
  for (int i = 0; i < 6; i++) {
    u128 t = (u128)a[i] - FQ_P[i] - br;
    a[i] = (uint64_t)t;
    br = (t >> 64) & 1;
  }
}
static inline void fq_add(fq* r, const fq* a, const fq* b) {
  uint64_t c = 0;
  for (int i = 0; i < 6; i++) {
    u128 t = (u128)a->l[i] + b->l[i] + c;
    r->l[i] = (uint64_t)t;
    c = (uint64_t)(t >> 64);
  }
  if (fq_geq_p(r->l)) sub_p(r->l);
}
static inline void fq_sub(fq* r, const fq* a, const fq* b) {
  u128 br = 0;
  uint64_t t[6];
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a->l[i] - b->l[i] - br;
    t[i] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 6; i++) {
      u128 s = (u128)t[i] + FQ_P[i] + c;
      t[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  memcpy(r->l, t, sizeof t);
}
static inline void fq_dbl(fq* r, const fq* a) { fq_add(r, a, a); }
static inline int fq_is_zero(const fq* a) {
  uint64_t o = 0;
  for (int i = 0; i < 6; i++) o |= a->l[i];
  return o == 0;
}
static inline void fq_neg(fq* r, const fq* a) {
  if (fq_is_zero(a)) { *r = *a; return; }
  fq p;
  memcpy(p.l, FQ_P, sizeof p.l);
  fq_sub(r, &p, a);
}
static inline int fq_eq(const fq* a, const fq* b) { return memcmp(a->l, b->l, 48) == 0; }

static inline void mont_reduce(fq* r, uint64_t t[12]) {
  uint64_t carry2 = 0;
  for (int i = 0; i < 6; i++) {
    uint64_t k = t[i] * FQ_INV;
    uint64_t c = 0;
    for (int j = 0; j < 6; j++) {
      u128 s = (u128)k * FQ_P[j] + t[i + j] + c;
      t[i + j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[i + 6] + c + carry2;
    t[i + 6] = (uint64_t)s;
    carry2 = (uint64_t)(s >> 64);
  }
  memcpy(r->l, t + 6, 48);
  if (fq_geq_p(r->l)) sub_p(r->l);
}
static inline void fq_mul(fq* r, const fq* a, const fq* b) {
  uint64_t t[12] = {0};
  for (int i = 0; i < 6; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 6; j++) {
      u128 s = (u128)a->l[i] * b->l[j] + t[i + j] + c;
      t[i + j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    t[i + 6] = c;
  }
  mont_reduce(r, t);
}
static inline void fq_sqr(fq* r, const fq* a) {
  uint64_t t[12] = {0};
  for (int i = 0; i < 5; i++) {
    uint64_t c = 0;
    for (int j = i + 1; j < 6; j++) {
      u128 s = (u128)a->l[i] * a->l[j] + t[i + j] + c;
      t[i + j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    t[i + 6] = c;
  }
  t[11] = t[10] >> 63;
  for (int i = 10; i > 0; i--) t[i] = (t[i] << 1) | (t[i - 1] >> 63);
  t[0] <<= 1;
  uint64_t c = 0;
  for (int i = 0; i < 6; i++) {
    u128 s = (u128)a->l[i] * a->l[i] + t[2 * i] + c;
    t[2 * i] = (uint64_t)s;
    s = (u128)t[2 * i + 1] + (uint64_t)(s >> 64);
    t[2 * i + 1] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  mont_reduce(r, t);
}
static void fq_from_canon(fq* r, const uint8_t* le48) {
  fq a, r2;
  memcpy(a.l, le48, 48);
  memcpy(r2.l, FQ_R2, 48);
  fq_mul(r, &a, &r2);
}
static void fq_to_canon(uint8_t* le48, const fq* a) {
  uint64_t t[12] = {0};
  memcpy(t, a->l, 48);
  fq r;
  mont_reduce(&r, t);
  memcpy(le48, r.l, 48);
}
static void fq_one(fq* r) { memcpy(r->l, FQ_R, 48); }
static void fq_zero(fq* r) { memset(r->l, 0, 48); }

/* binary inversion (ff 0.4 Fq::inverse); input non-zero Montgomery form */
static inline int repr_is_one(const uint64_t* a) {
  if (a[0] != 1) return 0;
  for (int i = 1; i < 6; i++) if (a[i]) return 0;
  return 1;
}
static inline void repr_div2(uint64_t* a) {
  for (int i = 0; i < 5; i++) a[i] = (a[i] >> 1) | (a[i + 1] << 63);
  a[5] >>= 1;
}
static inline void repr_add_nocarry(uint64_t* a, const uint64_t* b) {
  uint64_t c = 0;
  for (int i = 0; i < 6; i++) {
    u128 s = (u128)a[i] + b[i] + c;
    a[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
}
static inline int repr_lt(const uint64_t* a, const uint64_t* b) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] < b[i]) return 1;
    if (a[i] > b[i]) return 0;
  }
  return 0;
}
static inline void repr_sub_noborrow(uint64_t* a, const uint64_t* b) {
  u128 br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a[i] - b[i] - br;
    a[i] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
}
static int fq_inv(fq* r, const fq* a) {
  if (fq_is_zero(a)) return 0;
  uint64_t u[6], v[6];
  fq b, c;
  memcpy(u, a->l, 48);
  memcpy(v, FQ_P, 48);
  memcpy(b.l, FQ_R2, 48);
  fq_zero(&c);
  while (!repr_is_one(u) && !repr_is_one(v)) {
    while (!(u[0] & 1)) {
      repr_div2(u);
      if (!(b.l[0] & 1)) repr_div2(b.l);
      else { repr_add_nocarry(b.l, FQ_P); repr_div2(b.l); }
    }
    while (!(v[0] & 1)) {
      repr_div2(v);
      if (!(c.l[0] & 1)) repr_div2(c.l);
      else { repr_add_nocarry(c.l, FQ_P); repr_div2(c.l); }
    }
    if (repr_lt(v, u)) { repr_sub_noborrow(u, v); fq_sub(&b, &b, &c); }
    else { repr_sub_noborrow(v, u); fq_sub(&c, &c, &b); }
  }
  *r = repr_is_one(u) ? b : c;
  return 1;
}

/* ------------------------------------------------------------------ Fq2 */
static inline void fq2_add(fq2* r, const fq2* a, const fq2* b) { fq_add(&r->c0, &a->c0, &b->c0); fq_add(&r->c1, &a->c1, &b->c1); }
static inline void fq2_sub(fq2* r, const fq2* a, const fq2* b) { fq_sub(&r->c0, &a->c0, &b->c0); fq_sub(&r->c1, &a->c1, &b->c1); }
static inline void fq2_dbl(fq2* r, const fq2* a) { fq2_add(r, a, a); }
static inline void fq2_neg(fq2* r, const fq2* a) { fq_neg(&r->c0, &a->c0); fq_neg(&r->c1, &a->c1); }
static inline void fq2_conj(fq2* r, const fq2* a) { r->c0 = a->c0; fq_neg(&r->c1, &a->c1); }
static inline int fq2_is_zero(const fq2* a) { return fq_is_zero(&a->c0) && fq_is_zero(&a->c1); }
static inline int fq2_eq(const fq2* a, const fq2* b) { return fq_eq(&a->c0, &b->c0) && fq_eq(&a->c1, &b->c1); }
static inline void fq2_mul(fq2* r, const fq2* a, const fq2* b) {
  fq aa, bb, o, s;
  fq_mul(&aa, &a->c0, &b->c0);
  fq_mul(&bb, &a->c1, &b->c1);
  fq_add(&o, &b->c0, &b->c1);
  fq_add(&s, &a->c1, &a->c0);
  fq_mul(&s, &s, &o);
  fq_sub(&s, &s, &aa);
  fq_sub(&r->c1, &s, &bb);
  fq_sub(&r->c0, &aa, &bb);
}
static inline void fq2_sqr(fq2* r, const fq2* a) {
  fq ab, c0c1, c0;
  fq_mul(&ab, &a->c0, &a->c1);
  fq_add(&c0c1, &a->c0, &a->c1);
  fq_neg(&c0, &a->c1);
  fq_add(&c0, &c0, &a->c0);
  fq_mul(&c0, &c0, &c0c1);
  fq_dbl(&r->c1, &ab);
  r->c0 = c0;
}
static inline void fq2_mul_fq(fq2* r, const fq2* a, const fq* s) { fq_mul(&r->c0, &a->c0, s); fq_mul(&r->c1, &a->c1, s); }
static inline void fq2_mul_nr(fq2* r, const fq2* a) { /* * (u + 1) */
  fq t0 = a->c0;
  fq_sub(&r->c0, &a->c0, &a->c1);
  fq_add(&r->c1, &a->c1, &t0);
}
static inline void fq2_frob(fq2* r, const fq2* a, int power) {
  r->c0 = a->c0;
  fq c;
  memcpy(c.l, FROB_FQ2_C1[power % 2], 48);
  fq_mul(&r->c1, &a->c1, &c);
}
static int fq2_inv(fq2* r, const fq2* a) {
  fq t0, t1;
  fq_sqr(&t0, &a->c0);
  fq_sqr(&t1, &a->c1);
  fq_add(&t0, &t0, &t1);
  if (!fq_inv(&t0, &t0)) return 0;
  fq_mul(&r->c0, &a->c0, &t0);
  fq_mul(&t1, &a->c1, &t0);
  fq_neg(&r->c1, &t1);
  return 1;
}
static void fq2_one(fq2* r) { fq_one(&r->c0); fq_zero(&r->c1); }
static void fq2_zero(fq2* r) { fq_zero(&r->c0); fq_zero(&r->c1); }
static inline void fq2_load(fq2* r, const uint64_t c[2][6]) { memcpy(r->c0.l, c[0], 48); memcpy(r->c1.l, c[1], 48); }

/* ------------------------------------------------------------------ Fq6 */
static inline void fq6_add(fq6* r, const fq6* a, const fq6* b) { fq2_add(&r->c0, &a->c0, &b->c0); fq2_add(&r->c1, &a->c1, &b->c1); fq2_add(&r->c2, &a->c2, &b->c2); }
static inline void fq6_sub(fq6* r, const fq6* a, const fq6* b) { fq2_sub(&r->c0, &a->c0, &b->c0); fq2_sub(&r->c1, &a->c1, &b->c1); fq2_sub(&r->c2, &a->c2, &b->c2); }
static inline void fq6_neg(fq6* r, const fq6* a) { fq2_neg(&r->c0, &a->c0); fq2_neg(&r->c1, &a->c1); fq2_neg(&r->c2, &a->c2); }
static inline void fq6_mul_nr(fq6* r, const fq6* a) {
  fq2 t = a->c2;
  r->c2 = a->c1;
  r->c1 = a->c0;
  fq2_mul_nr(&r->c0, &t);
}
static void fq6_mul(fq6* r, const fq6* a, const fq6* b) {
  fq2 a_a, b_b, c_c, t1, t2, t3, tmp;
  fq2_mul(&a_a, &a->c0, &b->c0);
  fq2_mul(&b_b, &a->c1, &b->c1);
  fq2_mul(&c_c, &a->c2, &b->c2);
  fq2_add(&t1, &b->c1, &b->c2);
  fq2_add(&tmp, &a->c1, &a->c2);
  fq2_mul(&t1, &t1, &tmp);
  fq2_sub(&t1, &t1, &b_b);
  fq2_sub(&t1, &t1, &c_c);
  fq2_mul_nr(&t1, &t1);
  fq2_add(&t1, &t1, &a_a);
  fq2_add(&t3, &b->c0, &b->c2);
  fq2_add(&tmp, &a->c0, &a->c2);
  fq2_mul(&t3, &t3, &tmp);
  fq2_sub(&t3, &t3, &a_a);
  fq2_add(&t3, &t3, &b_b);
  fq2_sub(&t3, &t3, &c_c);
  fq2_add(&t2, &b->c0, &b->c1);
  fq2_add(&tmp, &a->c0, &a->c1);
  fq2_mul(&t2, &t2, &tmp);
  fq2_sub(&t2, &t2, &a_a);
  fq2_sub(&t2, &t2, &b_b);
  fq2_mul_nr(&tmp, &c_c);
  fq2_add(&t2, &t2, &tmp);
  r->c0 = t1;
  r->c1 = t2;
  r->c2 = t3;
}
static void fq6_sqr(fq6* r, const fq6* a) {
  fq2 s0, ab, s1, s2, bc, s3, s4, t;
  fq2_sqr(&s0, &a->c0);
  fq2_mul(&ab, &a->c0, &a->c1);
  fq2_dbl(&s1, &ab);
  fq2_sub(&s2, &a->c0, &a->c1);
  fq2_add(&s2, &s2, &a->c2);
  fq2_sqr(&s2, &s2);
  fq2_mul(&bc, &a->c1, &a->c2);
  fq2_dbl(&s3, &bc);
  fq2_sqr(&s4, &a->c2);
  fq2_mul_nr(&t, &s3);
  fq2_add(&r->c0, &t, &s0);
  fq2_mul_nr(&t, &s4);
  fq2 c1;
  fq2_add(&c1, &t, &s1);
  fq2 c2;
  fq2_add(&c2, &s1, &s2);
  fq2_add(&c2, &c2, &s3);
  fq2_sub(&c2, &c2, &s0);
  fq2_sub(&c2, &c2, &s4);
  r->c1 = c1;
  r->c2 = c2;
}
static void fq6_mul_by_1(fq6* r, const fq6* a, const fq2* c1) {
  fq2 b_b, t1, t2;
  fq2_mul(&b_b, &a->c1, c1);
  fq2_add(&t1, &a->c1, &a->c2);
  fq2_mul(&t1, &t1, c1);
  fq2_sub(&t1, &t1, &b_b);
  fq2_mul_nr(&t1, &t1);
  fq2_add(&t2, &a->c0, &a->c1);
  fq2_mul(&t2, &t2, c1);
  fq2_sub(&t2, &t2, &b_b);
  r->c0 = t1;
  r->c1 = t2;
  r->c2 = b_b;
}
static void fq6_mul_by_01(fq6* r, const fq6* a, const fq2* c0, const fq2* c1) {
  fq2 a_a, b_b, t1, t2, t3, tmp;
  fq2_mul(&a_a, &a->c0, c0);
  fq2_mul(&b_b, &a->c1, c1);
  fq2_add(&t1, &a->c1, &a->c2);
  fq2_mul(&t1, &t1, c1);
  fq2_sub(&t1, &t1, &b_b);
  fq2_mul_nr(&t1, &t1);
  fq2_add(&t1, &t1, &a_a);
  fq2_add(&t3, &a->c0, &a->c2);
  fq2_mul(&t3, &t3, c0);
  fq2_sub(&t3, &t3, &a_a);
  fq2_add(&t3, &t3, &b_b);
  fq2_add(&t2, c0, c1);
  fq2_add(&tmp, &a->c0, &a->c1);
  fq2_mul(&t2, &t2, &tmp);
  fq2_sub(&t2, &t2, &a_a);
  fq2_sub(&t2, &t2, &b_b);
  r->c0 = t1;
  r->c1 = t2;
  r->c2 = t3;
}
static void fq6_frob(fq6* r, const fq6* a, int power) {
  fq2 c;
  fq2_frob(&r->c0, &a->c0, power);
  fq2_frob(&r->c1, &a->c1, power);
  fq2_frob(&r->c2, &a->c2, power);
  fq2_load(&c, FROB_FQ6_C1[power % 6]);
  fq2_mul(&r->c1, &r->c1, &c);
  fq2_load(&c, FROB_FQ6_C2[power % 6]);
  fq2_mul(&r->c2, &r->c2, &c);
}
static int fq6_inv(fq6* r, const fq6* a) {
  fq2 c0, c1, c2, t, tmp;
  fq2_mul_nr(&c0, &a->c2);
  fq2_mul(&c0, &c0, &a->c1);
  fq2_neg(&c0, &c0);
  fq2_sqr(&tmp, &a->c0);
  fq2_add(&c0, &c0, &tmp);
  fq2_sqr(&c1, &a->c2);
  fq2_mul_nr(&c1, &c1);
  fq2_mul(&tmp, &a->c0, &a->c1);
  fq2_sub(&c1, &c1, &tmp);
  fq2_sqr(&c2, &a->c1);
  fq2_mul(&tmp, &a->c0, &a->c2);
  fq2_sub(&c2, &c2, &tmp);
  fq2_mul(&t, &a->c2, &c1);
  fq2_mul(&tmp, &a->c1, &c2);
  fq2_add(&t, &t, &tmp);
  fq2_mul_nr(&t, &t);
  fq2_mul(&tmp, &a->c0, &c0);
  fq2_add(&t, &t, &tmp);
  if (!fq2_inv(&t, &t)) return 0;
  fq2_mul(&r->c0, &c0, &t);
  fq2_mul(&r->c1, &c1, &t);
  fq2_mul(&r->c2, &c2, &t);
  return 1;
}

/* ------------------------------------------------------------------ Fq12 */
static void fq12_one(fq12* r) {
  memset(r, 0, sizeof *r);
  fq_one(&r->c0.c0.c0);
}
__attribute__((unused)) static int fq12_is_one(const fq12* a) {
  fq12 one;
  fq12_one(&one);
  return memcmp(a, &one, sizeof one) == 0;
}
static int fq12_eq(const fq12* a, const fq12* b) { return memcmp(a, b, sizeof *a) == 0; }
static inline void fq12_conj(fq12* a) { fq6_neg(&a->c1, &a->c1); }
static void fq12_mul(fq12* r, const fq12* a, const fq12* b) {
  fq6 aa, bb, o, c1;
  fq6_mul(&aa, &a->c0, &b->c0);
  fq6_mul(&bb, &a->c1, &b->c1);
  fq6_add(&o, &b->c0, &b->c1);
  fq6_add(&c1, &a->c1, &a->c0);
  fq6_mul(&c1, &c1, &o);
  fq6_sub(&c1, &c1, &aa);
  fq6_sub(&c1, &c1, &bb);
  fq6_mul_nr(&bb, &bb);
  fq6_add(&r->c0, &bb, &aa);
  r->c1 = c1;
}
static void fq12_sqr(fq12* r, const fq12* a) {
  fq6 ab, c0c1, c0;
  fq6_mul(&ab, &a->c0, &a->c1);
  fq6_add(&c0c1, &a->c0, &a->c1);
  fq6_mul_nr(&c0, &a->c1);
  fq6_add(&c0, &c0, &a->c0);
  fq6_mul(&c0, &c0, &c0c1);
  fq6_sub(&c0, &c0, &ab);
  fq6_add(&r->c1, &ab, &ab);
  fq6_mul_nr(&ab, &ab);
  fq6_sub(&r->c0, &c0, &ab);
}
static void fq12_mul_by_014(fq12* f, const fq2* c0, const fq2* c1, const fq2* c4) {
  fq6 aa, bb, t;
  fq2 o;
  fq6_mul_by_01(&aa, &f->c0, c0, c1);
  fq6_mul_by_1(&bb, &f->c1, c4);
  fq2_add(&o, c1, c4);
  fq6_add(&t, &f->c1, &f->c0);
  fq6_mul_by_01(&t, &t, c0, &o);
  fq6_sub(&t, &t, &aa);
  fq6_sub(&f->c1, &t, &bb);
  fq6_mul_nr(&bb, &bb);
  fq6_add(&f->c0, &bb, &aa);
}
static void fq12_frob(fq12* r, const fq12* a, int power) {
  fq2 c;
  fq6_frob(&r->c0, &a->c0, power);
  fq6_frob(&r->c1, &a->c1, power);
  fq2_load(&c, FROB_FQ12_C1[power % 12]);
  fq2_mul(&r->c1.c0, &r->c1.c0, &c);
  fq2_mul(&r->c1.c1, &r->c1.c1, &c);
  fq2_mul(&r->c1.c2, &r->c1.c2, &c);
}
static int fq12_inv(fq12* r, const fq12* a) {
  fq6 c0s, c1s, t;
  fq6_sqr(&c0s, &a->c0);
  fq6_sqr(&c1s, &a->c1);
  fq6_mul_nr(&c1s, &c1s);
  fq6_sub(&c0s, &c0s, &c1s);
  if (!fq6_inv(&t, &c0s)) return 0;
  fq6 r0, r1;
  fq6_mul(&r0, &a->c0, &t);
  fq6_mul(&r1, &a->c1, &t);
  fq6_neg(&r1, &r1);
  r->c0 = r0;
  r->c1 = r1;
  return 1;
}
/* ff Field::pow over one u64 limb */
static void fq12_pow_u64(fq12* r, const fq12* a, uint64_t e) {
  fq12 res;
  fq12_one(&res);
  int found = 0;
  for (int i = 63; i >= 0; i--) {
    int bit = (e >> i) & 1;
    if (found) fq12_sqr(&res, &res);
    else found = bit;
    if (bit) fq12_mul(&res, &res, a);
  }
  *r = res;
}

/* ------------------------------------------------------------------ pairing (pairing 0.14 Bls12) */
#define BLS_X 0xd201000000010000ULL

typedef struct { fq2 c0, c1, c2; } ell_coeff;
typedef struct { ell_coeff coeffs[70]; int n; int infinity; } g2_prepared;

static void doubling_step(g2p* r, ell_coeff* out) {
  fq2 tmp0, tmp1, tmp2, tmp3, tmp4, tmp5, tmp6, zsq;
  fq2_sqr(&tmp0, &r->x);
  fq2_sqr(&tmp1, &r->y);
  fq2_sqr(&tmp2, &tmp1);
  fq2_add(&tmp3, &tmp1, &r->x);
  fq2_sqr(&tmp3, &tmp3);
  fq2_sub(&tmp3, &tmp3, &tmp0);
  fq2_sub(&tmp3, &tmp3, &tmp2);
  fq2_dbl(&tmp3, &tmp3);
  fq2_dbl(&tmp4, &tmp0);
  fq2_add(&tmp4, &tmp4, &tmp0);
  fq2_add(&tmp6, &r->x, &tmp4);
  fq2_sqr(&tmp5, &tmp4);
  fq2_sqr(&zsq, &r->z);
  fq2_sub(&r->x, &tmp5, &tmp3);
  fq2_sub(&r->x, &r->x, &tmp3);
  fq2_add(&r->z, &r->z, &r->y);
  fq2_sqr(&r->z, &r->z);
  fq2_sub(&r->z, &r->z, &tmp1);
  fq2_sub(&r->z, &r->z, &zsq);
  fq2_sub(&r->y, &tmp3, &r->x);
  fq2_mul(&r->y, &r->y, &tmp4);
  fq2_dbl(&tmp2, &tmp2);
  fq2_dbl(&tmp2, &tmp2);
  fq2_dbl(&tmp2, &tmp2);
  fq2_sub(&r->y, &r->y, &tmp2);
  fq2_mul(&tmp3, &tmp4, &zsq);
  fq2_dbl(&tmp3, &tmp3);
  fq2_neg(&tmp3, &tmp3);
  fq2_sqr(&tmp6, &tmp6);
  fq2_sub(&tmp6, &tmp6, &tmp0);
  fq2_sub(&tmp6, &tmp6, &tmp5);
  fq2_dbl(&tmp1, &tmp1);
  fq2_dbl(&tmp1, &tmp1);
  fq2_sub(&tmp6, &tmp6, &tmp1);
  fq2_mul(&tmp0, &r->z, &zsq);
  fq2_dbl(&tmp0, &tmp0);
  out->c0 = tmp0;
  out->c1 = tmp3;
  out->c2 = tmp6;
}

static void addition_step(g2p* r, const g2a* q, ell_coeff* out) {
  fq2 zsq, ysq, t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, ztsq;
  fq2_sqr(&zsq, &r->z);
  fq2_sqr(&ysq, &q->y);
  fq2_mul(&t0, &zsq, &q->x);
  fq2_add(&t1, &q->y, &r->z);
  fq2_sqr(&t1, &t1);
  fq2_sub(&t1, &t1, &ysq);
  fq2_sub(&t1, &t1, &zsq);
  fq2_mul(&t1, &t1, &zsq);
  fq2_sub(&t2, &t0, &r->x);
  fq2_sqr(&t3, &t2);
  fq2_dbl(&t4, &t3);
  fq2_dbl(&t4, &t4);
  fq2_mul(&t5, &t4, &t2);
  fq2_sub(&t6, &t1, &r->y);
  fq2_sub(&t6, &t6, &r->y);
  fq2_mul(&t9, &t6, &q->x);
  fq2_mul(&t7, &t4, &r->x);
  fq2_sqr(&r->x, &t6);
  fq2_sub(&r->x, &r->x, &t5);
  fq2_sub(&r->x, &r->x, &t7);
  fq2_sub(&r->x, &r->x, &t7);
  fq2_add(&r->z, &r->z, &t2);
  fq2_sqr(&r->z, &r->z);
  fq2_sub(&r->z, &r->z, &zsq);
  fq2_sub(&r->z, &r->z, &t3);
  fq2_add(&t10, &q->y, &r->z);
  fq2_sub(&t8, &t7, &r->x);
  fq2_mul(&t8, &t8, &t6);
  fq2_mul(&t0, &r->y, &t5);
  fq2_dbl(&t0, &t0);
  fq2_sub(&r->y, &t8, &t0);
  fq2_sqr(&t10, &t10);
  fq2_sub(&t10, &t10, &ysq);
  fq2_sqr(&ztsq, &r->z);
  fq2_sub(&t10, &t10, &ztsq);
  fq2_dbl(&t9, &t9);
  fq2_sub(&t9, &t9, &t10);
  fq2_dbl(&t10, &r->z);
  fq2_neg(&t6, &t6);
  fq2_dbl(&t1, &t6);
  out->c0 = t10;
  out->c1 = t1;
  out->c2 = t9;
}

static void g2_prepare(g2_prepared* out, const g2a* q) {
  out->n = 0;
  out->infinity = q->inf;
  if (q->inf) return;
  g2p r;
  r.x = q->x;
  r.y = q->y;
  fq2_one(&r.z);
  uint64_t x = BLS_X >> 1;
  int found = 0;
  for (int i = 63; i >= 0; i--) {
    int bit = (x >> i) & 1;
    if (!found) { found = bit; continue; }
    doubling_step(&r, &out->coeffs[out->n++]);
    if (bit) addition_step(&r, q, &out->coeffs[out->n++]);
  }
  doubling_step(&r, &out->coeffs[out->n++]);
}

static void ell(fq12* f, const ell_coeff* c, const g1a* p) {
  fq2 c0 = c->c0, c1 = c->c1;
  fq_mul(&c0.c0, &c0.c0, &p->y);
  fq_mul(&c0.c1, &c0.c1, &p->y);
  fq_mul(&c1.c0, &c1.c0, &p->x);
  fq_mul(&c1.c1, &c1.c1, &p->x);
  fq12_mul_by_014(f, &c->c2, &c1, &c0);
}

/* pairing 0.14 Bls12::miller_loop over (G1Affine, G2Prepared) pairs */
static void miller_loop(fq12* f, int npairs, const g1a* const* ps, const g2_prepared* const* qs) {
  int idx[4] = {0, 0, 0, 0};
  fq12_one(f);
  uint64_t x = BLS_X >> 1;
  int found = 0;
  for (int i = 63; i >= 0; i--) {
    int bit = (x >> i) & 1;
    if (!found) { found = bit; continue; }
    for (int k = 0; k < npairs; k++)
      if (!ps[k]->inf && !qs[k]->infinity) ell(f, &qs[k]->coeffs[idx[k]++], ps[k]);
    if (bit)
      for (int k = 0; k < npairs; k++)
        if (!ps[k]->inf && !qs[k]->infinity) ell(f, &qs[k]->coeffs[idx[k]++], ps[k]);
    fq12_sqr(f, f);
  }
  for (int k = 0; k < npairs; k++)
    if (!ps[k]->inf && !qs[k]->infinity) ell(f, &qs[k]->coeffs[idx[k]++], ps[k]);
  fq12_conj(f); /* x is negative */
}

static void exp_by_x(fq12* f, uint64_t x) {
  fq12_pow_u64(f, f, x);
  fq12_conj(f);
}

static int final_exponentiation(fq12* out, const fq12* r_in) {
  fq12 f1 = *r_in, f2, r;
  fq12_conj(&f1);
  if (!fq12_inv(&f2, r_in)) return 0;
  fq12_mul(&r, &f1, &f2);
  f2 = r;
  fq12_frob(&r, &r, 2);
  fq12_mul(&r, &r, &f2);
  uint64_t x = BLS_X;
  fq12 y0, y1, y2, y3;
  fq12_sqr(&y0, &r);
  y1 = y0;
  exp_by_x(&y1, x);
  x >>= 1;
  y2 = y1;
  exp_by_x(&y2, x);
  x <<= 1;
  y3 = r;
  fq12_conj(&y3);
  fq12_mul(&y1, &y1, &y3);
  fq12_conj(&y1);
  fq12_mul(&y1, &y1, &y2);
  y2 = y1;
  exp_by_x(&y2, x);
  y3 = y2;
  exp_by_x(&y3, x);
  fq12_conj(&y1);
  fq12_mul(&y3, &y3, &y1);
  fq12_conj(&y1);
  fq12_frob(&y1, &y1, 3);
  fq12_frob(&y2, &y2, 2);
  fq12_mul(&y1, &y1, &y2);
  y2 = y3;
  exp_by_x(&y2, x);
  fq12_mul(&y2, &y2, &y0);
  fq12_mul(&y2, &y2, &r);
  fq12_mul(&y1, &y1, &y2);
  y2 = y3;
  fq12_frob(&y2, &y2, 1);
  fq12_mul(&y1, &y1, &y2);
  *out = y1;
  return 1;
}

/* Engine::pairing(p, q) */
static void pairing(fq12* out, const g1a* p, const g2a* q) {
  g2_prepared qp;
  g2_prepare(&qp, q);
  const g1a* ps[1] = {p};
  const g2_prepared* qs[1] = {&qp};
  fq12 f;
  miller_loop(&f, 1, ps, qs);
  if (!final_exponentiation(out, &f)) fq12_one(out);
}

/* ------------------------------------------------------------------ boundary decoding */
static void g1_load(g1a* p, const uint8_t* b) {
  int z = 1;
  for (int i = 0; i < 96; i++) if (b[i]) { z = 0; break; }
  p->inf = z;
  if (z) { fq_zero(&p->x); fq_zero(&p->y); return; }
  fq_from_canon(&p->x, b);
  fq_from_canon(&p->y, b + 48);
}
static void g2_load(g2a* p, const uint8_t* b) {
  int z = 1;
  for (int i = 0; i < 192; i++) if (b[i]) { z = 0; break; }
  p->inf = z;
  if (z) { memset(p, 0, sizeof *p); p->inf = 1; return; }
  fq_from_canon(&p->x.c0, b);
  fq_from_canon(&p->x.c1, b + 48);
  fq_from_canon(&p->y.c0, b + 96);
  fq_from_canon(&p->y.c1, b + 144);
}
static void g1_generator(g1a* g) {
  memcpy(g->x.l, G1_GEN_X, 48);
  memcpy(g->y.l, G1_GEN_Y, 48);
  g->inf = 0;
}

/* ------------------------------------------------------------------ curve arithmetic (Jacobian) */
static void g1p_zero(g1p* r) { fq_zero(&r->x); fq_one(&r->y); fq_zero(&r->z); }
static int g1p_is_zero(const g1p* a) { return fq_is_zero(&a->z); }
static void g1p_dbl(g1p* r, const g1p* a) { /* dbl-2009-l */
  if (g1p_is_zero(a)) { *r = *a; return; }
  fq A, B, C, D, E, F, t;
  fq_sqr(&A, &a->x);
  fq_sqr(&B, &a->y);
  fq_sqr(&C, &B);
  fq_add(&D, &a->x, &B);
  fq_sqr(&D, &D);
  fq_sub(&D, &D, &A);
  fq_sub(&D, &D, &C);
  fq_dbl(&D, &D);
  fq_dbl(&E, &A);
  fq_add(&E, &E, &A);
  fq_sqr(&F, &E);
  fq z3;
  fq_mul(&z3, &a->z, &a->y);
  fq_dbl(&z3, &z3);
  fq x3;
  fq_dbl(&t, &D);
  fq_sub(&x3, &F, &t);
  fq y3;
  fq_sub(&y3, &D, &x3);
  fq_mul(&y3, &y3, &E);
  fq_dbl(&C, &C);
  fq_dbl(&C, &C);
  fq_dbl(&C, &C);
  fq_sub(&y3, &y3, &C);
  r->x = x3;
  r->y = y3;
  r->z = z3;
}
static void g1p_add_mixed(g1p* r, const g1p* a, const g1a* b) { /* madd-2007-bl */
  if (b->inf) { *r = *a; return; }
  if (g1p_is_zero(a)) { r->x = b->x; r->y = b->y; fq_one(&r->z); return; }
  fq z1z1, u2, s2, h, hh, i, j, rr, v, t;
  fq_sqr(&z1z1, &a->z);
  fq_mul(&u2, &b->x, &z1z1);
  fq_mul(&s2, &b->y, &a->z);
  fq_mul(&s2, &s2, &z1z1);
  if (fq_eq(&a->x, &u2) && fq_eq(&a->y, &s2)) { g1p_dbl(r, a); return; }
  fq_sub(&h, &u2, &a->x);
  fq_sqr(&hh, &h);
  fq_dbl(&i, &hh);
  fq_dbl(&i, &i);
  fq_mul(&j, &h, &i);
  fq_sub(&rr, &s2, &a->y);
  fq_dbl(&rr, &rr);
  fq_mul(&v, &a->x, &i);
  fq x3, y3, z3;
  fq_sqr(&x3, &rr);
  fq_sub(&x3, &x3, &j);
  fq_sub(&x3, &x3, &v);
  fq_sub(&x3, &x3, &v);
  fq_sub(&t, &v, &x3);
  fq_mul(&y3, &rr, &t);
  fq_mul(&t, &a->y, &j);
  fq_dbl(&t, &t);
  fq_sub(&y3, &y3, &t);
  fq_add(&z3, &a->z, &h);
  fq_sqr(&z3, &z3);
  fq_sub(&z3, &z3, &z1z1);
  fq_sub(&z3, &z3, &hh);
  if (fq_is_zero(&h)) { g1p_zero(r); return; } /* a == -b */
  r->x = x3;
  r->y = y3;
  r->z = z3;
}
static void g1p_add(g1p* r, const g1p* a, const g1p* b) { /* add-2007-bl */
  if (g1p_is_zero(a)) { *r = *b; return; }
  if (g1p_is_zero(b)) { *r = *a; return; }
  fq z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
  fq_sqr(&z1z1, &a->z);
  fq_sqr(&z2z2, &b->z);
  fq_mul(&u1, &a->x, &z2z2);
  fq_mul(&u2, &b->x, &z1z1);
  fq_mul(&s1, &a->y, &b->z);
  fq_mul(&s1, &s1, &z2z2);
  fq_mul(&s2, &b->y, &a->z);
  fq_mul(&s2, &s2, &z1z1);
  if (fq_eq(&u1, &u2)) {
    if (fq_eq(&s1, &s2)) { g1p_dbl(r, a); return; }
    g1p_zero(r);
    return;
  }
  fq_sub(&h, &u2, &u1);
  fq_dbl(&i, &h);
  fq_sqr(&i, &i);
  fq_mul(&j, &h, &i);
  fq_sub(&rr, &s2, &s1);
  fq_dbl(&rr, &rr);
  fq_mul(&v, &u1, &i);
  fq x3, y3, z3;
  fq_sqr(&x3, &rr);
  fq_sub(&x3, &x3, &j);
  fq_sub(&x3, &x3, &v);
  fq_sub(&x3, &x3, &v);
  fq_sub(&t, &v, &x3);
  fq_mul(&y3, &rr, &t);
  fq_mul(&t, &s1, &j);
  fq_dbl(&t, &t);
  fq_sub(&y3, &y3, &t);
  fq_add(&z3, &a->z, &b->z);
  fq_sqr(&z3, &z3);
  fq_sub(&z3, &z3, &z1z1);
  fq_sub(&z3, &z3, &z2z2);
  fq_mul(&z3, &z3, &h);
  r->x = x3;
  r->y = y3;
  r->z = z3;
}
static void g1p_to_affine(g1a* r, const g1p* a) {
  if (g1p_is_zero(a)) { memset(r, 0, sizeof *r); r->inf = 1; return; }
  fq zi, zi2;
  fq_inv(&zi, &a->z);
  fq_sqr(&zi2, &zi);
  fq_mul(&r->x, &a->x, &zi2);
  fq_mul(&zi2, &zi2, &zi);
  fq_mul(&r->y, &a->y, &zi2);
  r->inf = 0;
}
/* G1Affine::mul: double-and-add over all bits of the scalar (most significant first) */
static void g1_mul_bits(g1p* r, const g1a* p, const uint64_t* k, int nbits) {
  g1p acc;
  g1p_zero(&acc);
  for (int i = nbits - 1; i >= 0; i--) {
    g1p_dbl(&acc, &acc);
    if ((k[i >> 6] >> (i & 63)) & 1) g1p_add_mixed(&acc, &acc, p);
  }
  *r = acc;
}

static void g2p_zero(g2p* r) { fq2_zero(&r->x); fq2_one(&r->y); fq2_zero(&r->z); }
static int g2p_is_zero(const g2p* a) { return fq2_is_zero(&a->z); }
static void g2p_dbl(g2p* r, const g2p* a) {
  if (g2p_is_zero(a)) { *r = *a; return; }
  fq2 A, B, C, D, E, F, t, x3, y3, z3;
  fq2_sqr(&A, &a->x);
  fq2_sqr(&B, &a->y);
  fq2_sqr(&C, &B);
  fq2_add(&D, &a->x, &B);
  fq2_sqr(&D, &D);
  fq2_sub(&D, &D, &A);
  fq2_sub(&D, &D, &C);
  fq2_dbl(&D, &D);
  fq2_dbl(&E, &A);
  fq2_add(&E, &E, &A);
  fq2_sqr(&F, &E);
  fq2_mul(&z3, &a->z, &a->y);
  fq2_dbl(&z3, &z3);
  fq2_dbl(&t, &D);
  fq2_sub(&x3, &F, &t);
  fq2_sub(&y3, &D, &x3);
  fq2_mul(&y3, &y3, &E);
  fq2_dbl(&C, &C);
  fq2_dbl(&C, &C);
  fq2_dbl(&C, &C);
  fq2_sub(&y3, &y3, &C);
  r->x = x3;
  r->y = y3;
  r->z = z3;
}
static void g2p_add_mixed(g2p* r, const g2p* a, const g2a* b) {
  if (b->inf) { *r = *a; return; }
  if (g2p_is_zero(a)) { r->x = b->x; r->y = b->y; fq2_one(&r->z); return; }
  fq2 z1z1, u2, s2, h, hh, i, j, rr, v, t, x3, y3, z3;
  fq2_sqr(&z1z1, &a->z);
  fq2_mul(&u2, &b->x, &z1z1);
  fq2_mul(&s2, &b->y, &a->z);
  fq2_mul(&s2, &s2, &z1z1);
  if (fq2_eq(&a->x, &u2)) {
    if (fq2_eq(&a->y, &s2)) { g2p_dbl(r, a); return; }
    g2p_zero(r);
    return;
  }
  fq2_sub(&h, &u2, &a->x);
  fq2_sqr(&hh, &h);
  fq2_dbl(&i, &hh);
  fq2_dbl(&i, &i);
  fq2_mul(&j, &h, &i);
  fq2_sub(&rr, &s2, &a->y);
  fq2_dbl(&rr, &rr);
  fq2_mul(&v, &a->x, &i);
  fq2_sqr(&x3, &rr);
  fq2_sub(&x3, &x3, &j);
  fq2_sub(&x3, &x3, &v);
  fq2_sub(&x3, &x3, &v);
  fq2_sub(&t, &v, &x3);
  fq2_mul(&y3, &rr, &t);
  fq2_mul(&t, &a->y, &j);
  fq2_dbl(&t, &t);
  fq2_sub(&y3, &y3, &t);
  fq2_add(&z3, &a->z, &h);
  fq2_sqr(&z3, &z3);
  fq2_sub(&z3, &z3, &z1z1);
  fq2_sub(&z3, &z3, &hh);
  r->x = x3;
  r->y = y3;
  r->z = z3;
}
static void g2p_add(g2p* r, const g2p* a, const g2p* b) {
  if (g2p_is_zero(a)) { *r = *b; return; }
  if (g2p_is_zero(b)) { *r = *a; return; }
  fq2 z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t, x3, y3, z3;
  fq2_sqr(&z1z1, &a->z);
  fq2_sqr(&z2z2, &b->z);
  fq2_mul(&u1, &a->x, &z2z2);
  fq2_mul(&u2, &b->x, &z1z1);
  fq2_mul(&s1, &a->y, &b->z);
  fq2_mul(&s1, &s1, &z2z2);
  fq2_mul(&s2, &b->y, &a->z);
  fq2_mul(&s2, &s2, &z1z1);
  if (fq2_eq(&u1, &u2)) {
    if (fq2_eq(&s1, &s2)) { g2p_dbl(r, a); return; }
    g2p_zero(r);
    return;
  }
  fq2_sub(&h, &u2, &u1);
  fq2_dbl(&i, &h);
  fq2_sqr(&i, &i);
  fq2_mul(&j, &h, &i);
  fq2_sub(&rr, &s2, &s1);
  fq2_dbl(&rr, &rr);
  fq2_mul(&v, &u1, &i);
  fq2_sqr(&x3, &rr);
  fq2_sub(&x3, &x3, &j);
  fq2_sub(&x3, &x3, &v);
  fq2_sub(&x3, &x3, &v);
  fq2_sub(&t, &v, &x3);
  fq2_mul(&y3, &rr, &t);
  fq2_mul(&t, &s1, &j);
  fq2_dbl(&t, &t);
  fq2_sub(&y3, &y3, &t);
  fq2_add(&z3, &a->z, &b->z);
  fq2_sqr(&z3, &z3);
  fq2_sub(&z3, &z3, &z1z1);
  fq2_sub(&z3, &z3, &z2z2);
  fq2_mul(&z3, &z3, &h);
  r->x = x3;
  r->y = y3;
  r->z = z3;
}
static void g2p_to_affine(g2a* r, const g2p* a) {
  if (g2p_is_zero(a)) { memset(r, 0, sizeof *r); r->inf = 1; return; }
  fq2 zi, zi2;
  fq2_inv(&zi, &a->z);
  fq2_sqr(&zi2, &zi);
  fq2_mul(&r->x, &a->x, &zi2);
  fq2_mul(&zi2, &zi2, &zi);
  fq2_mul(&r->y, &a->y, &zi2);
  r->inf = 0;
}
static void g2_mul_bits(g2p* r, const g2a* p, const uint64_t* k, int nbits) {
  g2p acc;
  g2p_zero(&acc);
  for (int i = nbits - 1; i >= 0; i--) {
    g2p_dbl(&acc, &acc);
    if ((k[i >> 6] >> (i & 63)) & 1) g2p_add_mixed(&acc, &acc, p);
  }
  *r = acc;
}

static void g1_store(uint8_t* out, const g1a* a) {
  if (a->inf) { memset(out, 0, 96); return; }
  fq_to_canon(out, &a->x);
  fq_to_canon(out + 48, &a->y);
}
static void g2_store(uint8_t* out, const g2a* a) {
  if (a->inf) { memset(out, 0, 192); return; }
  fq_to_canon(out, &a->x.c0);
  fq_to_canon(out + 48, &a->x.c1);
  fq_to_canon(out + 96, &a->y.c0);
  fq_to_canon(out + 144, &a->y.c1);
}

/* ------------------------------------------------------------------ Fr (scalar field) */
typedef struct { uint64_t l[4]; } fr;  /* Montgomery, R = 2^256 */
static inline int fr_geq(const uint64_t* a) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] > FR_R[i]) return 1;
    if (a[i] < FR_R[i]) return 0;
  }
  return 1;
}
static inline void fr_subr(uint64_t* a) {
  u128 br = 0;
  for (int i = 0; i < 4; i++) {
    u128 t = (u128)a[i] - FR_R[i] - br;
    a[i] = (uint64_t)t;
    br = (t >> 64) & 1;
  }
}
static void fr_mul(fr* r, const fr* a, const fr* b) {
  uint64_t t[9] = {0};
  for (int i = 0; i < 4; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 4; j++) {
      u128 s = (u128)a->l[i] * b->l[j] + t[j] + c;
      t[j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[4] + c;
    t[4] = (uint64_t)s;
    t[5] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * FR_INV;
    s = (u128)m * FR_R[0] + t[0];
    c = (uint64_t)(s >> 64);
    for (int j = 1; j < 4; j++) {
      s = (u128)m * FR_R[j] + t[j] + c;
      t[j - 1] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    s = (u128)t[4] + c;
    t[3] = (uint64_t)s;
    t[4] = t[5] + (uint64_t)(s >> 64);
  }
  uint64_t o[4] = {t[0], t[1], t[2], t[3]};
  if (t[4] || fr_geq(o)) fr_subr(o);
  memcpy(r->l, o, 32);
}
static void fr_sub(fr* r, const fr* a, const fr* b) {
  u128 br = 0;
  uint64_t t[4];
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a->l[i] - b->l[i] - br;
    t[i] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 4; i++) {
      u128 s = (u128)t[i] + FR_R[i] + c;
      t[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  memcpy(r->l, t, 32);
}
static void fr_from_canon(fr* r, const uint64_t* k) {
  fr a, rr;
  memcpy(a.l, k, 32);
  memcpy(rr.l, FR_RR, 32);
  fr_mul(r, &a, &rr);
}
static void fr_to_canon(uint64_t* k, const fr* a) {
  fr one = {{1, 0, 0, 0}};
  fr t;
  fr_mul(&t, a, &one);
  memcpy(k, t.l, 32);
}
static int fr_is_zero(const fr* a) { return !(a->l[0] | a->l[1] | a->l[2] | a->l[3]); }
static void fr_inv(fr* r, const fr* a) { /* a^(r-2) */
  uint64_t e[4];
  memcpy(e, FR_R, 32);
  e[0] -= 2;
  fr res;
  memcpy(res.l, FR_ONE, 32);
  for (int i = 255; i >= 0; i--) {
    fr_mul(&res, &res, &res);
    if ((e[i >> 6] >> (i & 63)) & 1) fr_mul(&res, &res, a);
  }
  *r = res;
}

/* threshold_crypto interpolate(): Lagrange coefficients at 0 for x_k = idx_k + 1, as the crate
 * computes them (prefix/suffix products of the x's, one inversion per sample).  Returns 0 on
 * success, 5 (DuplicateEntry) if a denominator vanishes. */
static int lagrange_at_zero(int m, const uint64_t* idx, fr* lam) {
  fr xs[256];
  for (int k = 0; k < m; k++) {
    uint64_t v[4] = {idx[k] + 1, 0, 0, 0};
    fr_from_canon(&xs[k], v);
  }
  fr xprod[256], tmp;
  memcpy(tmp.l, FR_ONE, 32);
  xprod[0] = tmp;
  for (int k = 0; k < m - 1; k++) { fr_mul(&tmp, &tmp, &xs[k]); xprod[k + 1] = tmp; }
  memcpy(tmp.l, FR_ONE, 32);
  for (int k = m - 2; k >= 0; k--) { fr_mul(&tmp, &tmp, &xs[k + 1]); fr_mul(&xprod[k], &xprod[k], &tmp); }
  for (int k = 0; k < m; k++) {
    fr denom;
    memcpy(denom.l, FR_ONE, 32);
    for (int j = 0; j < m; j++) {
      if (memcmp(&xs[j], &xs[k], sizeof(fr)) == 0) continue;
      fr d;
      fr_sub(&d, &xs[j], &xs[k]);
      fr_mul(&denom, &denom, &d);
    }
    if (fr_is_zero(&denom)) return 5;
    fr inv;
    fr_inv(&inv, &denom);
    fr_mul(&lam[k], &xprod[k], &inv);
  }
  return 0;
}

/* ================================================================== exported API */
#define API __attribute__((visibility("default")))

/* PublicKey(Share)::verify_g2: pairing(pk, H) == pairing(g1, sig) -- two full pairings. */
API int bls_verify_g2(const uint8_t* pk96, const uint8_t* sig192, const uint8_t* h192) {
  g1a pk, g1;
  g2a sig, h;
  g1_load(&pk, pk96);
  g2_load(&sig, sig192);
  g2_load(&h, h192);
  g1_generator(&g1);
  fq12 a, b;
  pairing(&a, &pk, &h);
  pairing(&b, &g1, &sig);
  return fq12_eq(&a, &b);
}

/* generic pairing equality e(p1, q1) == e(p2, q2), two pairings (reference-equivalent) */
API int bls_pairing_eq(const uint8_t* p1, const uint8_t* q1, const uint8_t* p2, const uint8_t* q2) {
  g1a a1, a2;
  g2a b1, b2;
  g1_load(&a1, p1);
  g1_load(&a2, p2);
  g2_load(&b1, q1);
  g2_load(&b2, q2);
  fq12 x, y;
  pairing(&x, &a1, &b1);
  pairing(&y, &a2, &b2);
  return fq12_eq(&x, &y);
}

/* pairing value (pairing 0.14 final exponentiation), 12 canonical Fq (c0.c0.c0 ... c1.c2.c1) */
API void bls_pairing(const uint8_t* p96, const uint8_t* q192, uint8_t* out576) {
  g1a p;
  g2a q;
  g1_load(&p, p96);
  g2_load(&q, q192);
  fq12 e;
  pairing(&e, &p, &q);
  const fq2* c[6] = {&e.c0.c0, &e.c0.c1, &e.c0.c2, &e.c1.c0, &e.c1.c1, &e.c1.c2};
  for (int k = 0; k < 6; k++) {
    fq_to_canon(out576 + 96 * k, &c[k]->c0);
    fq_to_canon(out576 + 96 * k + 48, &c[k]->c1);
  }
}

/* G1Affine::mul / G2Affine::mul by a 256-bit scalar (LE 32 bytes, any integer < 2^256). */
API void bls_g1_mul(const uint8_t* p96, const uint8_t* k32, uint8_t* out96) {
  g1a p, r;
  g1p acc;
  uint64_t k[4];
  memcpy(k, k32, 32);
  g1_load(&p, p96);
  g1_mul_bits(&acc, &p, k, 256);
  g1p_to_affine(&r, &acc);
  g1_store(out96, &r);
}
API void bls_g2_mul(const uint8_t* q192, const uint8_t* k32, uint8_t* out192) {
  g2a q, r;
  g2p acc;
  uint64_t k[4];
  memcpy(k, k32, 32);
  g2_load(&q, q192);
  g2_mul_bits(&acc, &q, k, 256);
  g2p_to_affine(&r, &acc);
  g2_store(out192, &r);
}
/* h2 * Q (G2 cofactor clearing inside pairing 0.14 G2::rand; used by hash_g2) */
API void bls_g2_clear_cofactor(const uint8_t* q192, uint8_t* out192) {
  g2a q, r;
  g2p acc;
  g2_load(&q, q192);
  g2_mul_bits(&acc, &q, G2_H2, G2_H2_BITS);
  g2p_to_affine(&r, &acc);
  g2_store(out192, &r);
}
API void bls_g1_add(const uint8_t* a96, const uint8_t* b96, uint8_t* out96) {
  g1a a, b, r;
  g1p pa, pb, s;
  g1_load(&a, a96);
  g1_load(&b, b96);
  g1p_zero(&pa);
  g1p_add_mixed(&pa, &pa, &a);
  g1p_zero(&pb);
  g1p_add_mixed(&pb, &pb, &b);
  g1p_add(&s, &pa, &pb);
  g1p_to_affine(&r, &s);
  g1_store(out96, &r);
}

/* PublicKeySet::combine_signatures / decrypt's interpolation: first t+1 samples, x_k = idx_k+1.
 * Returns 0, 4 (NotEnoughShares) or 5 (DuplicateEntry). */
API int bls_combine_g2(int t, int m, const uint64_t* idx, const uint8_t* pts192, uint8_t* out192) {
  if (m <= t) return 4;
  if (t == 0) { memcpy(out192, pts192, 192); return 0; }
  int s = t + 1;
  fr lam[256];
  int rc = lagrange_at_zero(s, idx, lam);
  if (rc) return rc;
  g2p acc, term;
  g2p_zero(&acc);
  for (int k = 0; k < s; k++) {
    g2a p;
    uint64_t kk[4];
    g2_load(&p, pts192 + 192 * (size_t)k);
    fr_to_canon(kk, &lam[k]);
    g2_mul_bits(&term, &p, kk, 256);
    g2p_add(&acc, &acc, &term);
  }
  g2a r;
  g2p_to_affine(&r, &acc);
  g2_store(out192, &r);
  return 0;
}
API int bls_combine_g1(int t, int m, const uint64_t* idx, const uint8_t* pts96, uint8_t* out96) {
  if (m <= t) return 4;
  if (t == 0) { memcpy(out96, pts96, 96); return 0; }
  int s = t + 1;
  fr lam[256];
  int rc = lagrange_at_zero(s, idx, lam);
  if (rc) return rc;
  g1p acc, term;
  g1p_zero(&acc);
  for (int k = 0; k < s; k++) {
    g1a p;
    uint64_t kk[4];
    g1_load(&p, pts96 + 96 * (size_t)k);
    fr_to_canon(kk, &lam[k]);
    g1_mul_bits(&term, &p, kk, 256);
    g1p_add(&acc, &acc, &term);
  }
  g1a r;
  g1p_to_affine(&r, &acc);
  g1_store(out96, &r);
  return 0;
}

/* BivarCommitment::evaluate(x, y) (threshold_crypto): Sum_{i,j<=t} C[coeff_pos(i,j)] * x^i * y^j,
 * with the crate's two scalar multiplications per term (by x^i, then by y^j). */
static int coeff_pos(int i, int j) { return i <= j ? j * (j + 1) / 2 + i : i * (i + 1) / 2 + j; }
API void bls_bivar_evaluate(int t, const uint8_t* commit96, uint64_t x, uint64_t y, uint8_t* out96) {
  fr fx, fy, xp, yp;
  uint64_t v[4] = {x, 0, 0, 0};
  fr_from_canon(&fx, v);
  v[0] = y;
  fr_from_canon(&fy, v);
  g1p acc;
  g1p_zero(&acc);
  memcpy(xp.l, FR_ONE, 32);
  for (int i = 0; i <= t; i++) {
    memcpy(yp.l, FR_ONE, 32);
    for (int j = 0; j <= t; j++) {
      g1a c, ci;
      g1p tmp;
      uint64_t k[4];
      g1_load(&c, commit96 + 96 * (size_t)coeff_pos(i, j));
      fr_to_canon(k, &xp);
      g1_mul_bits(&tmp, &c, k, 256);
      g1p_to_affine(&ci, &tmp);
      fr_to_canon(k, &yp);
      g1_mul_bits(&tmp, &ci, k, 256);
      g1p_add(&acc, &acc, &tmp);
      fr_mul(&yp, &yp, &fy);
    }
    fr_mul(&xp, &xp, &fx);
  }
  g1a r;
  g1p_to_affine(&r, &acc);
  g1_store(out96, &r);
}
/* BivarCommitment::row(x): out[i] = Sum_j C[coeff_pos(i,j)] * x^j, i = 0..t */
API void bls_bivar_row(int t, const uint8_t* commit96, uint64_t x, uint8_t* out96) {
  fr fx, xp;
  uint64_t v[4] = {x, 0, 0, 0};
  fr_from_canon(&fx, v);
  for (int i = 0; i <= t; i++) {
    g1p acc, tmp;
    g1p_zero(&acc);
    memcpy(xp.l, FR_ONE, 32);
    for (int j = 0; j <= t; j++) {
      g1a c;
      uint64_t k[4];
      g1_load(&c, commit96 + 96 * (size_t)coeff_pos(i, j));
      fr_to_canon(k, &xp);
      g1_mul_bits(&tmp, &c, k, 256);
      g1p_add(&acc, &acc, &tmp);
      fr_mul(&xp, &xp, &fx);
    }
    g1a r;
    g1p_to_affine(&r, &acc);
    g1_store(out96 + 96 * (size_t)i, &r);
  }
}

/* ------------------------------------------------------------------ batched, multi-threaded */
typedef struct {
  size_t lo, hi;
  const uint8_t *pks, *sigs, *hashes;
  const uint32_t* doc_idx;
  uint8_t* verdicts;
} vjob;
static void* vworker(void* arg) {
  vjob* j = (vjob*)arg;
  for (size_t i = j->lo; i < j->hi; i++) {
    uint32_t d = j->doc_idx ? j->doc_idx[i] : (uint32_t)i;
    j->verdicts[i] = (uint8_t)bls_verify_g2(j->pks + 96 * i, j->sigs + 192 * i, j->hashes + 192 * (size_t)d);
  }
  return 0;
}
/* n x PublicKeyShare::verify_g2 over `threads` std threads (the "rayon over all cores" analogue). */
API void bls_verify_g2_batch(size_t n, const uint8_t* pks, const uint8_t* sigs, const uint8_t* hashes,
                             const uint32_t* doc_idx, uint8_t* verdicts, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  vjob jobs[256];
  for (int k = 0; k < threads; k++) {
    jobs[k].lo = n * k / threads;
    jobs[k].hi = n * (k + 1) / threads;
    jobs[k].pks = pks;
    jobs[k].sigs = sigs;
    jobs[k].hashes = hashes;
    jobs[k].doc_idx = doc_idx;
    jobs[k].verdicts = verdicts;
    pthread_create(&th[k], 0, vworker, &jobs[k]);
  }
  for (int k = 0; k < threads; k++) pthread_join(th[k], 0);
}
