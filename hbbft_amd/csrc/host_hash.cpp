// Host stage of the path (C ABI in include/hbbft_hip.h, "host stage"): threshold_crypto 0.3's
// hash_g2, hash_g1_g2, xor_with_hash, Signature::parity and encrypt_with_rng, the secret-key
// scalar multiplications (sign_g2, decrypt_share) and the compressed point encodings, batched
// over std::thread workers.  Conventions (parity with threshold_crypto
// itself is unpinned):
//   SHA3-256      FIPS-202 (tiny-keccak 1.4 sha3_256)
//   ChaChaRng     rand_chacha 0.1 from_seed: key = the 32-byte seed as 8 LE words, 64-bit block
//                 counter in words 12-13, zero nonce; consumed as a flat LE word stream
//                 (next_u32 = next word, next_u64 = two words, low first)
//   Fq::rand      ff 0.4: 6 x next_u64 LE limbs, top 3 bits cleared, rejected if >= p, the limbs
//                 ARE the Montgomery representation
//   G2::rand      pairing 0.14: x = (rand, rand); greatest = next_u32 & 1; y = the larger root of
//                 x^3 + 4(1 + u) iff greatest (Fq2 order: c1, then c0); P = h2 (x, y); retry on
//                 a non-square or P = O
//   hash_g2(m)    G2::rand(ChaChaRng(sha3(m)))                (threshold_sign.rs:151)
//   hash_g1_g2    hash_g2((V if |V| <= 64 else sha3(V)) || compress(U))
//   xor_with_hash V xor low byte of successive next_u32 of ChaChaRng(sha3(compress(g)))
//   parity        popcount of the XOR-fold of the 192-byte uncompressed G2 encoding, odd
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/hbbft_hip.h"
#include "host_bls.hpp"

namespace hh {

// ---------------------------------------------------------------- constants
static Fq fq_from_canon_raw(const uint64_t* v, const Fq& r2) {
  Fq a;
  memcpy(a.l, v, sizeof(a.l));
  return fq_mul(a, r2);
}
static Consts make_consts() {
  Consts c;
  // R mod p = 2^384 mod p by modular doubling of 1; R^2 mod p = R * 2^384 mod p likewise
  uint64_t v[6] = {1, 0, 0, 0, 0, 0};
  for (int k = 0; k < 768; k++) {
    uint64_t carry = 0;
    for (int i = 0; i < 6; i++) {
      const uint64_t nc = v[i] >> 63;
      v[i] = (v[i] << 1) | carry;
      carry = nc;
    }
    if (carry || geq_p(v)) sub_p(v);
    if (k == 383) memcpy(c.one.l, v, sizeof(v));
  }
  memcpy(c.r2.l, v, sizeof(v));
  const uint64_t four[6] = {4, 0, 0, 0, 0, 0};
  c.b1 = fq_mul(*(const Fq*)four, c.r2);
  // 1/2 = (p + 1) / 2
  uint64_t half[6];
  memcpy(half, P, sizeof(P));
  half[0] += 1;  // p is odd: no carry
  for (int i = 0; i < 6; i++) half[i] = (half[i] >> 1) | (i < 5 ? half[i + 1] << 63 : 0);
  c.inv2 = fq_from_canon_raw(half, c.r2);
  // p - 2, (p - 3) / 4, (p - 1) / 2
  memcpy(c.pm2, P, sizeof(P));
  c.pm2[0] -= 2;
  uint64_t pm3[6];
  memcpy(pm3, P, sizeof(P));
  pm3[0] -= 3;
  for (int i = 0; i < 6; i++) c.pm3d4[i] = (pm3[i] >> 2) | (i < 5 ? pm3[i + 1] << 62 : 0);
  uint64_t pm1[6];
  memcpy(pm1, P, sizeof(P));
  pm1[0] -= 1;
  for (int i = 0; i < 6; i++) c.pm1d2[i] = (pm1[i] >> 1) | (i < 5 ? pm1[i + 1] << 63 : 0);
  return c;
}
const Consts& consts() {
  static const Consts c = make_consts();
  return c;
}

// Square root in Fq2 by the norm (p = 3 mod 4, u^2 = -1): with s = v^((p-3)/4), s v is a root of v and
// s^2 v = v^((p-1)/2) its Legendre symbol, so each Fq exponentiation decides and extracts at once.
// a = a0 + a1 u is a square iff its norm a0^2 + a1^2 is; then x0^2 = delta = (a0 +- sqrt(norm)) / 2
// (exactly one sign is a square) and x1 = a1 / (2 x0) = a1 t / 2 with t = delta^((p-3)/4) = 1 / x0.
// Two or three Fq exponentiations instead of two Fq2 ones (the previous algorithm); which of the
// two roots comes out does not matter: G2::rand keeps the one its `greatest` bit selects.
bool f2_sqrt(const Fq2& a, Fq2& out) {
  const Consts& k = consts();
  const Fq one = fq_one();
  if (fq_is_zero(a.c1)) {
    if (fq_is_zero(a.c0)) {
      out = a;
      return true;
    }
    const Fq s = fq_pow(a.c0, k.pm3d4, 6);
    const Fq root = fq_mul(s, a.c0);
    if (fq_eq(fq_mul(root, s), one))
      out = {root, fq_zero()};
    else
      out = {fq_zero(), root};  // root^2 = -a0, so (root u)^2 = a0
  } else {
    const Fq norm = fq_add(fq_sqr(a.c0), fq_sqr(a.c1));
    const Fq s = fq_pow(norm, k.pm3d4, 6);
    const Fq gamma = fq_mul(s, norm);
    if (!fq_eq(fq_mul(gamma, s), one)) return false;  // the norm is not a square
    Fq delta = fq_mul(fq_add(a.c0, gamma), k.inv2);
    Fq t = fq_pow(delta, k.pm3d4, 6);
    Fq x0 = fq_mul(t, delta);
    if (!fq_eq(fq_mul(x0, t), one)) {
      delta = fq_mul(fq_sub(a.c0, gamma), k.inv2);
      t = fq_pow(delta, k.pm3d4, 6);
      x0 = fq_mul(t, delta);
    }
    out = {x0, fq_mul(fq_mul(a.c1, t), k.inv2)};
  }
  return f2_eq(f2_sqr(out), a);
}

// ---------------------------------------------------------------- encodings
void g1_to_abi(const Jac<Fq>& p, uint8_t* out) {
  Fq x, y;
  if (!jac_affine(p, x, y)) {
    memset(out, 0, HBH_G1_BYTES);
    return;
  }
  fq_to_le(x, out);
  fq_to_le(y, out + 48);
}
void g2_to_abi(const Jac<Fq2>& p, uint8_t* out) {
  Fq2 x, y;
  if (!jac_affine(p, x, y)) {
    memset(out, 0, HBH_G2_BYTES);
    return;
  }
  fq_to_le(x.c0, out);
  fq_to_le(x.c1, out + 48);
  fq_to_le(y.c0, out + 96);
  fq_to_le(y.c1, out + 144);
}
void g1_aff_to_abi(const Aff<Fq>& p, uint8_t* out) {
  if (p.inf) {
    memset(out, 0, HBH_G1_BYTES);
    return;
  }
  fq_to_le(p.x, out);
  fq_to_le(p.y, out + 48);
}
void g2_aff_to_abi(const Aff<Fq2>& p, uint8_t* out) {
  if (p.inf) {
    memset(out, 0, HBH_G2_BYTES);
    return;
  }
  fq_to_le(p.x.c0, out);
  fq_to_le(p.x.c1, out + 48);
  fq_to_le(p.y.c0, out + 96);
  fq_to_le(p.y.c1, out + 144);
}
static bool all_zero(const uint8_t* b, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (b[i]) return false;
  return true;
}
bool g1_from_abi(const uint8_t* in, Jac<Fq>& p) {
  if (all_zero(in, HBH_G1_BYTES)) {
    p = jac_inf<Fq>();
    return true;
  }
  p.z = fq_one();
  return fq_from_le(in, p.x) && fq_from_le(in + 48, p.y);
}
bool g2_from_abi(const uint8_t* in, Jac<Fq2>& p) {
  if (all_zero(in, HBH_G2_BYTES)) {
    p = jac_inf<Fq2>();
    return true;
  }
  p.z = f2_one();
  return fq_from_le(in, p.x.c0) && fq_from_le(in + 48, p.x.c1) && fq_from_le(in + 96, p.y.c0) &&
         fq_from_le(in + 144, p.y.c1);
}
// pairing 0.14 G1Compressed (48 B): big-endian x, 0x80 compressed, 0x40 infinity, 0x20 y > -y;
// false if a coordinate is not canonical (>= p)
static bool g1_compress(const uint8_t* abi, uint8_t* out) {
  if (all_zero(abi, HBH_G1_BYTES)) {
    memset(out, 0, 48);
    out[0] = 0xc0;
    return true;
  }
  Fq x, y;
  const bool ok = fq_from_le(abi, x) & fq_from_le(abi + 48, y);
  fq_to_be(x, out);
  out[0] |= 0x80 | (fq_gt(y, fq_neg(y)) ? 0x20 : 0);
  return ok;
}
// G2Compressed (96 B): x.c1 || x.c0 big-endian, flags as G1 with the Fq2 order (c1, then c0)
static bool g2_compress(const uint8_t* abi, uint8_t* out) {
  if (all_zero(abi, HBH_G2_BYTES)) {
    memset(out, 0, 96);
    out[0] = 0xc0;
    return true;
  }
  Fq2 x, y;
  const bool ok = fq_from_le(abi, x.c0) & fq_from_le(abi + 48, x.c1) & fq_from_le(abi + 96, y.c0) &
                  fq_from_le(abi + 144, y.c1);
  fq_to_be(x.c1, out);
  fq_to_be(x.c0, out + 48);
  out[0] |= 0x80 | (f2_gt(y, f2_neg(y)) ? 0x20 : 0);
  return ok;
}
// G2Uncompressed (192 B): x.c1 x.c0 y.c1 y.c0 big-endian; infinity 0x40 || 0
static void g2_uncompressed(const uint8_t* abi, uint8_t* out) {
  memset(out, 0, 192);
  if (all_zero(abi, HBH_G2_BYTES)) {
    out[0] = 0x40;
    return;
  }
  const int order[4] = {1, 0, 3, 2};  // ABI word groups x.c0 x.c1 y.c0 y.c1
  for (int k = 0; k < 4; k++) {
    const uint8_t* le = abi + 48 * order[k];
    for (int i = 0; i < 48; i++) out[48 * k + i] = le[47 - i];
  }
}

// ---------------------------------------------------------------- SHA3-256 (FIPS-202)
static const uint64_t KECCAK_RC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
static const int KECCAK_ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
static inline uint64_t rotl64(uint64_t v, int c) { return c ? (v << c) | (v >> (64 - c)) : v; }
static void keccak_f(uint64_t* s) {
  for (int round = 0; round < 24; round++) {
    uint64_t c[5], d[5], b[25];
    for (int x = 0; x < 5; x++) c[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
    for (int x = 0; x < 5; x++) d[x] = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
    for (int i = 0; i < 25; i++) s[i] ^= d[i % 5];
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(s[x + 5 * y], KECCAK_ROT[x + 5 * y]);
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) s[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
    s[0] ^= KECCAK_RC[round];
  }
}
static void sha3_256(const uint8_t* msg, size_t len, uint8_t* out) {
  const size_t rate = 136;
  uint64_t s[25];
  memset(s, 0, sizeof(s));
  uint8_t block[136];
  while (len >= rate) {
    for (size_t i = 0; i < rate / 8; i++) {
      uint64_t w;
      memcpy(&w, msg + 8 * i, 8);
      s[i] ^= w;
    }
    keccak_f(s);
    msg += rate;
    len -= rate;
  }
  memset(block, 0, rate);
  memcpy(block, msg, len);
  block[len] ^= 0x06;
  block[rate - 1] ^= 0x80;
  for (size_t i = 0; i < rate / 8; i++) {
    uint64_t w;
    memcpy(&w, block + 8 * i, 8);
    s[i] ^= w;
  }
  keccak_f(s);
  memcpy(out, s, 32);
}

// ---------------------------------------------------------------- ChaCha20 word stream
struct ChaChaRng {
  uint32_t key[8];
  uint64_t counter = 0;
  uint32_t buf[16];
  int idx = 16;
  explicit ChaChaRng(const uint8_t* seed) { memcpy(key, seed, 32); }
  static inline uint32_t rotl(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }
  void refill() {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                      key[4], key[5], key[6], key[7], (uint32_t)counter, (uint32_t)(counter >> 32), 0, 0};
    uint32_t x[16];
    memcpy(x, s, sizeof(s));
    auto qr = [&](int a, int b, int c, int d) {
      x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16);
      x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12);
      x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8);
      x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7);
    };
    for (int r = 0; r < 10; r++) {
      qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
      qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
    }
    for (int i = 0; i < 16; i++) buf[i] = x[i] + s[i];
    counter++;
    idx = 0;
  }
  uint32_t next_u32() {
    if (idx >= 16) refill();
    return buf[idx++];
  }
  uint64_t next_u64() {
    const uint64_t lo = next_u32();
    const uint64_t hi = next_u32();
    return (hi << 32) | lo;
  }
  Fq gen_fq() {
    for (;;) {
      Fq a;
      for (int i = 0; i < 6; i++) a.l[i] = next_u64();
      a.l[5] &= 0xffffffffffffffffull >> 3;
      if (!geq_p(a.l)) return a;  // the limbs are the Montgomery representation
    }
  }
  bool gen_bool() { return (next_u32() & 1) == 1; }
};

// ---------------------------------------------------------------- scalars (Fr, little-endian 64-bit limbs)
static const uint64_t R_ORDER[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                                    0x73eda753299d7d48ull};
static bool geq_r(const uint64_t* a) {
  for (int i = 3; i >= 0; i--)
    if (a[i] != R_ORDER[i]) return a[i] > R_ORDER[i];
  return true;
}
static void sub_r(uint64_t* a) {
  uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    const u128 d = (u128)a[i] - R_ORDER[i] - br;
    a[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
}
// k mod r for any 256-bit k (k < 2^256 < 3 r): the group elements are of order r, so every scalar
// multiplication below is by the reduced scalar
static void reduce_r(uint64_t* k) {
  while (geq_r(k)) sub_r(k);
}
// a b mod r (a, b < r): Montgomery CIOS with R = 2^256, then one more product by R^2 mod r
static void fr_mont(const uint64_t* a, const uint64_t* b, uint64_t* out) {
  const uint64_t RINV = 0xfffffffeffffffffull;  // -r^-1 mod 2^64
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 4; j++) {
      const u128 s = (u128)a[j] * b[i] + t[j] + c;
      t[j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[4] + c;
    t[4] = (uint64_t)s;
    t[5] = (uint64_t)(s >> 64);
    const uint64_t m = t[0] * RINV;
    s = (u128)m * R_ORDER[0] + t[0];
    c = (uint64_t)(s >> 64);
    for (int j = 1; j < 4; j++) {
      s = (u128)m * R_ORDER[j] + t[j] + c;
      t[j - 1] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    s = (u128)t[4] + c;
    t[3] = (uint64_t)s;
    t[4] = t[5] + (uint64_t)(s >> 64);
  }
  memcpy(out, t, 32);
  if (t[4] || geq_r(out)) sub_r(out);
}
static void fr_mul(const uint64_t* a, const uint64_t* b, uint64_t* out) {
  static const uint64_t R2R[4] = {0xc999e990f3f29c6dull, 0x2b6cedcb87925c23ull, 0x05d314967254398full,
                                  0x0748d9d99f59ff11ull};  // 2^512 mod r
  uint64_t t[4];
  fr_mont(a, b, t);
  fr_mont(t, R2R, out);
}
static void fr_to_mont(const uint64_t* a, uint64_t* out) {
  static const uint64_t R2R[4] = {0xc999e990f3f29c6dull, 0x2b6cedcb87925c23ull, 0x05d314967254398full,
                                  0x0748d9d99f59ff11ull};
  fr_mont(a, R2R, out);
}
// a + b mod r (a, b < r)
static void fr_add(const uint64_t* a, const uint64_t* b, uint64_t* out) {
  uint64_t c = 0;
  for (int i = 0; i < 4; i++) {
    const u128 s = (u128)a[i] + b[i] + c;
    out[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (c || geq_r(out)) sub_r(out);
}
// k = q d + rem for a 64-bit d: k becomes q, returns rem
static uint64_t divmod_u64(uint64_t* k, int nl, uint64_t d) {
  u128 rem = 0;
  for (int i = nl - 1; i >= 0; i--) {
    const u128 cur = (rem << 64) | k[i];
    k[i] = (uint64_t)(cur / d);
    rem = cur % d;
  }
  return (uint64_t)rem;
}
// width-5 NAF of a non-negative integer (nl <= 2 little-endian limbs): digits in {0, +-1, ..., +-15},
// at most 64 nl + 1 of them, least significant first; returns the digit count
static int wnaf5(const uint64_t* a, int nl, int8_t* out) {
  uint64_t k[3] = {0, 0, 0};
  memcpy(k, a, 8 * (size_t)nl);
  int n = 0;
  while (k[0] | k[1] | k[2]) {
    int d = 0;
    if (k[0] & 1) {
      d = (int)(k[0] & 31);
      if (d >= 16) d -= 32;
      // k -= d
      if (d > 0) {
        const u128 s = (u128)k[0] - (uint64_t)d;
        k[0] = (uint64_t)s;
        uint64_t br = (uint64_t)(s >> 64) & 1;
        for (int i = 1; i < 3 && br; i++) br = (k[i]-- == 0);
      } else {
        const u128 s = (u128)k[0] + (uint64_t)(-d);
        k[0] = (uint64_t)s;
        uint64_t c = (uint64_t)(s >> 64);
        for (int i = 1; i < 3 && c; i++) c = (++k[i] == 0);
      }
    }
    out[n++] = (int8_t)d;
    k[0] = (k[0] >> 1) | (k[1] << 63);
    k[1] = (k[1] >> 1) | (k[2] << 63);
    k[2] >>= 1;
  }
  return n;
}
// sum_i [digit_i] base_i for M bases with width-5 NAF digits, one doubling chain; tab[i][j] = (2 j + 1) base_i
template <class F, int M>
static Jac<F> multi_wnaf(const Jac<F> (*tab)[8], int8_t (*naf)[130], const int* len) {
  int top = 0;
  for (int i = 0; i < M; i++) top = std::max(top, len[i]);
  Jac<F> r = jac_inf<F>();
  for (int b = top - 1; b >= 0; b--) {
    r = jac_dbl(r);
    for (int i = 0; i < M; i++) {
      if (b >= len[i] || !naf[i][b]) continue;
      const int d = naf[i][b];
      r = jac_add(r, d > 0 ? tab[i][d >> 1] : jac_neg(tab[i][(-d) >> 1]));
    }
  }
  return r;
}
template <class F>
static void odd_multiples(const Jac<F>& p, Jac<F>* t8) {
  t8[0] = p;
  const Jac<F> p2 = jac_dbl(p);
  for (int j = 1; j < 8; j++) t8[j] = jac_add(t8[j - 1], p2);
}

// ---------------------------------------------------------------- endomorphisms
// G1: phi(x, y) = (beta x, y) acts as [lambda] on G1, lambda = z^2 - 1 (z = -0xd201000000010000), and
// r = lambda^2 + lambda + 1, so k = k2 lambda + k1 with k1, k2 < 2^128 (GLV).
static const uint64_t BETA_CANON[6] = {0x8bfd00000000aaacull, 0x409427eb4f49fffdull, 0x897d29650fb85f9bull,
                                       0xaa0d857d89759ad4ull, 0xec02408663d4de85ull, 0x1a0111ea397fe699ull};
static const u128 LAMBDA = ((u128)0xac45a4010001a402ull << 64) | 0x00000000ffffffffull;
// G2: psi(x, y) = (conj(x) cx, conj(y) cy) (untwist-Frobenius-twist) on all of E'(Fq2); on G2 it acts
// as [p] = [z] mod r.  cx = CX1 u.
static const uint64_t CX1_CANON[6] = {0x8bfd00000000aaadull, 0x409427eb4f49fffdull, 0x897d29650fb85f9bull,
                                      0xaa0d857d89759ad4ull, 0xec02408663d4de85ull, 0x1a0111ea397fe699ull};
static const uint64_t CY_CANON[2][6] = {
    {0xf1ee7b04121bdea2ull, 0x304466cf3e67fa0aull, 0xef396489f61eb45eull, 0x1c3dedd930b1cf60ull,
     0xe2e9c448d77a2cd9ull, 0x135203e60180a68eull},
    {0xc81084fbede3cc09ull, 0xee67992f72ec05f4ull, 0x77f76e17009241c5ull, 0x48395dabc2d3435eull,
     0x6831e36d6bd17ffeull, 0x06af0e0437ff400bull}};
static const uint64_t Z_ABS = 0xd201000000010000ull;
// h2 P = [KCOF] Q_bp for every P on E'(Fq2), Q_bp the Budroni-Pintore image below (KCOF = h2 s^-1 mod r,
// s = (z^2 - z - 1) + (z - 1) p + 2 p^2 mod r, the scalar by which Q_bp's map acts on G2)
static const uint64_t KCOF[4] = {0x55555554aaaaaaabull, 0x37d2aaab55543d54ull, 0x66689d580335f2acull,
                                 0x26a48d1bb889d46dull};
struct EndoConsts {
  Fq beta, cx1;
  Fq2 cy;
};
static const EndoConsts& endo() {
  static const EndoConsts e = [] {
    EndoConsts c;
    c.beta = fq_from_canon(BETA_CANON);
    c.cx1 = fq_from_canon(CX1_CANON);
    c.cy = {fq_from_canon(CY_CANON[0]), fq_from_canon(CY_CANON[1])};
    return c;
  }();
  return e;
}
static Jac<Fq2> psi(const Jac<Fq2>& p) {
  const EndoConsts& e = endo();
  const Fq2 x = f2_conj(p.x);
  return {{fq_neg(fq_mul(x.c1, e.cx1)), fq_mul(x.c0, e.cx1)}, f2_mul(f2_conj(p.y), e.cy), f2_conj(p.z)};
}
static Jac<Fq> phi(const Jac<Fq>& p) { return {fq_mul(p.x, endo().beta), p.y, p.z}; }
template <class F>
static Jac<F> mul_zabs(const Jac<F>& p) {
  Jac<F> r = p;
  for (int b = 62; b >= 0; b--) {
    r = jac_dbl(r);
    if ((Z_ABS >> b) & 1) r = jac_add(r, p);
  }
  return r;
}

// [k] P for P in G1 (subgroup contract): GLV split, width-5 NAF, 129 doublings
static Jac<Fq> g1_mul_glv(const Jac<Fq>& p, const uint64_t* k_in) {
  uint64_t k[4];
  memcpy(k, k_in, 32);
  reduce_r(k);
  // k = q lambda + rem by shift-subtract (lambda > 2^127: track the bit shifted out of rem)
  u128 rem = 0, q = 0;
  for (int b = 255; b >= 0; b--) {
    const bool carry = (rem >> 127) != 0;
    rem = (rem << 1) | ((k[b >> 6] >> (b & 63)) & 1);
    if (carry || rem >= LAMBDA) {
      rem -= LAMBDA;
      q |= (u128)1 << b;  // q < 2^128: b < 128 whenever this fires
    }
  }
  const uint64_t k1[2] = {(uint64_t)rem, (uint64_t)(rem >> 64)};
  const uint64_t k2[2] = {(uint64_t)q, (uint64_t)(q >> 64)};
  Jac<Fq> tab[2][8];
  odd_multiples(p, tab[0]);
  for (int j = 0; j < 8; j++) tab[1][j] = phi(tab[0][j]);
  int8_t naf[2][130];
  const int len[2] = {wnaf5(k1, 2, naf[0]), wnaf5(k2, 2, naf[1])};
  return multi_wnaf<Fq, 2>(tab, naf, len);
}

// [k] Q for Q in G2 (subgroup contract): k mod r in base |z| (four digits < 2^64), [|z|] = -psi on G2,
// so k Q = sum_i d_i (-psi)^i (Q); width-5 NAF per digit, 65 doublings
static Jac<Fq2> g2_mul_gls(const Jac<Fq2>& q, const uint64_t* k_in) {
  uint64_t k[4];
  memcpy(k, k_in, 32);
  reduce_r(k);
  uint64_t d[4];
  for (int i = 0; i < 3; i++) d[i] = divmod_u64(k, 4, Z_ABS);
  d[3] = k[0];  // k < r < |z|^4: the last quotient fits one limb
  Jac<Fq2> tab[4][8];
  odd_multiples(q, tab[0]);
  for (int i = 1; i < 4; i++)
    for (int j = 0; j < 8; j++) tab[i][j] = jac_neg(psi(tab[i - 1][j]));
  int8_t naf[4][130];
  int len[4];
  for (int i = 0; i < 4; i++) len[i] = wnaf5(&d[i], 1, naf[i]);
  return multi_wnaf<Fq2, 4>(tab, naf, len);
}

// Q_bp = [z^2 - z - 1] P + [z - 1] psi(P) + psi^2(2P) for any P on E'(Fq2) (Budroni-Pintore 2017, the
// chain of the IETF hash-to-curve clear_cofactor): Q_bp lies in G2 and h2 P = [KCOF] Q_bp, so pairing
// 0.14's cofactor multiplication by the 636-bit h2 becomes two 64-bit chains by |z| plus a GLS
// multiplication (or none at all when the caller multiplies by a scalar anyway: W = H r).
static Jac<Fq2> cofactor_bp(const Jac<Fq2>& p) {
  const Jac<Fq2> t1 = jac_neg(mul_zabs(p));  // [z] P
  Jac<Fq2> t2 = psi(p);
  Jac<Fq2> t3 = psi(psi(jac_dbl(p)));
  t3 = jac_add(t3, jac_neg(t2));
  t2 = jac_add(t1, t2);
  t2 = jac_neg(mul_zabs(t2));  // [z] ([z] P + psi(P))
  t3 = jac_add(t3, t2);
  t3 = jac_add(t3, jac_neg(t1));
  return jac_add(t3, jac_neg(p));
}

// fixed-base comb of g1 (encrypt_with_rng's U = g1 r): T[w][d - 1] = d 2^(8 w) g1 (affine), 32 x 255 points
// built once per process; [k] g1 = sum_w T[w][byte_w(k)]: 32 mixed additions, no doubling
static const uint64_t G1_CANON[12] = {0xfb3af00adb22c6bbull, 0x6c55e83ff97a1aefull, 0xa14e3a3f171bac58ull,
                                      0xc3688c4f9774b905ull, 0x2695638c4fa9ac0full, 0x17f1d3a73197d794ull,
                                      0x0caa232946c5e7e1ull, 0xd03cc744a2888ae4ull, 0x00db18cb2c04b3edull,
                                      0xfcf5e095d5d00af6ull, 0xa09e30ed741d8ae4ull, 0x08b3f481e3aaa0f1ull};
static const std::vector<Aff<Fq>>& g1_comb() {
  static const std::vector<Aff<Fq>> tab = [] {
    std::vector<Aff<Fq>> t(32 * 255);
    Aff<Fq> base = {fq_from_canon(G1_CANON), fq_from_canon(G1_CANON + 6), false};
    std::vector<Jac<Fq>> row(256);
    for (int w = 0; w < 32; w++) {
      row[0] = jac_from_aff(base);
      for (int d = 1; d < 256; d++) row[d] = jac_add_aff(row[d - 1], base.x, base.y);  // row[d] = (d+1) base
      std::vector<Aff<Fq>> aff(256);
      jac_batch_affine(row.data(), aff.data(), 256);
      for (int d = 0; d < 255; d++) t[w * 255 + d] = aff[d];
      base = aff[255];  // 256 base
    }
    return t;
  }();
  return tab;
}
static Jac<Fq> g1_mul_gen(const uint64_t* k_in) {
  uint64_t k[4];
  memcpy(k, k_in, 32);
  reduce_r(k);
  const std::vector<Aff<Fq>>& t = g1_comb();
  Jac<Fq> r = jac_inf<Fq>();
  for (int w = 0; w < 32; w++) {
    const int d = (int)((k[w >> 3] >> (8 * (w & 7))) & 0xff);
    if (d) r = jac_add_aff(r, t[w * 255 + d - 1].x, t[w * 255 + d - 1].y);
  }
  return r;
}

// 4-bit fixed-base comb of a G1 point used by many multiplications in one call (encrypt_with_rng's pk r
// when a batch encrypts to a few keys, as a SyncKeyGen node does: 100 values to each of N keys):
// T[w * 15 + d - 1] = d 16^w P, 64 x 15 affine points from one batch normalisation; [k] P = 64 mixed
// additions instead of GLV's 129 doublings + ~43 additions
static std::vector<Aff<Fq>> comb4_build(const Jac<Fq>& p) {
  std::vector<Jac<Fq>> j(64 * 16);
  Jac<Fq> base = p;
  for (int w = 0; w < 64; w++) {
    j[w * 16] = base;
    for (int d = 1; d < 16; d++) j[w * 16 + d] = jac_add(j[w * 16 + d - 1], base);  // (d + 1) base
    base = j[w * 16 + 15];                                                           // 16 base
  }
  std::vector<Aff<Fq>> a(64 * 16), t(64 * 15);
  jac_batch_affine(j.data(), a.data(), j.size());
  for (int w = 0; w < 64; w++)
    for (int d = 0; d < 15; d++) t[w * 15 + d] = a[w * 16 + d];
  return t;
}
static Jac<Fq> comb4_mul(const std::vector<Aff<Fq>>& t, const uint64_t* k_in) {
  uint64_t k[4];
  memcpy(k, k_in, 32);
  reduce_r(k);
  Jac<Fq> r = jac_inf<Fq>();
  for (int w = 0; w < 64; w++) {
    const int d = (int)((k[w >> 4] >> (4 * (w & 15))) & 15);
    if (d && !t[w * 15 + d - 1].inf) r = jac_add_aff(r, t[w * 15 + d - 1].x, t[w * 15 + d - 1].y);
  }
  return r;
}

// ---------------------------------------------------------------- hash to G2
// pairing 0.14 G2::rand up to the cofactor multiplication: the first sampled curve point (x, y) whose
// h2 multiple is not O, returned as Q_bp (h2 (x, y) = [KCOF] Q_bp; Q_bp = O exactly when h2 (x, y) = O)
static Jac<Fq2> g2_rand_bp(ChaChaRng& rng) {
  const Fq four = consts().b1;
  const Fq2 b2 = {four, four};  // 4 (1 + u)
  for (;;) {
    Fq2 x;
    x.c0 = rng.gen_fq();
    x.c1 = rng.gen_fq();
    const bool greatest = rng.gen_bool();
    Fq2 y;
    if (!f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), b2), y)) continue;
    const Fq2 ny = f2_neg(y);
    // keep y iff (y > -y) == greatest
    if (f2_gt(y, ny) != greatest) y = ny;
    const Jac<Fq2> q = cofactor_bp(Jac<Fq2>{x, y, f2_one()});
    if (!f2_is_zero(q.z)) return q;
  }
}

// Q_bp of hash_g2(msg)
static Jac<Fq2> hash_g2_bp(const uint8_t* msg, size_t len) {
  uint8_t seed[32];
  sha3_256(msg, len, seed);
  ChaChaRng rng(seed);
  return g2_rand_bp(rng);
}

static void hash_g2(const uint8_t* msg, size_t len, uint8_t* out) {
  g2_to_abi(g2_mul_gls(hash_g2_bp(msg, len), KCOF), out);
}

// the message hash_g1_g2 hashes: (V if |V| <= 64 else sha3(V)) || compress(U)
static std::vector<uint8_t> g1_g2_msg(const uint8_t* u_abi, const uint8_t* v, size_t vlen) {
  std::vector<uint8_t> m;
  if (vlen > 64) {
    m.resize(32);
    sha3_256(v, vlen, m.data());
  } else {
    m.assign(v, v + vlen);
  }
  uint8_t cu[48];
  g1_compress(u_abi, cu);
  m.insert(m.end(), cu, cu + 48);
  return m;
}

static void hash_g1_g2(const uint8_t* u_abi, const uint8_t* v, size_t vlen, uint8_t* out) {
  const std::vector<uint8_t> m = g1_g2_msg(u_abi, v, vlen);
  hash_g2(m.data(), m.size(), out);
}

static void xor_with_hash(const uint8_t* g_abi, const uint8_t* data, size_t len, uint8_t* out) {
  uint8_t cg[48], seed[32];
  g1_compress(g_abi, cg);
  sha3_256(cg, 48, seed);
  ChaChaRng rng(seed);
  for (size_t i = 0; i < len; i++) out[i] = data[i] ^ (uint8_t)(rng.next_u32() & 0xff);
}

// ---------------------------------------------------------------- batching
// CPUs this process may actually use: the affinity mask, capped by a cgroup v2 CPU quota
// (cpu.max) and by OMP_NUM_THREADS / HBH_HOST_THREADS when set -- on a shared host
// hardware_concurrency() counts the whole machine, and a thread per item beyond the quota only
// adds creation cost and throttling.
static size_t usable_cpus() {
  static const size_t cached = [] {
    size_t t = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) t = std::min(t, (size_t)std::max(1, CPU_COUNT(&set)));
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char quota[32] = {0};
      long period = 0;
      if (std::fscanf(f, "%31s %ld", quota, &period) == 2 && std::strcmp(quota, "max") != 0 && period > 0) {
        const long q = std::atol(quota);
        if (q > 0) t = std::min(t, (size_t)std::max(1L, (q + period - 1) / period));
      }
      std::fclose(f);
    }
    for (const char* env : {"HBH_HOST_THREADS", "OMP_NUM_THREADS"}) {
      const char* v = std::getenv(env);
      if (v && std::atoi(v) > 0) {
        t = std::min(t, (size_t)std::atoi(v));
        break;
      }
    }
    return t;
  }();
  return cached;
}

// run f(i) for i < n over `threads` workers (0 = the usable CPUs)
template <class F>
static void parallel_for(size_t n, int threads, F f) {
  size_t t = threads > 0 ? (size_t)threads : usable_cpus();
  t = std::min(t, n);
  if (t <= 1) {
    for (size_t i = 0; i < n; i++) f(i);
    return;
  }
  std::atomic<size_t> next(0);
  std::vector<std::thread> ws;
  for (size_t w = 0; w < t; w++)
    ws.emplace_back([&]() {
      for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
    });
  for (auto& w : ws) w.join();
}

}  // namespace hh

namespace {
thread_local std::string g_host_error;
int host_fail(int code, const char* msg) {
  g_host_error = msg;
  return code;
}
// scalar (32 B LE) -> 4 limbs
void scalar_limbs(const uint8_t* s, uint64_t* k) { memcpy(k, s, 32); }
}  // namespace

extern "C" {

const char* hbh_host_last_error(void) { return g_host_error.c_str(); }

int hbh_hash_g2(size_t n, const uint8_t* data, const size_t* offsets, uint8_t* out, int threads) {
  if (n == 0) return HBH_OK;
  if (!offsets || !out || (!data && offsets[n] != 0)) return host_fail(HBH_ERR_ARG, "null pointer");
  for (size_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i]) return host_fail(HBH_ERR_ARG, "offsets not ascending");
  hh::parallel_for(n, threads, [&](size_t i) {
    hh::hash_g2(data + offsets[i], offsets[i + 1] - offsets[i], out + i * HBH_G2_BYTES);
  });
  return HBH_OK;
}

int hbh_hash_g1_g2(size_t n, const uint8_t* u, const uint8_t* data, const size_t* offsets, uint8_t* out,
                   int threads) {
  if (n == 0) return HBH_OK;
  if (!u || !offsets || !out || (!data && offsets[n] != 0)) return host_fail(HBH_ERR_ARG, "null pointer");
  for (size_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i]) return host_fail(HBH_ERR_ARG, "offsets not ascending");
  hh::parallel_for(n, threads, [&](size_t i) {
    hh::hash_g1_g2(u + i * HBH_G1_BYTES, data + offsets[i], offsets[i + 1] - offsets[i], out + i * HBH_G2_BYTES);
  });
  return HBH_OK;
}

int hbh_hash_g1_g2_bp(size_t n, const uint8_t* u, const uint8_t* data, const size_t* offsets, uint8_t* out,
                      int threads) {
  if (n == 0) return HBH_OK;
  if (!u || !offsets || !out || (!data && offsets[n] != 0)) return host_fail(HBH_ERR_ARG, "null pointer");
  for (size_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i]) return host_fail(HBH_ERR_ARG, "offsets not ascending");
  hh::parallel_for(n, threads, [&](size_t i) {
    const std::vector<uint8_t> m = hh::g1_g2_msg(u + i * HBH_G1_BYTES, data + offsets[i], offsets[i + 1] - offsets[i]);
    hh::g2_to_abi(hh::hash_g2_bp(m.data(), m.size()), out + i * HBH_G2_BYTES);
  });
  return HBH_OK;
}

int hbh_hash_bp_g1(uint8_t* out) {
  if (!out) return host_fail(HBH_ERR_ARG, "null pointer");
  // [KCOF^-1 mod r] g1 = [KCOF^(r-2)] g1: exponentiation in Fr by square-and-multiply on fr_mul
  static const uint64_t RM2[4] = {0xfffffffeffffffffull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                                  0x73eda753299d7d48ull};
  uint64_t acc[4] = {1, 0, 0, 0};
  for (int b = 254; b >= 0; b--) {
    uint64_t t[4];
    hh::fr_mul(acc, acc, t);
    memcpy(acc, t, 32);
    if ((RM2[b >> 6] >> (b & 63)) & 1) {
      hh::fr_mul(acc, hh::KCOF, t);
      memcpy(acc, t, 32);
    }
  }
  hh::g1_to_abi(hh::g1_mul_gen(acc), out);
  return HBH_OK;
}

int hbh_xor_with_hash(size_t n, const uint8_t* g, const uint8_t* data, const size_t* offsets, uint8_t* out,
                      int threads) {
  if (n == 0) return HBH_OK;
  if (!g || !offsets || (offsets[n] && (!data || !out))) return host_fail(HBH_ERR_ARG, "null pointer");
  for (size_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i]) return host_fail(HBH_ERR_ARG, "offsets not ascending");
  hh::parallel_for(n, threads, [&](size_t i) {
    hh::xor_with_hash(g + i * HBH_G1_BYTES, data + offsets[i], offsets[i + 1] - offsets[i], out + offsets[i]);
  });
  return HBH_OK;
}

int hbh_host_threads(int* out) {
  if (!out) return host_fail(HBH_ERR_ARG, "null pointer");
  *out = (int)hh::usable_cpus();
  return HBH_OK;
}

int hbh_signature_parity(size_t n, const uint8_t* sigs, uint8_t* out) {
  if (n == 0) return HBH_OK;
  if (!sigs || !out) return host_fail(HBH_ERR_ARG, "null pointer");
  for (size_t i = 0; i < n; i++) {
    uint8_t u[192];
    hh::g2_uncompressed(sigs + i * HBH_G2_BYTES, u);
    uint8_t x = 0;
    for (int k = 0; k < 192; k++) x ^= u[k];
    out[i] = (uint8_t)(__builtin_popcount(x) & 1);
  }
  return HBH_OK;
}

int hbh_g1_compress(size_t n, const uint8_t* pts, uint8_t* out) {
  if (n && (!pts || !out)) return host_fail(HBH_ERR_ARG, "null pointer");
  for (size_t i = 0; i < n; i++)
    if (!hh::g1_compress(pts + i * HBH_G1_BYTES, out + i * 48)) return host_fail(HBH_ERR_ARG, "coordinate >= p");
  return HBH_OK;
}

int hbh_g2_compress(size_t n, const uint8_t* pts, uint8_t* out) {
  if (n && (!pts || !out)) return host_fail(HBH_ERR_ARG, "null pointer");
  for (size_t i = 0; i < n; i++)
    if (!hh::g2_compress(pts + i * HBH_G2_BYTES, out + i * 96)) return host_fail(HBH_ERR_ARG, "coordinate >= p");
  return HBH_OK;
}

int hbh_host_g1_mul(size_t n, const uint8_t* pts, const uint8_t* scalars, uint8_t* out, int threads) {
  if (n == 0) return HBH_OK;
  if (!pts || !scalars || !out) return host_fail(HBH_ERR_ARG, "null pointer");
  std::atomic<int> bad(0);
  hh::parallel_for(n, threads, [&](size_t i) {
    hh::Jac<hh::Fq> p;
    if (!hh::g1_from_abi(pts + i * HBH_G1_BYTES, p)) {
      bad = 1;
      return;
    }
    uint64_t k[4];
    scalar_limbs(scalars + i * 32, k);
    hh::g1_to_abi(hh::g1_mul_glv(p, k), out + i * HBH_G1_BYTES);
  });
  return bad ? host_fail(HBH_ERR_ARG, "coordinate >= p") : HBH_OK;
}

int hbh_host_g2_mul(size_t n, const uint8_t* pts, const uint8_t* scalars, uint8_t* out, int threads) {
  if (n == 0) return HBH_OK;
  if (!pts || !scalars || !out) return host_fail(HBH_ERR_ARG, "null pointer");
  std::atomic<int> bad(0);
  hh::parallel_for(n, threads, [&](size_t i) {
    hh::Jac<hh::Fq2> p;
    if (!hh::g2_from_abi(pts + i * HBH_G2_BYTES, p)) {
      bad = 1;
      return;
    }
    uint64_t k[4];
    scalar_limbs(scalars + i * 32, k);
    hh::g2_to_abi(hh::g2_mul_gls(p, k), out + i * HBH_G2_BYTES);
  });
  return bad ? host_fail(HBH_ERR_ARG, "coordinate >= p") : HBH_OK;
}

int hbh_host_g1_add(size_t n, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  if (n == 0) return HBH_OK;
  if (!a || !b || !out) return host_fail(HBH_ERR_ARG, "null pointer");
  for (size_t i = 0; i < n; i++) {
    hh::Jac<hh::Fq> p, q;
    if (!hh::g1_from_abi(a + i * HBH_G1_BYTES, p) || !hh::g1_from_abi(b + i * HBH_G1_BYTES, q))
      return host_fail(HBH_ERR_ARG, "coordinate >= p");
    hh::g1_to_abi(hh::jac_add(p, q), out + i * HBH_G1_BYTES);
  }
  return HBH_OK;
}

int hbh_encrypt(size_t n, const uint8_t* pks, int pk_per_item, const uint8_t* data, const size_t* offsets,
                const uint8_t* nonces, uint8_t* u_out, uint8_t* v_out, uint8_t* w_out, int threads) {
  if (n == 0) return HBH_OK;
  if (!pks || !offsets || !nonces || !u_out || !w_out || (offsets[n] && (!data || !v_out)))
    return host_fail(HBH_ERR_ARG, "null pointer");
  for (size_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i]) return host_fail(HBH_ERR_ARG, "offsets not ascending");
  hh::g1_comb();  // build the fixed-base table before the workers share it
  // keys: one, or one per item; a key that encrypts at least COMB_MIN items of this call gets a comb
  const size_t COMB_MIN = 16;
  std::vector<uint32_t> key_of(n, 0);
  std::vector<const uint8_t*> keys;
  if (pk_per_item) {
    std::unordered_map<std::string, uint32_t> seen;
    for (size_t i = 0; i < n; i++) {
      const uint8_t* k = pks + i * HBH_G1_BYTES;
      auto it = seen.emplace(std::string((const char*)k, HBH_G1_BYTES), (uint32_t)keys.size());
      if (it.second) keys.push_back(k);
      key_of[i] = it.first->second;
    }
  } else {
    keys.push_back(pks);
  }
  std::vector<size_t> uses(keys.size(), 0);
  for (size_t i = 0; i < n; i++) uses[key_of[i]]++;
  std::vector<hh::Jac<hh::Fq>> key_pt(keys.size());
  std::vector<std::vector<hh::Aff<hh::Fq>>> combs(keys.size());
  std::atomic<int> bad(0);
  hh::parallel_for(keys.size(), threads, [&](size_t j) {
    if (!hh::g1_from_abi(keys[j], key_pt[j])) {
      bad = 1;
      return;
    }
    if (uses[j] >= COMB_MIN) combs[j] = hh::comb4_build(key_pt[j]);
  });
  if (bad) return host_fail(HBH_ERR_ARG, "coordinate >= p");
  hh::parallel_for(n, threads, [&](size_t i) {
    const uint32_t kj = key_of[i];
    uint64_t r[4];
    scalar_limbs(nonces + i * 32, r);
    hh::reduce_r(r);
    // U = g1 r (g1's comb) and pk r (the key's comb, or GLV), made affine with one inversion
    const hh::Jac<hh::Fq> jp[2] = {hh::g1_mul_gen(r),
                                   combs[kj].empty() ? hh::g1_mul_glv(key_pt[kj], r) : hh::comb4_mul(combs[kj], r)};
    hh::Aff<hh::Fq> ap[2];
    hh::jac_batch_affine(jp, ap, 2);
    uint8_t* u = u_out + i * HBH_G1_BYTES;
    hh::g1_aff_to_abi(ap[0], u);
    uint8_t g[HBH_G1_BYTES];
    hh::g1_aff_to_abi(ap[1], g);
    const size_t len = offsets[i + 1] - offsets[i];
    hh::xor_with_hash(g, data + offsets[i], len, v_out + offsets[i]);  // V = msg xor stream
    // W = hash_g1_g2(U, V) r = [KCOF] Q_bp r = [KCOF r mod r] Q_bp: one GLS multiplication
    const std::vector<uint8_t> m = hh::g1_g2_msg(u, v_out + offsets[i], len);
    uint64_t kr[4];
    hh::fr_mul(hh::KCOF, r, kr);
    hh::g2_to_abi(hh::g2_mul_gls(hh::hash_g2_bp(m.data(), m.size()), kr), w_out + i * HBH_G2_BYTES);
  });
  return bad ? host_fail(HBH_ERR_ARG, "coordinate >= p") : HBH_OK;
}

int hbh_fr_poly_eval(size_t npoly, size_t ncoef, const uint8_t* coeffs, size_t npts, const uint64_t* xs, uint8_t* out,
                     int threads) {
  if (npoly == 0 || npts == 0) return HBH_OK;
  if (!xs || !out || (ncoef && !coeffs)) return host_fail(HBH_ERR_ARG, "null pointer");
  std::atomic<int> bad(0);
  // Horner in the Montgomery domain (R = 2^256): x_k and the coefficients enter as a R, the result
  // leaves through one product by 1
  hh::parallel_for(npoly, threads, [&](size_t q) {
    std::vector<uint64_t> c(4 * ncoef);
    for (size_t j = 0; j < ncoef; j++) {
      uint64_t v[4];
      scalar_limbs(coeffs + (q * ncoef + j) * 32, v);
      if (hh::geq_r(v)) bad = 1;
      hh::fr_to_mont(v, &c[4 * j]);
    }
    for (size_t k = 0; k < npts; k++) {
      uint64_t x[4] = {xs[k], 0, 0, 0}, xm[4], acc[4] = {0, 0, 0, 0};
      hh::reduce_r(x);
      hh::fr_to_mont(x, xm);
      for (size_t j = ncoef; j-- > 0;) {
        uint64_t t[4];
        hh::fr_mont(acc, xm, t);
        hh::fr_add(t, &c[4 * j], acc);
      }
      uint64_t one[4] = {1, 0, 0, 0}, res[4];
      hh::fr_mont(acc, one, res);
      memcpy(out + (q * npts + k) * 32, res, 32);
    }
  });
  return bad ? host_fail(HBH_ERR_ARG, "coefficient >= r") : HBH_OK;
}

}  // extern "C"

// Not part of the public ABI (engine.hip's split master check of hbh_combine_verify_g2): neg_out = -pk
// for the ABI point pk (infinity stays all-zero).
extern "C" int hbh__host_g1_neg(const uint8_t* pk, uint8_t* neg_out) {
  hh::Jac<hh::Fq> p;
  if (!hh::g1_from_abi(pk, p)) return host_fail(HBH_ERR_ARG, "coordinate >= p");
  hh::g1_to_abi(hh::jac_neg(p), neg_out);
  return HBH_OK;
}
