// Host-side BLS12-381 arithmetic for the parts of the path that stay on the CPU (north star:
// hashing to G2, transcript parsing and secret-key operations stay on the host): hash_g2 /
// hash_g1_g2 (ThresholdSign::set_document, Ciphertext checks), xor_with_hash, Signature::parity,
// the secret scalar multiplications sign_g2 / decrypt_share / encrypt_with_rng, and the point
// encodings.  Fq is 6 x 64-bit limbs in Montgomery form (R = 2^384), as pairing 0.14's Fq, so
// ff 0.4's Fq::rand (limbs read AS the Montgomery representation) is reproduced directly.
#pragma once
#include <stdint.h>
#include <string.h>

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
inline Fq fq_add(const Fq& a, const Fq& b) {
  Fq r;
  uint64_t c = 0;
  for (int i = 0; i < 6; i++) {
    const u128 s = (u128)a.l[i] + b.l[i] + c;
    r.l[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (c || geq_p(r.l)) sub_p(r.l);
  return r;
}
inline Fq fq_sub(const Fq& a, const Fq& b) {
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
inline Fq fq_neg(const Fq& a) { return fq_is_zero(a) ? a : fq_sub(fq_zero(), a); }

// CIOS Montgomery product
inline Fq fq_mul(const Fq& a, const Fq& b) {
  uint64_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 6; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 6; j++) {
      const u128 s = (u128)a.l[j] * b.l[i] + t[j] + c;
      t[j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[6] + c;
    t[6] = (uint64_t)s;
    t[7] = (uint64_t)(s >> 64);
    const uint64_t m = t[0] * PINV;
    s = (u128)m * P[0] + t[0];
    c = (uint64_t)(s >> 64);
    for (int j = 1; j < 6; j++) {
      s = (u128)m * P[j] + t[j] + c;
      t[j - 1] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    s = (u128)t[6] + c;
    t[5] = (uint64_t)s;
    t[6] = t[7] + (uint64_t)(s >> 64);
  }
  Fq r;
  memcpy(r.l, t, sizeof(r.l));
  if (t[6] || geq_p(r.l)) sub_p(r.l);
  return r;
}
inline Fq fq_sqr(const Fq& a) { return fq_mul(a, a); }

struct Consts {
  Fq one;     // R mod p
  Fq r2;      // R^2 mod p
  Fq b1;      // 4 (G1 curve constant), Montgomery
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
inline Fq fq_pow(const Fq& a, const uint64_t* e, int nlimbs) {
  Fq r = fq_one();
  bool started = false;
  for (int i = nlimbs * 64 - 1; i >= 0; i--) {
    if (started) r = fq_sqr(r);
    if ((e[i / 64] >> (i % 64)) & 1) {
      r = started ? fq_mul(r, a) : a;
      started = true;
    }
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
inline bool f2_is_zero(const Fq2& a) { return fq_is_zero(a.c0) && fq_is_zero(a.c1); }
inline bool f2_eq(const Fq2& a, const Fq2& b) { return fq_eq(a.c0, b.c0) && fq_eq(a.c1, b.c1); }
inline Fq2 f2_zero() { return {fq_zero(), fq_zero()}; }
inline Fq2 f2_one() { return {fq_one(), fq_zero()}; }
inline Fq2 f2_pow(const Fq2& a, const uint64_t* e, int nlimbs) {
  Fq2 r = f2_one();
  bool started = false;
  for (int i = nlimbs * 64 - 1; i >= 0; i--) {
    if (started) r = f2_sqr(r);
    if ((e[i / 64] >> (i % 64)) & 1) {
      r = started ? f2_mul(r, a) : a;
      started = true;
    }
  }
  return r;
}
inline Fq2 f2_inv(const Fq2& a) {
  const Fq t = fq_inv(fq_add(fq_sqr(a.c0), fq_sqr(a.c1)));
  return {fq_mul(a.c0, t), fq_neg(fq_mul(a.c1, t))};
}
// pairing 0.14 Ord for Fq2: c1 first, then c0 (canonical integers)
inline bool f2_gt(const Fq2& a, const Fq2& b) {
  if (!fq_eq(a.c1, b.c1)) return fq_gt(a.c1, b.c1);
  return fq_gt(a.c0, b.c0);
}
// square root for p = 3 mod 4 (Adj / Rodriguez-Henriquez Alg. 9); false if a is not a square
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
};

// Jacobian point over F (y^2 = x^3 + b, a = 0); z = 0 is the point at infinity
template <class F>
struct Jac {
  F x, y, z;
};
template <class F>
inline Jac<F> jac_inf() {
  return {Ops<F>::one(), Ops<F>::one(), Ops<F>::zero_v()};
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
template <class F>
inline Jac<F> jac_neg(const Jac<F>& p) {
  Jac<F> r = p;
  r.y = Ops<F>::sub(Ops<F>::zero_v(), p.y);
  return r;
}
// k * P for a little-endian multi-limb scalar, 4-bit fixed window
template <class F>
inline Jac<F> jac_mul(const Jac<F>& p, const uint64_t* k, int nlimbs) {
  Jac<F> tab[16];
  tab[0] = jac_inf<F>();
  tab[1] = p;
  for (int i = 2; i < 16; i++) tab[i] = (i & 1) ? jac_add(tab[i - 1], p) : jac_dbl(tab[i / 2]);
  Jac<F> r = jac_inf<F>();
  for (int w = nlimbs * 16 - 1; w >= 0; w--) {
    for (int d = 0; d < 4; d++) r = jac_dbl(r);
    const int nib = (int)((k[w / 16] >> (4 * (w % 16))) & 15);
    if (nib) r = jac_add(r, tab[nib]);
  }
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

// ---------------------------------------------------------------- ABI encodings (include/hbbft_hip.h)
// G1 = x || y (48-byte LE canonical each), G2 = x.c0 || x.c1 || y.c0 || y.c1; infinity = all zero
void g1_to_abi(const Jac<Fq>& p, uint8_t* out);
void g2_to_abi(const Jac<Fq2>& p, uint8_t* out);
bool g1_from_abi(const uint8_t* in, Jac<Fq>& p);  // false: a coordinate >= p
bool g2_from_abi(const uint8_t* in, Jac<Fq2>& p);

}  // namespace hh
