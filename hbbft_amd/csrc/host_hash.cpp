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
#include <vector>

#include "../../include/hbbft_hip.h"
#include "host_bls.hpp"

namespace hh {

// ---------------------------------------------------------------- constants
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

bool f2_sqrt(const Fq2& a, Fq2& out) {
  if (f2_is_zero(a)) {
    out = a;
    return true;
  }
  const Consts& k = consts();
  const Fq2 a1 = f2_pow(a, k.pm3d4, 6);
  const Fq2 alpha = f2_mul(f2_sqr(a1), a);
  const Fq2 a0 = f2_mul(f2_conj(alpha), alpha);  // alpha^p alpha
  const Fq2 minus_one = {fq_neg(fq_one()), fq_zero()};
  if (f2_eq(a0, minus_one)) return false;
  const Fq2 x0 = f2_mul(a1, a);
  Fq2 r;
  if (f2_eq(alpha, minus_one)) {
    r = {fq_neg(x0.c1), x0.c0};  // x0 * u
  } else {
    r = f2_mul(f2_pow(f2_add(f2_one(), alpha), k.pm1d2, 6), x0);
  }
  if (!f2_eq(f2_sqr(r), a)) return false;
  out = r;
  return true;
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

// ---------------------------------------------------------------- hash to G2
static const uint64_t H2_LIMBS[8] = {0xcf1c38e31c7238e5ull, 0x1616ec6e786f0c70ull, 0x21537e293a6691aeull,
                                     0xa628f1cb4d9e82efull, 0xa68a205b2e5a7ddfull, 0xcd91de4547085abaull,
                                     0x091d50792876a202ull, 0x05d543a95414e7f1ull};

static Jac<Fq2> g2_rand(ChaChaRng& rng) {
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
    const Jac<Fq2> p = jac_mul(Jac<Fq2>{x, y, f2_one()}, H2_LIMBS, 8);
    if (!f2_is_zero(p.z)) return p;
  }
}

static void hash_g2(const uint8_t* msg, size_t len, uint8_t* out) {
  uint8_t seed[32];
  sha3_256(msg, len, seed);
  ChaChaRng rng(seed);
  g2_to_abi(g2_rand(rng), out);
}

static void hash_g1_g2(const uint8_t* u_abi, const uint8_t* v, size_t vlen, uint8_t* out) {
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
    hh::g1_to_abi(hh::jac_mul(p, k, 4), out + i * HBH_G1_BYTES);
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
    hh::g2_to_abi(hh::jac_mul(p, k, 4), out + i * HBH_G2_BYTES);
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
  static const uint64_t G1_CANON[12] = {0xfb3af00adb22c6bbull, 0x6c55e83ff97a1aefull, 0xa14e3a3f171bac58ull,
                                        0xc3688c4f9774b905ull, 0x2695638c4fa9ac0full, 0x17f1d3a73197d794ull,
                                        0x0caa232946c5e7e1ull, 0xd03cc744a2888ae4ull, 0x00db18cb2c04b3edull,
                                        0xfcf5e095d5d00af6ull, 0xa09e30ed741d8ae4ull, 0x08b3f481e3aaa0f1ull};
  const hh::Jac<hh::Fq> g1 = {hh::fq_from_canon(G1_CANON), hh::fq_from_canon(G1_CANON + 6), hh::fq_one()};
  std::atomic<int> bad(0);
  hh::parallel_for(n, threads, [&](size_t i) {
    hh::Jac<hh::Fq> pk;
    if (!hh::g1_from_abi(pks + (pk_per_item ? i : 0) * HBH_G1_BYTES, pk)) {
      bad = 1;
      return;
    }
    uint64_t r[4];
    scalar_limbs(nonces + i * 32, r);
    uint8_t* u = u_out + i * HBH_G1_BYTES;
    hh::g1_to_abi(hh::jac_mul(g1, r, 4), u);  // U = g1 r
    uint8_t g[HBH_G1_BYTES];
    hh::g1_to_abi(hh::jac_mul(pk, r, 4), g);  // pk r
    const size_t len = offsets[i + 1] - offsets[i];
    hh::xor_with_hash(g, data + offsets[i], len, v_out + offsets[i]);  // V = msg xor stream
    uint8_t h[HBH_G2_BYTES];
    hh::hash_g1_g2(u, v_out + offsets[i], len, h);
    hh::Jac<hh::Fq2> hp;
    hh::g2_from_abi(h, hp);
    hh::g2_to_abi(hh::jac_mul(hp, r, 4), w_out + i * HBH_G2_BYTES);  // W = hash_g1_g2(U, V) r
  });
  return bad ? host_fail(HBH_ERR_ARG, "coordinate >= p") : HBH_OK;
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
