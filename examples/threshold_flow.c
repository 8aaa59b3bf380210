/* threshold_flow.c -- the ThresholdSign and ThresholdDecrypt flows of one hbbft network driven
 * through the C ABI alone (include/hbbft_hip.h): no Python, no torch -- what a Rust `extern "C"`
 * binding would call.  It restates tests/threshold_sign.rs's scenario (N = 10,
 * f = 3: key set from a degree-3 polynomial, every node signs the document, shares verified, the
 * first t + 1 valid ones combined and checked against the master key) and a ThresholdDecrypt round
 * (src/threshold_decrypt.rs: Ciphertext::verify, verify_decryption_share, decrypt), with one
 * forged share of each kind that must be rejected.
 *
 *   gcc -O2 -I include examples/threshold_flow.c -L hbbft_amd -lhbbft_hip \
 *       -Wl,-rpath,$PWD/hbbft_amd -o threshold_flow && ./threshold_flow [seed]
 *
 * Exit status 0 and a final "threshold_flow OK" line when every check holds.  Key material is
 * derived from the seed with SplitMix64 (synthetic keys, as the benches use). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hbbft_hip.h"

#define N 10
#define T 3 /* f = 3: t = f, t + 1 = 4 shares combine */
#define G1B HBH_G1_BYTES
#define G2B HBH_G2_BYTES

static int failures = 0;
#define CHECK(cond, ...)                      \
  do {                                        \
    if (!(cond)) {                            \
      fprintf(stderr, "FAIL: " __VA_ARGS__);  \
      fprintf(stderr, "\n");                  \
      failures++;                             \
    }                                         \
  } while (0)
#define OK(call)                                                                    \
  do {                                                                              \
    int st_ = (call);                                                               \
    if (st_ != HBH_OK) {                                                            \
      fprintf(stderr, "%s -> %d (%s / %s)\n", #call, st_, hbh_last_error(),         \
              hbh_host_last_error());                                               \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)

/* ---------------------------------------------------------------- Fr (mod r), enough for Horner
 * with small x: values are 4 x 64-bit little-endian limbs < r */
static const uint64_t R_MOD[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                                  0x73eda753299d7d48ull};
typedef struct { uint64_t w[5]; } fr; /* w[4]: overflow limb during reduction */

static int fr_geq_r(const fr* a) {
  if (a->w[4]) return 1;
  for (int i = 3; i >= 0; i--) {
    if (a->w[i] != R_MOD[i]) return a->w[i] > R_MOD[i];
  }
  return 1;
}
static void fr_sub_r(fr* a) {
  unsigned __int128 borrow = 0;
  for (int i = 0; i < 5; i++) {
    const unsigned __int128 s = (unsigned __int128)(i < 4 ? R_MOD[i] : 0) + borrow;
    borrow = (unsigned __int128)a->w[i] < s;
    a->w[i] = (uint64_t)((unsigned __int128)a->w[i] - s);
  }
}
static void fr_reduce(fr* a) {
  while (fr_geq_r(a)) fr_sub_r(a);
}
/* a = a * x + c, x < 2^16 */
static void fr_mul_small_add(fr* a, uint32_t x, const fr* c) {
  unsigned __int128 carry = 0;
  for (int i = 0; i < 5; i++) {
    const unsigned __int128 v = (unsigned __int128)a->w[i] * x + carry + (i < 5 ? c->w[i] : 0);
    a->w[i] = (uint64_t)v;
    carry = v >> 64;
  }
  fr_reduce(a);
}
static void fr_bytes(const fr* a, uint8_t out[32]) {
  for (int i = 0; i < 32; i++) out[i] = (uint8_t)(a->w[i / 8] >> (8 * (i % 8)));
}

static uint64_t sm_state;
static uint64_t splitmix64(void) {
  uint64_t z = (sm_state += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
static fr fr_random(void) {
  fr a;
  memset(&a, 0, sizeof a);
  for (int i = 0; i < 4; i++) a.w[i] = splitmix64();
  a.w[3] &= 0x3fffffffffffffffull; /* < 2^254 < r */
  return a;
}

int main(int argc, char** argv) {
  sm_state = argc > 1 ? strtoull(argv[1], NULL, 10) : 7;
  int ndev = 0;
  OK(hbh_device_count(&ndev));
  if (ndev < 1) {
    fprintf(stderr, "no HIP device\n");
    return 3;
  }
  hbh_engine* eng = NULL;
  OK(hbh_engine_create(0, &eng));

  /* ---- key set: master polynomial c_0..c_T, sk_i = poly(i + 1) (SecretKeySet::secret_key_share) */
  fr coef[T + 1];
  for (int j = 0; j <= T; j++) coef[j] = fr_random();
  uint8_t sk[N][32], coef_b[T + 1][32], msk[32];
  for (int i = 0; i < N; i++) {
    fr acc;
    memset(&acc, 0, sizeof acc);
    for (int j = T; j >= 0; j--) fr_mul_small_add(&acc, (uint32_t)(i + 1), &coef[j]);
    fr_bytes(&acc, sk[i]);
  }
  for (int j = 0; j <= T; j++) fr_bytes(&coef[j], coef_b[j]);
  memcpy(msk, coef_b[0], 32);

  /* public side: commitment g1 * c_j, pk_i = commitment(i + 1) (NetworkInfo::new), mpk = g1 * c_0;
   * cross-checked against g1 * sk_i on the fixed-base path */
  uint8_t commit[T + 1][G1B], pk[N][G1B], pk_direct[N][G1B], g1[G1B];
  uint8_t one[32] = {1};
  OK(hbh_g1_mul_gen(eng, 1, one, g1));
  OK(hbh_g1_mul_gen(eng, T + 1, &coef_b[0][0], &commit[0][0]));
  uint32_t cidx[N], xs[N];
  for (int i = 0; i < N; i++) {
    cidx[i] = 0;
    xs[i] = (uint32_t)(i + 1);
  }
  OK(hbh_commitment_eval(eng, N, T, 1, &commit[0][0], cidx, xs, &pk[0][0]));
  OK(hbh_g1_mul_gen(eng, N, &sk[0][0], &pk_direct[0][0]));
  CHECK(memcmp(pk, pk_direct, sizeof pk) == 0, "public key shares: commitment evaluation != g1 * sk_i");
  const uint8_t* mpk = commit[0];

  /* ---- ThresholdSign: H = hash_g2(doc), sigma_i = H * sk_i on the host (secret keys never reach
   * the GPU), node 2's share replaced by its share of another document */
  const char* doc = "Hello, world!";
  const char* other = "Goodbye";
  size_t offs[2] = {0, strlen(doc)}, offs2[2] = {0, strlen(other)};
  uint8_t H[G2B], H2[G2B], sig[N][G2B], forged[G2B];
  OK(hbh_hash_g2(1, (const uint8_t*)doc, offs, H, 0));
  OK(hbh_hash_g2(1, (const uint8_t*)other, offs2, H2, 0));
  for (int i = 0; i < N; i++) OK(hbh_host_g2_mul(1, H, sk[i], sig[i], 0));
  OK(hbh_host_g2_mul(1, H2, sk[2], forged, 0));
  memcpy(sig[2], forged, G2B);

  uint32_t doc_idx[N] = {0};
  uint8_t verdict[N];
  OK(hbh_verify_sig_shares(eng, N, &pk[0][0], &sig[0][0], H, 1, doc_idx, verdict));
  for (int i = 0; i < N; i++) CHECK(verdict[i] == (i != 2), "share %d verdict %d", i, verdict[i]);

  /* combine the first t + 1 valid shares in node order (BTreeMap order), verify against mpk */
  uint32_t idx[T + 1];
  uint8_t shares[T + 1][G2B];
  int k = 0;
  for (int i = 0; i < N && k <= T; i++) {
    if (!verdict[i]) continue;
    idx[k] = (uint32_t)i;
    memcpy(shares[k], sig[i], G2B);
    k++;
  }
  uint8_t combined[G2B], want[G2B], ok_sig;
  int status;
  OK(hbh_combine_verify_g2(eng, 1, T, idx, &shares[0][0], mpk, H, combined, &status, &ok_sig));
  OK(hbh_host_g2_mul(1, H, msk, want, 0));
  CHECK(status == HBH_OK && ok_sig == 1, "combine status %d verdict %d", status, ok_sig);
  CHECK(memcmp(combined, want, G2B) == 0, "combined signature != msk * H");
  uint8_t parity;
  OK(hbh_signature_parity(1, combined, &parity));
  /* a duplicate index is threshold_crypto's DuplicateEntry */
  uint32_t dup[T + 1];
  memcpy(dup, idx, sizeof dup);
  dup[1] = dup[0];
  OK(hbh_combine_verify_g2(eng, 1, T, dup, &shares[0][0], mpk, H, combined, &status, &ok_sig));
  CHECK(status == HBH_ERR_DUPLICATE_ENTRY, "duplicate index status %d", status);

  /* ---- ThresholdDecrypt: encrypt to mpk, Ciphertext::verify, D_i = U * sk_i, share checks,
   * interpolation at 0, xor_with_hash -> the plaintext */
  const char* msg = "threshold decryption through the C ABI";
  const size_t mlen = strlen(msg);
  size_t moffs[2] = {0, mlen};
  uint8_t U[G1B], V[64], W[G2B], nonce[32], huv[G2B];
  fr nr = fr_random();
  fr_bytes(&nr, nonce);
  OK(hbh_encrypt(1, mpk, 0, (const uint8_t*)msg, moffs, nonce, U, V, W, 0));
  OK(hbh_hash_g1_g2(1, U, V, moffs, huv, 0));
  uint8_t ct_ok;
  OK(hbh_verify_ciphertexts(eng, 1, U, W, huv, &ct_ok));
  CHECK(ct_ok == 1, "Ciphertext::verify rejected a fresh ciphertext");
  uint8_t W_bad[G2B];
  memcpy(W_bad, H, G2B); /* W of the wrong point */
  OK(hbh_verify_ciphertexts(eng, 1, U, W_bad, huv, &ct_ok));
  CHECK(ct_ok == 0, "Ciphertext::verify accepted a tampered W");

  uint8_t dshare[N][G1B];
  for (int i = 0; i < N; i++) OK(hbh_host_g1_mul(1, U, sk[i], dshare[i], 0));
  memcpy(dshare[5], pk[5], G1B); /* node 5 sends a garbage share */
  uint32_t ct_idx[N] = {0};
  OK(hbh_verify_dec_shares(eng, N, &dshare[0][0], &pk[0][0], huv, W, 1, ct_idx, verdict));
  for (int i = 0; i < N; i++) CHECK(verdict[i] == (i != 5), "decryption share %d verdict %d", i, verdict[i]);
  uint8_t dpts[T + 1][G1B], g[G1B], plain[64];
  k = 0;
  for (int i = 0; i < N && k <= T; i++) {
    if (!verdict[i]) continue;
    idx[k] = (uint32_t)i;
    memcpy(dpts[k], dshare[i], G1B);
    k++;
  }
  OK(hbh_interpolate_g1(eng, 1, T, idx, &dpts[0][0], g, &status));
  CHECK(status == HBH_OK, "interpolate_g1 status %d", status);
  OK(hbh_xor_with_hash(1, g, V, moffs, plain, 0));
  CHECK(memcmp(plain, msg, mlen) == 0, "decrypted plaintext differs");

  OK(hbh_engine_destroy(eng));
  if (failures) {
    fprintf(stderr, "threshold_flow: %d check(s) failed\n", failures);
    return 1;
  }
  printf("signature parity %d\nthreshold_flow OK\n", parity);
  return 0;
}
