/* hbbft_hip.h -- C ABI of the MI355X batch engine for hbbft's BLS12-381 threshold-crypto hot path.
 *
 * This is the drop-in boundary.  hbbft itself never calls curve arithmetic: its
 * three protocol modules call `threshold_crypto` 0.3 methods synchronously, one share at a time.
 * Each entry point below is the batched replacement for one of those calls; a Rust binding
 *  drains the shares a `Step` would verify into one call.
 *
 * Conventions
 *  - Plain pointers + sizes, caller-owned buffers, nothing retained after return.
 *  - Points are affine, canonical (non-Montgomery) little-endian integers:
 *      G1 = x(48 B) || y(48 B)                         (HBH_G1_BYTES = 96)
 *      G2 = x.c0 || x.c1 || y.c0 || y.c1 (48 B each)   (HBH_G2_BYTES = 192)
 *    The point at infinity is all-zero bytes.  Points must be on the curve and in the prime-order
 *    subgroup, as threshold_crypto's deserialisation guarantees for every point that reaches the
 *    reference's verify calls; the engine does not re-check membership.
 *  - Scalars (Fr) are 32-byte little-endian canonical integers.
 *  - Verdicts are one byte per item (1 = valid, 0 = invalid), never an error: an invalid share is
 *    a Fault in hbbft, not an Err (src/threshold_sign.rs:191-194, src/threshold_decrypt.rs:192-195).
 *  - Every function returns an hbh_status; HBH_OK = 0.
 *  - `_dev` variants take device pointers (HBM-resident inputs) and an optional hipStream_t
 *    (passed as void*, NULL = the engine's stream); they are asynchronous on that stream.
 *  - One engine handle binds one GPU.  Calls on one handle are serialised by the handle's mutex;
 *    distinct handles may be used from distinct threads.
 */
#ifndef HBBFT_HIP_H
#define HBBFT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HBH_G1_BYTES 96
#define HBH_G2_BYTES 192
#define HBH_FR_BYTES 32

typedef enum {
  HBH_OK = 0,
  HBH_ERR_ARG = 1,       /* null pointer / size out of range / index out of range */
  HBH_ERR_DEVICE = 2,    /* HIP runtime error (message via hbh_last_error) */
  HBH_ERR_NOMEM = 3,     /* device allocation failed */
  HBH_ERR_NOT_ENOUGH_SHARES = 4,  /* threshold_crypto Error::NotEnoughShares */
  HBH_ERR_DUPLICATE_ENTRY = 5     /* threshold_crypto Error::DuplicateEntry */
} hbh_status;

typedef struct hbh_engine hbh_engine;

/* Engine lifetime.  `device` is a HIP device ordinal. */
int hbh_engine_create(int device, hbh_engine** out);
int hbh_engine_destroy(hbh_engine* eng);
/* Last error message of this thread (static storage, never NULL). */
const char* hbh_last_error(void);
/* Number of HIP devices visible to this process. */
int hbh_device_count(int* out);

/* ---------------------------------------------------------------- device-resident variants
 * Same results as the host-pointer calls, with every array in device memory (HBM) and the call
 * asynchronous on `stream` (hipStream_t as void*, NULL = engine stream); ordered after the
 * engine's previous call as hbh_verify_pairing_eq_dev.  Index arrays are not inspected on the host.
 *   hbh_interpolate_g*_dev: d_idx node indices (x = idx + 1; an index of 0xffffffff gives status
 *     HBH_ERR_ARG for its combine), d_status written per combine as hbh_interpolate_g*.
 *   hbh_g*_decompress_dev: compressed encodings in HBM, flags parsed on the device.
 *   hbh_bivar_ack_check_dev: the caller supplies the row plan -- nrow distinct (part, x) requests
 *     (d_row_part, d_row_x, part < nparts of d_commits) and d_row_of[a] = the row of ack a -- that
 *     hbh_bivar_ack_check derives on the host; d_vals = 32-byte LE scalars. */
int hbh_interpolate_g1_dev(hbh_engine* eng, void* stream, size_t ncomb, int t, const uint32_t* d_idx,
                           const void* d_pts, void* d_out, int* d_status);
int hbh_interpolate_g2_dev(hbh_engine* eng, void* stream, size_t ncomb, int t, const uint32_t* d_idx,
                           const void* d_pts, void* d_out, int* d_status);
int hbh_g1_decompress_dev(hbh_engine* eng, void* stream, size_t n, const uint8_t* d_in, void* d_out, uint8_t* d_ok);
int hbh_g2_decompress_dev(hbh_engine* eng, void* stream, size_t n, const uint8_t* d_in, void* d_out, uint8_t* d_ok);
int hbh_bivar_ack_check_dev(hbh_engine* eng, void* stream, size_t nack, int t, const void* d_commits, size_t nrow,
                            const uint32_t* d_row_part, const uint32_t* d_row_x, const uint32_t* d_row_of,
                            const uint32_t* d_ys, const void* d_vals, uint8_t* d_verdicts);

/* ---------------------------------------------------------------- engine pool (multi-device)
 * One engine per shard; devices[s] is shard s's device (a device may appear more than once: each
 * shard has its own stream and workspaces).  A pool call splits its batch by INSTANCE (document /
 * ciphertext / combine / SyncKeyGen part) into contiguous instance ranges of about equal item
 * counts, runs every shard on its own host thread, and writes verdicts and points back in the
 * caller's order -- byte-identical to the single-engine call.  No cross-device collective exists
 * on this path.  Errors: the first failing shard's code, with "shard s: ..." in
 * hbh_last_error.  Replaces the reference's single synchronous verifier per node
 * (src/traits.rs:297-336) with a node-wide fan-out over the GPUs of one host. */
typedef struct hbh_pool hbh_pool;
int hbh_pool_create(const int* devices, int nshards, hbh_pool** out);
int hbh_pool_destroy(hbh_pool* pool);
int hbh_pool_shards(const hbh_pool* pool, int* out);
int hbh_pool_engine(hbh_pool* pool, int shard, hbh_engine** out);
int hbh_pool_set_pairing_impl(hbh_pool* pool, int impl);
int hbh_pool_verify_sig_shares(hbh_pool* pool, size_t n, const uint8_t* pks, const uint8_t* sigs,
                               const uint8_t* hashes, size_t ndocs, const uint32_t* doc_idx, uint8_t* verdicts);
int hbh_pool_verify_dec_shares(hbh_pool* pool, size_t n, const uint8_t* shares, const uint8_t* pks,
                               const uint8_t* huv, const uint8_t* w, size_t ncts, const uint32_t* ct_idx,
                               uint8_t* verdicts);
int hbh_pool_combine_verify_g2(hbh_pool* pool, size_t ncomb, int t, const uint32_t* idx, const uint8_t* shares,
                               const uint8_t* master_pk, const uint8_t* hashes, uint8_t* out, int* status,
                               uint8_t* verdicts);
int hbh_pool_interpolate_g1(hbh_pool* pool, size_t ncomb, int t, const uint32_t* idx, const uint8_t* pts,
                            uint8_t* out, int* status);
int hbh_pool_bivar_ack_check(hbh_pool* pool, size_t nack, int t, size_t nparts, const uint8_t* commits,
                             const uint32_t* part_idx, const uint32_t* xs, const uint32_t* ys, const uint8_t* vals,
                             uint8_t* verdicts);

/* ---------------------------------------------------------------- pairing-equality checks
 * Generic batched check  e(P1[i], Q1[q1_idx[i]]) == e(P2[i], Q2[q2_idx[i]])  for i < n,
 * computed as one 2-pair multi-Miller loop + one final exponentiation per item.
 * Q tables hold the G2 points shared by many items (H per document, W / H_uv per ciphertext);
 * q*_idx == NULL means the identity map (table size must then be n).
 * Replaces every pairing comparison on the path:
 *   PublicKeyShare::verify_g2   (src/threshold_sign.rs:223)   P1=pk_i, Q1=H, P2=g1, Q2=sig_i
 *   PublicKey::verify_g2        (src/threshold_sign.rs:264)   P1=pk,   Q1=H, P2=g1, Q2=sig
 *   PublicKey::verify (signed votes / key-gen messages, src/dynamic_honey_badger/votes.rs:157,
 *     dynamic_honey_badger.rs:520)                                P1=pk,   Q1=hash_g2(msg), P2=g1, Q2=sig
 *   Ciphertext::verify          (src/threshold_decrypt.rs:142) P1=g1, Q1=W, P2=U, Q2=H_uv
 *   verify_decryption_share     (src/threshold_decrypt.rs:227) P1=D_i, Q1=H_uv, P2=pk_i, Q2=W
 */
int hbh_verify_pairing_eq(hbh_engine* eng, size_t n,
                          const uint8_t* p1, const uint8_t* q1_table, size_t nq1, const uint32_t* q1_idx,
                          const uint8_t* p2, const uint8_t* q2_table, size_t nq2, const uint32_t* q2_idx,
                          uint8_t* verdicts);

/* PublicKeyShare::verify_g2(share, hash) batched (src/threshold_sign.rs:216-225):
 *   verdict[i] = e(pk[i], hashes[doc_idx[i]]) == e(g1, sigs[i]). */
int hbh_verify_sig_shares(hbh_engine* eng, size_t n, const uint8_t* pks, const uint8_t* sigs,
                          const uint8_t* hashes, size_t ndocs, const uint32_t* doc_idx, uint8_t* verdicts);

/* PublicKeyShare::verify_decryption_share(share, ct) batched (src/threshold_decrypt.rs:220-229):
 *   verdict[i] = e(D[i], huv[ct_idx[i]]) == e(pk[i], w[ct_idx[i]]);
 * huv = hash_g1_g2(U, V) is computed once per ciphertext on the host (the reference recomputes it
 * per check, SURVEY §8a a8 -- the value is identical). */
int hbh_verify_dec_shares(hbh_engine* eng, size_t n, const uint8_t* shares, const uint8_t* pks,
                          const uint8_t* huv, const uint8_t* w, size_t ncts, const uint32_t* ct_idx,
                          uint8_t* verdicts);

/* Ciphertext::verify batched (src/threshold_decrypt.rs:142): verdict[i] = e(g1, w[i]) == e(u[i], huv[i]). */
int hbh_verify_ciphertexts(hbh_engine* eng, size_t n, const uint8_t* u, const uint8_t* w,
                           const uint8_t* huv, uint8_t* verdicts);

/* Device-pointer variant of hbh_verify_pairing_eq (inputs already in HBM).  Asynchronous on
 * `stream` (hipStream_t as void*, NULL = engine stream).  d_p1 / d_p2 == NULL means the G1
 * generator for every item (PublicKeyShare::verify_g2 has P2 = g1, Ciphertext::verify P1 = g1).
 * Calls on different streams are ordered by the engine (each call waits for the previous call's
 * device work before reusing the engine's workspaces).  Index arrays live in device memory and are
 * not inspected on the host: an index >= its table size yields verdict 0 (both implementations). */
int hbh_verify_pairing_eq_dev(hbh_engine* eng, void* stream, size_t n,
                              const void* d_p1, const void* d_q1_table, size_t nq1, const uint32_t* d_q1_idx,
                              const void* d_p2, const void* d_q2_table, size_t nq2, const uint32_t* d_q2_idx,
                              uint8_t* d_verdicts);

/* ---------------------------------------------------------------- combine (interpolate at 0)
 * threshold_crypto interpolate(t, samples) for `ncomb` independent combines of exactly t+1
 * samples each (the first t+1 of the reference's iterator, in its order): out[c] =
 * sum_k lambda_k(0) * P[c][k] with x_k = idx[c][k] + 1.  status[c] = HBH_OK or
 * HBH_ERR_DUPLICATE_ENTRY (two equal indices), as threshold_crypto reports it.  t = 0 returns the
 * single sample.  A caller holding fewer than t+1 shares reports HBH_ERR_NOT_ENOUGH_SHARES itself
 * (the reference checks that before interpolating).
 *   PublicKeySet::combine_signatures (src/threshold_sign.rs:249-259)   -> hbh_interpolate_g2
 *   PublicKeySet::decrypt's G1 interpolation (src/threshold_decrypt.rs:242-250; the XOR with
 *   hash(g) stays on the host)                                         -> hbh_interpolate_g1 */
int hbh_interpolate_g2(hbh_engine* eng, size_t ncomb, int t, const uint32_t* idx, const uint8_t* pts, uint8_t* out,
                       int* status);
int hbh_interpolate_g1(hbh_engine* eng, size_t ncomb, int t, const uint32_t* idx, const uint8_t* pts, uint8_t* out,
                       int* status);

/* ThresholdSign::combine_and_verify_sig (src/threshold_sign.rs:249-270) for `ncomb` documents in
 * one device pass: out[c] = combine_signatures(first t+1 shares) as hbh_interpolate_g2, then
 * verdict[c] = PublicKey::verify_g2(out[c], hashes[c]) = (e(master_pk, H_c) == e(g1, out[c]))
 * (:260-266) without a host round trip in between.  status[c] as hbh_interpolate_g2; verdict[c]
 * = 0 is the reference's Error::VerificationFailed; verdicts of a combine whose status is not
 * HBH_OK are meaningless (the reference returns the combine error first).  A master_pk coordinate
 * >= p is HBH_ERR_ARG.  Calls of at most 540 + 24 t one-pair Miller waves (ncomb x (t + 2); at most
 * 384 combines) evaluate the same verdict as prod_k e(lambda_k g1, share_k) * e(-master_pk, H_c) == 1 on a
 * second stream while the first interpolates ("split master check"; the environment
 * variable HBH_SPLIT_CHECK=0 at engine creation selects interpolate-then-verify for every size;
 * HBH_SPLIT_MAX=<n> replaces the wave-count rule by "at most n combines per call"). */
int hbh_combine_verify_g2(hbh_engine* eng, size_t ncomb, int t, const uint32_t* idx, const uint8_t* shares,
                          const uint8_t* master_pk, const uint8_t* hashes, uint8_t* out, int* status,
                          uint8_t* verdicts);

/* ---------------------------------------------------------------- scalar multiplication
 * out[i] = k_i * P_i, k_i a 32-byte little-endian integer (any value < 2^256).  Public-data helper
 * for commitments (Poly::commitment = g1 * c_i, src/sync_key_gen.rs:508), public-key-share
 * derivation (src/network_info.rs:59-62) and synthetic-input generation.  Secret keys stay on the
 * host in the reference flow (sign_g2 / decrypt_share). */
int hbh_g1_mul(hbh_engine* eng, size_t n, const uint8_t* pts, const uint8_t* scalars, uint8_t* out);
int hbh_g2_mul(hbh_engine* eng, size_t n, const uint8_t* pts, const uint8_t* scalars, uint8_t* out);
/* out[i] = g1 * k_i with a fixed-base comb table of the generator (32 mixed additions per scalar,
 * table built on the engine's first use): BivarPoly::commitment / Poly::commitment
 * (src/sync_key_gen.rs:346-357, 508) and key derivation.  Same points as hbh_g1_mul(g1, k). */
int hbh_g1_mul_gen(hbh_engine* eng, size_t n, const uint8_t* scalars, uint8_t* out);

/* ---------------------------------------------------------------- SyncKeyGen commitments
 * commits: nparts BivarCommitments of degree t, each (t+1)(t+2)/2 G1 points in threshold_crypto's
 * coeff_pos order (j(j+1)/2 + i for i <= j).
 * hbh_bivar_row: BivarCommitment::row(x) (src/sync_key_gen.rs:496) for nrow (part_idx, x) pairs;
 *   out = nrow * (t+1) G1 points.  Compare with Poly::commitment (hbh_g1_mul of g1) for :508.
 * hbh_bivar_ack_check: verdict[a] = (BivarCommitment::evaluate(x_a, y_a) == g1 * val_a)
 *   (src/sync_key_gen.rs:542); vals are 32-byte LE Fr values (the decrypted Ack values).
 *   x, y are the 1-based node indices the reference passes (our_idx + 1, sender_idx + 1). */
int hbh_bivar_row(hbh_engine* eng, size_t nrow, int t, size_t nparts, const uint8_t* commits, const uint32_t* part_idx,
                  const uint32_t* xs, uint8_t* out);
int hbh_bivar_ack_check(hbh_engine* eng, size_t nack, int t, size_t nparts, const uint8_t* commits,
                        const uint32_t* part_idx, const uint32_t* xs, const uint32_t* ys, const uint8_t* vals,
                        uint8_t* verdicts);

/* Device-resident commitments.  A SyncKeyGen instance keeps every Part's BivarCommitment for its
 * lifetime (ProposalState::commit, src/sync_key_gen.rs:254-262) and checks rows (:496) and Acks
 * (:542) against it on every drain.  A commitment set holds such commitments (one degree t per set)
 * in HBM, uploaded once, plus the Jacobian rows row(x) computed so far; calls name parts by their
 * index in the set and upload only indices and values.
 *   hbh_commit_set_create / _destroy: an empty set of degree t on `eng` (destroy waits for the
 *     engine's work).  The engine owns its sets' device memory: hbh_engine_destroy frees it and
 *     detaches the sets, after which every call on such a set returns HBH_ERR_ARG and
 *     hbh_commit_set_destroy only frees the handle (either destruction order is safe).
 *   hbh_commit_set_add: append nparts commitments ((t+1)(t+2)/2 ABI G1 points each, coeff_pos
 *     order); *first (may be NULL) = the set index of the first one.
 *   hbh_commit_set_size: commitments and cached rows held.
 *   hbh_bivar_row_set / hbh_bivar_ack_check_set: hbh_bivar_row / hbh_bivar_ack_check with part_idx
 *     into the set (same outputs). */
typedef struct hbh_commit_set hbh_commit_set;
int hbh_commit_set_create(hbh_engine* eng, int t, hbh_commit_set** out);
int hbh_commit_set_destroy(hbh_commit_set* cs);
int hbh_commit_set_add(hbh_commit_set* cs, size_t nparts, const uint8_t* commits, size_t* first);
int hbh_commit_set_size(const hbh_commit_set* cs, size_t* nparts, size_t* nrows);
int hbh_bivar_row_set(hbh_commit_set* cs, size_t nrow, const uint32_t* part_idx, const uint32_t* xs, uint8_t* out);
int hbh_bivar_ack_check_set(hbh_commit_set* cs, size_t nack, const uint32_t* part_idx, const uint32_t* xs,
                            const uint32_t* ys, const uint8_t* vals, uint8_t* verdicts);

/* Commitment::evaluate(x) = sum_j C_j x^j for n (commitment, x) requests; commits holds ncommits
 * Commitments of t+1 G1 points each, out = n G1 points.  PublicKeySet::public_key_share(i) is
 * evaluate(i + 1): NetworkInfo::new precomputes it for every node (src/network_info.rs:59-62), and
 * a SyncKeyGen node does the same for the generated key (src/sync_key_gen.rs:449 via
 * PublicKeySet::from(commit)).  xs are the 1-based integers the reference passes. */
int hbh_commitment_eval(hbh_engine* eng, size_t n, int t, size_t ncommits, const uint8_t* commits,
                        const uint32_t* commit_idx, const uint32_t* xs, uint8_t* out);

/* ---------------------------------------------------------------- wire formats
 * pairing 0.14 G1Compressed::into_affine for n 48-byte compressed G1 points (zcash encoding:
 * big-endian x, 0x80 = compressed, 0x40 = infinity, 0x20 = larger y).  out[i] = the ABI point,
 * ok[i] = 1 iff the encoding is well formed, x < p, x^3 + 4 is a square and the point lies in the
 * prime-order subgroup -- the checks threshold_crypto's deserialisation runs on every PublicKey,
 * PublicKeyShare, DecryptionShare and Ciphertext U before it reaches the verify calls (serde
 * decoding of hbbft's messages; decode sites listed in SURVEY §8f f2).
 * A point with ok[i] == 0 is written as all-zero bytes; the caller rejects the message as the
 * reference's deserialisation error does. */
int hbh_g1_decompress(hbh_engine* eng, size_t n, const uint8_t* in, uint8_t* out, uint8_t* ok);
/* G2Compressed::into_affine for n 96-byte compressed G2 points (x.c1 || x.c0 big-endian, flags in
 * the first byte; y^2 = x^3 + 4(1 + u); larger y by pairing 0.14's Fq2 order: c1, then c0);
 * out = ABI G2 points.  Same ok / all-zero convention as hbh_g1_decompress. */
int hbh_g2_decompress(hbh_engine* eng, size_t n, const uint8_t* in, uint8_t* out, uint8_t* ok);

/* ---------------------------------------------------------------- host stage (CPU, no engine)
 * What the north star keeps on the host, batched over `threads` std::thread workers (0 = all
 * hardware threads).  Variable-length inputs are concatenated in `data` with n+1 ascending byte
 * offsets (item i = data[offsets[i] .. offsets[i+1])).  Conventions: host_hash.cpp header and
 * SURVEY.md Appendix B.  Error text of these functions: hbh_host_last_error().
 *   hbh_hash_g2       threshold_crypto hash_g2(msg) -> G2 (ThresholdSign::set_document,
 *                     src/threshold_sign.rs:151; BA coin documents, binary_agreement.rs:442)
 *   hbh_hash_g1_g2    hash_g1_g2(U, V) -> G2 (Ciphertext::verify / verify_decryption_share's H_uv,
 *                     src/threshold_decrypt.rs:142,227)
 *   hbh_xor_with_hash V xor ChaCha20(sha3(compress(g))) low bytes; out has data's layout
 *                     (PublicKeySet::decrypt, src/threshold_decrypt.rs:249; SecretKey::decrypt,
 *                     src/sync_key_gen.rs:505,537)
 *   hbh_signature_parity  Signature::parity() per G2 point (the BA coin, binary_agreement.rs:402)
 *   hbh_g1_compress / hbh_g2_compress  pairing 0.14 compressed encodings (48 / 96 B)
 *   hbh_host_g1_mul / hbh_host_g2_mul  k * P with SECRET k on the host: SecretKeyShare::sign_g2
 *                     (threshold_sign.rs:167), decrypt_share_no_verify (threshold_decrypt.rs:161),
 *                     SecretKey::decrypt's U * sk (sync_key_gen.rs:505,537)
 *   hbh_host_g1_add   out[i] = a[i] + b[i] (public points; SyncKeyGen::generate's sum of
 *                     commitment rows, src/sync_key_gen.rs:449)
 *   hbh_encrypt       PublicKey::encrypt_with_rng with caller-drawn Fr nonces (32 B LE each):
 *                     U = g1 r, V = msg xor stream(pk r), W = hash_g1_g2(U, V) r
 *                     (sync_key_gen.rs:346-357,386-390; honey_badger/epoch_state.rs:224-237);
 *                     pks holds one key, or one per item when pk_per_item != 0
 *   hbh_fr_poly_eval  Poly::evaluate over Fr for many polynomials and points: out[p * npts + k] =
 *                     sum_j coeffs[p * ncoef + j] x_k^j mod r (32 B LE scalars in and out, coefficients
 *                     < r; xs are small node indices).  SyncKeyGen's rows of BivarPoly::row(x)
 *                     (sync_key_gen.rs:349-352) and the Ack values row.evaluate(i + 1) (:386-390)
 *   hbh_host_threads  the worker count `threads` = 0 means: the CPUs this process may use
 *                     (affinity mask, cgroup v2 cpu.max quota, HBH_HOST_THREADS / OMP_NUM_THREADS) */
const char* hbh_host_last_error(void);
int hbh_host_threads(int* out);
int hbh_hash_g2(size_t n, const uint8_t* data, const size_t* offsets, uint8_t* out, int threads);
int hbh_hash_g1_g2(size_t n, const uint8_t* u, const uint8_t* data, const size_t* offsets, uint8_t* out,
                   int threads);
int hbh_xor_with_hash(size_t n, const uint8_t* g, const uint8_t* data, const size_t* offsets, uint8_t* out,
                      int threads);
/* Ciphertext::verify without the last scalar multiplication of hash_g1_g2 (round 5): out[i] = Q_i,
 * a G2 point with hash_g1_g2(U_i, V_i) = [KCOF] Q_i for one fixed scalar KCOF (G2::rand's cofactor
 * multiplication h2 (x, y) = [KCOF] Q, Q = the Budroni-Pintore image of (x, y)).  By
 * bilinearity Ciphertext::verify(U, V, W) = e(g1, W) == e(U, [KCOF] Q) = e(G1K, W) == e(U, Q) with
 * G1K = [KCOF^-1 mod r] g1 (hbh_hash_bp_g1): hbh_verify_pairing_eq(P1 = G1K, Q1 = W, P2 = U, Q2 = Q)
 * gives the reference's verdict bit for bit (SecretKey::decrypt, sync_key_gen.rs:503-506, 535-538). */
int hbh_hash_g1_g2_bp(size_t n, const uint8_t* u, const uint8_t* data, const size_t* offsets, uint8_t* out,
                      int threads);
int hbh_hash_bp_g1(uint8_t* out);
int hbh_signature_parity(size_t n, const uint8_t* sigs, uint8_t* out);
int hbh_g1_compress(size_t n, const uint8_t* pts, uint8_t* out);
int hbh_g2_compress(size_t n, const uint8_t* pts, uint8_t* out);
int hbh_host_g1_mul(size_t n, const uint8_t* pts, const uint8_t* scalars, uint8_t* out, int threads);
int hbh_host_g2_mul(size_t n, const uint8_t* pts, const uint8_t* scalars, uint8_t* out, int threads);
int hbh_host_g1_add(size_t n, const uint8_t* a, const uint8_t* b, uint8_t* out);
int hbh_encrypt(size_t n, const uint8_t* pks, int pk_per_item, const uint8_t* data, const size_t* offsets,
                const uint8_t* nonces, uint8_t* u_out, uint8_t* v_out, uint8_t* w_out, int threads);
int hbh_fr_poly_eval(size_t npoly, size_t ncoef, const uint8_t* coeffs, size_t npts, const uint64_t* xs, uint8_t* out,
                     int threads);

/* ---------------------------------------------------------------- implementation selection
 * Pairing implementations with identical verdicts (tests/test_gpu_pairing.py cross-checks them
 * against each other and the C oracle):
 *   HBH_IMPL_PAIR (k_pair.hip): TWO lanes per check, each lane holding one component of every Fp2
 *     value; the Miller loop walks per-check G2 points in registers and reads line tables only for
 *     G2 points shared through an index map; Miller loop and final exponentiation in one kernel.
 *     Throughput path.
 *   HBH_IMPL_WAVE (k_wave.hip): one 64-lane wave per check; the check's Fp2 products run on 32 lane
 *     pairs side by side.  Latency path (one check: the master check of combine_and_verify_sig).
 *   HBH_IMPL_QUAD (k_quad.hip): FOUR lanes per check -- two lane pairs holding the check's state
 *     side by side and splitting each step's independent products (k_pair's work per check in
 *     ~0.55 of its per-lane time).  Mid-size path: 16,384 checks are one wave per SIMD.
 *   HBH_IMPL_OCT (k_oct.hpp): EIGHT lanes per check -- four lane pairs, four independent products per
 *     round.  Small-batch path: 8,192 checks are one wave per SIMD.
 *   HBH_IMPL_WAVE2 (k_wave64.hip, round 6): TWO 64-lane waves per check (64 lane pairs): the Miller
 *     loop multiplies a step's two lines together beside f^2 and takes their product in one stage,
 *     149 stages per two-pair check instead of WAVE's 210-211.  Latency path for calls of up to
 *     HBH_AUTO_WAVE2_MAX checks (AUTO; plain checks -- the split master check's modes stay on WAVE).
 *   HBH_IMPL_AUTO (the default): WAVE2 up to HBH_AUTO_WAVE2_MAX checks per call, WAVE up to
 *     HBH_AUTO_WAVE_MAX checks per call, OCT up to
 *     HBH_AUTO_OCT_MAX, QUAD up to HBH_AUTO_QUAD_MAX (each one wave per SIMD at its maximum), PAIR
 *     above -- the measured crossovers (profiles/r04/c8_sweep_wave_quad_pair.txt,
 *     c23_oct_wave_sweep.txt, kernel ms per call on the sign workload): 4,096 checks WAVE 5.3 /
 *     OCT 5.5 / QUAD 7.0 / PAIR 10.6; 4,608: WAVE 6.6 / OCT 5.5; 8,192: 10.2 / 5.5 / 7.0 / 10.7;
 *     16,384: WAVE 20.1 / OCT 11.6 / QUAD 7.1 / PAIR 11.1; 24,576: QUAD 14.3 (two rounds of waves) /
 *     PAIR 11.2.  Between 32,768 and 49,152 checks the lane
 *     pair needs a second wave on some SIMDs (40,960: 20.5 ms), so AUTO runs the first 32,768 on
 *     PAIR (one wave per SIMD, 11.5 ms) and the rest by the rules above (WAVE / OCT / QUAD) on the same
 *     stream; above 49,152, whole rounds of 65,536 checks (two lane-pair waves per SIMD) run on
 *     PAIR and the remainder follows the same rules.
 * Retired (selecting them returns HBH_ERR_ARG): HBH_IMPL_THREAD (0, round 1's one-thread kernel),
 * HBH_IMPL_LANE_COOP (1, six lanes per check) and HBH_IMPL_THREAD_SIGNED (2, one thread per check
 * on signed limbs) -- WAVE and PAIR cover every batch size faster. */
#define HBH_IMPL_THREAD 0
#define HBH_IMPL_LANE_COOP 1
#define HBH_IMPL_THREAD_SIGNED 2
#define HBH_IMPL_AUTO 3
#define HBH_IMPL_PAIR 4
#define HBH_IMPL_WAVE 5
#define HBH_IMPL_QUAD 6
#define HBH_IMPL_OCT 7
#define HBH_IMPL_WAVE2 8
#define HBH_AUTO_WAVE2_MAX 512  /* AUTO: WAVE2 up to here (two waves per check), then WAVE (profiles/r06/latency_c6.txt) */
#define HBH_AUTO_WAVE_MAX 4096
#define HBH_AUTO_OCT_MAX 8192
#define HBH_AUTO_QUAD_MAX 16384
#define HBH_AUTO_SPLIT_LO 32768  /* AUTO: (32,768, 49,152] checks = PAIR on 32,768 + the rest by size */
#define HBH_AUTO_SPLIT_HI 49152
#define HBH_AUTO_PAIR_ROUND 65536  /* AUTO above HBH_AUTO_SPLIT_HI: whole rounds of 65,536 on PAIR, the rest by size */
int hbh_engine_set_pairing_impl(hbh_engine* eng, int impl);
/* Ack-check kernel of hbh_bivar_ack_check_set: HBH_ACK_QUAD (k_bivar_check_quad: four lanes per ack
 * split each G1 operation, Jacobian rows -- latency), HBH_ACK_LANE (k_bivar_check: one lane per ack,
 * affine rows and mixed additions -- throughput), HBH_ACK_AUTO (default: LANE from HBH_ACK_LANE_MIN
 * acks per call; measured crossover ~50,000 acks, profiles/r03/ack_kernel_sweep.txt: 40,000 acks
 * quad 6.4 / lane 7.0 ms, 160,000 acks 18.9 / 13.1 ms, 10^6 acks 112 / 53 ms).  Same verdicts.
 * Round 5: on the LANE path (and AUTO's), the acks of a row whose y form a dense run (>= 2 (t + 1) acks
 * over <= twice as many consecutive y: a node's drain, one Ack per sender per Part) are checked by
 * finite differences -- t + 1 Horner points, then t G1 additions per further y;
 * HBH_ACK_LANE_HORNER keeps every ack on the Horner kernel (A/B, parity tests). */
#define HBH_ACK_AUTO 0
#define HBH_ACK_QUAD 1
#define HBH_ACK_LANE 2
#define HBH_ACK_LANE_HORNER 3
#define HBH_ACK_LANE_MIN 65536
int hbh_engine_set_ack_impl(hbh_engine* eng, int impl);

/* ---------------------------------------------------------------- profiling
 * With profiling on, the engine records HIP events around each stage's kernels on the stream they
 * run on; hbh_engine_stage_time returns the summed device time and launch count since the last
 * hbh_engine_set_profiling call. */
#define HBH_STAGE_PREPARE 0 /* Miller-loop line tables (G2 walks) */
#define HBH_STAGE_PAIRING 1 /* multi-Miller loop + final exponentiation */
#define HBH_STAGE_CURVE 2   /* scalar multiplication / interpolation / bivariate checks */
#define HBH_NUM_STAGES 3
int hbh_engine_set_profiling(hbh_engine* eng, int on);
int hbh_engine_stage_time(hbh_engine* eng, int stage, double* total_ms, int* launches);

/* ---------------------------------------------------------------- debug / test entry points
 * hbh_dbg_pairing: out[i] = e(P[i], Q[i])^3 as 12 canonical Fp2 coefficients (c0.c0.c0, c0.c0.c1,
 * c0.c1.c0, ... c1.c2.c1; 48 B LE each = 576 B) -- the pairing value itself, for parity tests
 * against the oracle (the kernel's final exponentiation uses the exponent 3(p^12-1)/r). */
int hbh_dbg_pairing(hbh_engine* eng, size_t n, const uint8_t* p, const uint8_t* q, uint8_t* out);

#ifdef __cplusplus
}
#endif

#endif /* HBBFT_HIP_H */
