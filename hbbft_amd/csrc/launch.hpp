// Host-side launchers of the HIP kernels.  Each kernel family lives in its own translation unit
// (k_pair.hip, k_quad.hip, k_wave.hip, k_curve.hip, k_g1quad.hip, k_interp_pair.hip, k_wire.hip) so the Makefile
// compiles them in parallel; engine.hip owns the C ABI, device buffers and streams and calls only
// these functions.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace hbl {

constexpr int HBL_DUPLICATE = 5;  // == HBH_ERR_DUPLICATE_ENTRY
constexpr int HBL_BAD_INDEX = 1;  // == HBH_ERR_ARG
// --------------------------------------------------------------- lane-pair pairing (k_pair.hip)
// One side of a pairing-equality check.  TABLE side: `lines`/`qinf` from oct_prep over the nq
// shared G2 points, `idx` picks the table per check.  WALK side (lines == nullptr): `q` holds G2
// points walked inside the Miller loop, `idx` picks the point per check (nullptr = identity).
// p == nullptr means the G1 generator for every check.  Indices >= nq yield verdict 0.
struct PairSideDesc {
  const void* p;
  const void* q;
  const void* lines;
  const uint8_t* qinf;
  const uint32_t* idx;
  size_t nq;
};
size_t pair_table_bytes(size_t nq);
// the same tables from lane octos (k_oct_prep.hip: eight lanes per point)
hipError_t oct_prep(hipStream_t s, int n, const void* q, void* lines, uint8_t* qinf);
// flags: bit 0 negates P2 (pairing equality), bit 1 conjugates f (single pairing value, with
// value_out: e(P1,Q1)^3 e(P2,Q2)^3 as 144 canonical words per check)
hipError_t pair_verify(hipStream_t s, int n, const PairSideDesc& s1, const PairSideDesc& s2, int flags,
                       uint8_t* verdict, uint32_t* value_out);

// --------------------------------------------------------------- lane-quad pairing (k_quad.hip)
// The same verdicts / values as pair_verify with FOUR lanes per check (two lane pairs splitting
// each step's independent products): the mid-size batches, one wave per SIMD at 16,384 checks.
// TABLE sides read oct_prep tables.
hipError_t quad_verify(hipStream_t s, int n, const PairSideDesc& s1, const PairSideDesc& s2, int flags,
                       uint8_t* verdict, uint32_t* value_out);

// --------------------------------------------------------------- lane-octo pairing (k_oct.hpp)
// The same with EIGHT lanes per check (four lane pairs, four products per round): one wave per SIMD
// at 8,192 checks.
hipError_t oct_verify(hipStream_t s, int n, const PairSideDesc& s1, const PairSideDesc& s2, int flags,
                      uint8_t* verdict, uint32_t* value_out);

// --------------------------------------------------------------- wave-per-check pairing (k_wave.hip)
// The same verdicts / values as pair_verify with one 64-lane workgroup per check (the latency
// kernel: a check's Fp2 products run on 32 lane pairs side by side).  TABLE sides read oct_prep
// tables; wave_lds_bytes() of LDS per workgroup.
size_t wave_lds_bytes();
hipError_t wave_verify(hipStream_t s, int n, const PairSideDesc& s1, const PairSideDesc& s2, int flags,
                       uint8_t* verdict, uint32_t* value_out);
// flags bit 2 (WAVE_MILLER_ONLY): wave_verify writes each check's Miller value f (144 canonical words,
// w-basis) to value_out and stops there; wave_prod_fe then verifies prod_k fin[i][k] (nf values per
// check) with one final exponentiation: verdict[i] = (FE(prod) == 1).
constexpr int WAVE_MILLER_ONLY = 4;
// flags bit 3 (WAVE_JAC_P): every P is Jacobian, X || Y || Z canonical (36 words, Z = 0 at infinity);
// both sides must WALK.  The lines are scaled by Z^3, so no inversion of Z is needed.
constexpr int WAVE_JAC_P = 8;
// flags bit 4 (WAVE_ONE_SIDE, with WAVE_JAC_P): one pair per check, side 0 only (side 1 is not read):
// the homogeneous-walk Miller program (two stages per step instead of three)
constexpr int WAVE_ONE_SIDE = 16;
hipError_t wave_prod_fe(hipStream_t s, int n, int nf, const uint32_t* fin, uint8_t* verdict);
// wave_verify's Miller-only mode with the product and the final exponentiation in the same launch:
// the n = ngroup * nw checks form ngroup groups of nw consecutive checks; within a group the Miller
// values are multiplied up a binary tree (the later-arriving wave of each sibling pair multiplies,
// the other leaves), and the wave holding the group's product runs the final exponentiation:
// verdict[g] = (FE(prod_k f_{g nw + k}) == 1).  value_out (n x 144 words) holds the tree's values;
// counters: wave_tree_counter_bytes(ngroup, nw) bytes, zeroed by the launcher.
size_t wave_tree_counter_bytes(int ngroup, int nw);
hipError_t wave_miller_tree(hipStream_t s, int ngroup, int nw, const PairSideDesc& s1, const PairSideDesc& s2,
                            int flags, uint32_t* value_out, uint32_t* counters, uint8_t* verdict);
// The same verdicts / values as wave_verify with TWO waves (64 lane pairs) per check (k_wave64.hip,
// round 6): 149 Miller stages per two-pair check instead of 210-211 -- the latency kernel for calls
// of few checks.  Plain checks only (flags WAVE_NEG_P2 / WAVE_CONJ_VALUE).
constexpr int WAVE_NEG_P2 = 1;
constexpr int WAVE_CONJ_VALUE = 2;
size_t wave64_lds_bytes();
hipError_t wave64_verify(hipStream_t s, int n, const PairSideDesc& s1, const PairSideDesc& s2, int flags,
                         uint8_t* verdict, uint32_t* value_out);

// --------------------------------------------------------------- curve / MSM (k_curve.hip)
// out[i] = k_i * P_i (G1 or G2 ABI words; scalars 8 LE words, any 256-bit integer).
hipError_t g1_mul(hipStream_t s, int n, const void* pts, const uint32_t* scalars, void* out);
hipError_t g2_mul(hipStream_t s, int n, const void* pts, const uint32_t* scalars, void* out);
// Lagrange interpolation at 0 (threshold_crypto interpolate) of `ncomb` combines of m = t+1
// samples each: x[c*m + k] = idx + 1 (Fr, small integers), pts[c*m + k] the samples.
// status[c] (zeroed by the caller) becomes HBL_DUPLICATE when two x coincide.  out: ncomb affine
// points (ABI words).  One workgroup per combine (endomorphism-split terms + LDS tree sum).
hipError_t combine_g1(hipStream_t s, int ncomb, int m, const uint32_t* xs, const void* pts, void* out, int* status);
hipError_t combine_g2(hipStream_t s, int ncomb, int m, const uint32_t* xs, const void* pts, void* out, int* status);
// BivarCommitment::row(x) (t+1 outputs) for nrow (part, x) pairs; commit = (t+1)(t+2)/2 G1 points
// per part.  out[r*(t+1) + i].
hipError_t bivar_row(hipStream_t s, int nrow, int t, const void* commits, const uint32_t* part_idx, const uint32_t* xs,
                     void* out);
// BivarCommitment::evaluate(x, y) == g1 * val for nack checks, given the rows R = row(x) of each
// check's part: verdict[a] = (sum_j R[row_idx[a]][j] * y^j == g1 * val[a]).
// fbtab: the fixed-base comb table of g1 (fb_table), used for the g1 * val side.
// The same verdicts on lane quads (k_g1quad.hip): four lanes per ack split each point operation.
// Rows from bivar_row_quad: Jacobian signed-limb points, bivar_rows_quad_bytes(nrow, t) of scratch.
size_t bivar_rows_quad_bytes(int nrow, int t);
hipError_t bivar_row_quad(hipStream_t s, int nrow, int t, const void* commits, const uint32_t* part_idx,
                          const uint32_t* xs, void* rows);
hipError_t bivar_check_quad(hipStream_t s, int nack, int t, const void* rows, const uint32_t* row_idx,
                            const uint32_t* ys, const uint32_t* vals, const void* fbtab, uint8_t* verdict,
                            const uint32_t* order);
// order (may be null): thread k checks ack order[k] (acks sorted by y keep a wave's lanes in step).
// Ack checks by finite differences over dense runs of y (k_curve.hip): FD row f evaluates the affine row
// slot fd_slot[f] at y = fd_y0[f] .. fd_y0[f] + fd_len[f] - 1 (fd_len >= t + 1) into ebuf from point
// fd_off[f] on (fd_point_bytes() each); bivar_fd_check then compares ack list[k]'s point epos[a] with
// g1 * val from the 16-bit comb fb16 (fb16_table).  t + 1 <= 256.
size_t fd_point_bytes();
// 16-bit fixed-base comb of g1 for bivar_fd_check (16 windows x 65,536 affine points, fb16_table_bytes()),
// built once through fb16_scratch_bytes() of scratch
size_t fb16_table_bytes();
size_t fb16_scratch_bytes();
hipError_t fb16_table(hipStream_t s, void* tab, void* scratch);
hipError_t bivar_fd(hipStream_t s, int nfd, int t, const void* rows, const uint32_t* fd_slot, const uint32_t* fd_y0,
                    const uint32_t* fd_off, const uint32_t* fd_len, void* ebuf);
hipError_t bivar_fd_check(hipStream_t s, int n, const void* ebuf, const uint32_t* epos, const uint32_t* vals,
                          const void* fb16, const uint32_t* list, uint8_t* verdict);
hipError_t bivar_check(hipStream_t s, int nack, int t, const void* rows, const uint32_t* row_idx, const uint32_t* ys,
                       const uint32_t* vals, const void* fbtab, uint8_t* verdict, const uint32_t* order = nullptr);
// Fixed-base comb table of the G1 generator (32 windows x 256 affine points, fb_table_bytes()) and
// out[i] = g1 * k_i from it (32 mixed additions per scalar).
size_t fb_table_bytes();
hipError_t fb_table(hipStream_t s, void* tab);
hipError_t g1_mul_gen(hipStream_t s, int n, const void* tab, const uint32_t* scalars, void* out);
// lambda_k g1 (scalars 8 LE words each, n = ncomb * m) by a 5-level tree over the comb table, in
// Jacobian form (36 words: X || Y || Z canonical, all zero at infinity) to entry c * nw + k / 2 of out0 /
// out1 (even / odd k; pairs = 2) or entry c * nw + k of out0 (pairs = 1): the P sides of the split master
// check (k_wave with WAVE_JAC_P)
hipError_t g1_gen_tree(hipStream_t s, int n, int m, int nw, int pairs, const void* tab, const uint32_t* scalars,
                       void* out0, void* out1);
// xs[k] = idx[k] + 1 for n = ncomb * m device-resident indices; status[k / m] = HBL_BAD_INDEX for
// an index of 0xffffffff (status zeroed by the caller beforehand).
hipError_t index_plus_one(hipStream_t s, int n, int m, const uint32_t* idx, uint32_t* xs, int* status);
// Commitment::evaluate(x) for n (commitment, x) requests; commitments of t+1 G1 points.  out[r].
hipError_t commit_eval(hipStream_t s, int n, int t, const void* commits, const uint32_t* commit_idx, const uint32_t* xs,
                       void* out);

}  // namespace hbl
