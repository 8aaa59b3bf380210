// HBH_IMPL_WAVE: one WAVE per pairing check -- the latency kernel (gfx950).
//
// The lane-pair kernel (k_pair.hip) gives a check two lanes and runs its ~5,400 Fp2 products one
// after another; that is the right shape for 65,536 checks and the wrong one for the master check
// of combine_and_verify_sig (src/threshold_sign.rs:264) or the small per-message batches of the
// protocol flows, where one check's serial chain is the whole latency.  Here a check owns a wave:
// 32 lane pairs, each computing one Fp2 product (pfp.hpp lane-pair split: even lane c0, odd lane
// c1), so every Fp12 / curve operation of a step runs as ~20 independent products side by side.
//
// The kernel is an interpreter of the stage programs built by tools/gen_wave_prog.py
// (wave_prog.inc): the check's state lives in LDS slots (one Fp2 = 2 x 16 words, stride 36 words);
// each stage is a product phase (pair j: X = +-(S[a] +- S[b]), Y = +-(S[c] +- S[d]);
// PROD_j = X*Y | X1*Y1 + X2*Y2 | X^2) and an assembly phase (pair o: S[dst_o] = sum c V + xi sum
// c' V', reduced, optionally replaced by 1 / 0 when its pair is inactive), separated by barriers.
// The programs are the formulas of k_pair.hip (pairing 0.14 lines, final_exp_x3 chain); their
// exact emulation is checked against the oracle on the CPU (tests/test_wave_prog.py).
//
// One 64-thread workgroup per check; 118 slots = 17 KiB of LDS per check.  The kernel body is
// k_wave.hpp (shared with k_wave64.hip, two waves per check).
#define WV_NS hbs
#define WV_PROG hbw
#define WV_THREADS 64
#define WV_FULL 1
#include "wave_prog.inc"
#include "k_wave.hpp"

namespace hbl {

size_t wave_lds_bytes() { return (size_t)hbw::WP_NSLOTS * hbs::WV_STRIDE * 4; }

hipError_t wave_verify(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
                       uint8_t* verdict, uint32_t* value_out) {
  if (n <= 0) return hipSuccess;
  hbs::WaveArgs a;
  a.n = n;
  const PairSideDesc* d[2] = {&d1, &d2};
  for (int k = 0; k < 2; k++) {
    a.s[k].p = (const uint32_t*)d[k]->p;
    a.s[k].q = (const uint32_t*)d[k]->q;
    a.s[k].lines = (const int4*)d[k]->lines;
    a.s[k].qinf = d[k]->qinf;
    a.s[k].idx = d[k]->idx;
    a.s[k].nq = (uint32_t)d[k]->nq;
  }
  a.flags = flags;
  a.verdict = verdict;
  a.value_out = value_out;
  a.fin = nullptr;
  a.nf = 0;
  a.tree_cnt = nullptr;
  a.tree_nw = 0;
  hipLaunchKernelGGL(hbs::k_wave, dim3((unsigned)n), dim3(64), wave_lds_bytes(), s, a);
  return hipGetLastError();
}

size_t wave_tree_counter_bytes(int ngroup, int nw) { return (size_t)ngroup * hbs::TREE_LEVELS * nw * 4; }
hipError_t wave_miller_tree(hipStream_t s, int ngroup, int nw, const PairSideDesc& d1, const PairSideDesc& d2,
                            int flags, uint32_t* value_out, uint32_t* counters, uint8_t* verdict) {
  if (ngroup <= 0) return hipSuccess;
  if (nw <= 0 || nw >= (1 << (hbs::TREE_LEVELS - 1)) || !value_out || !counters || !(flags & WAVE_MILLER_ONLY))
    return hipErrorInvalidValue;
  // a group whose tree never completes (a check index out of range) keeps verdict 0
  hipError_t z = hipMemsetAsync(counters, 0, wave_tree_counter_bytes(ngroup, nw), s);
  if (z == hipSuccess && verdict) z = hipMemsetAsync(verdict, 0, (size_t)ngroup, s);
  if (z != hipSuccess) return z;
  hbs::WaveArgs a = {};
  a.n = ngroup * nw;
  const PairSideDesc* d[2] = {&d1, &d2};
  for (int k = 0; k < 2; k++) {
    a.s[k].p = (const uint32_t*)d[k]->p;
    a.s[k].q = (const uint32_t*)d[k]->q;
    a.s[k].lines = (const int4*)d[k]->lines;
    a.s[k].qinf = d[k]->qinf;
    a.s[k].idx = d[k]->idx;
    a.s[k].nq = (uint32_t)d[k]->nq;
  }
  a.flags = flags;
  a.verdict = verdict;
  a.value_out = value_out;
  a.tree_cnt = counters;
  a.tree_nw = nw;
  hipLaunchKernelGGL(hbs::k_wave, dim3((unsigned)a.n), dim3(64), wave_lds_bytes(), s, a);
  return hipGetLastError();
}

hipError_t wave_prod_fe(hipStream_t s, int n, int nf, const uint32_t* fin, uint8_t* verdict) {
  if (n <= 0) return hipSuccess;
  if (nf <= 0 || !fin) return hipErrorInvalidValue;
  hbs::WaveArgs a = {};
  a.n = n;
  a.flags = 0;
  a.verdict = verdict;
  a.value_out = nullptr;
  a.fin = fin;
  a.nf = nf;
  hipLaunchKernelGGL(hbs::k_wave, dim3((unsigned)n), dim3(64), wave_lds_bytes(), s, a);
  return hipGetLastError();
}

}  // namespace hbl
