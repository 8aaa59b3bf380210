// HBH_IMPL_WAVE2: TWO waves per pairing check -- the single-check latency kernel (gfx950, round 6).
//
// k_wave.hip's interpreter over 64 lane pairs (128 threads, one workgroup per check; the two waves
// land on two SIMDs of one CU and share the check's LDS slots).  What the extra pairs buy is a
// shorter program, not wider stages: with 64 products per stage the Miller loop multiplies the
// step's two lines together beside f^2 and takes their product in one 30-product stage, and a walked
// side keeps T in homogeneous coordinates (two product levels per doubling) -- 149 Miller stages
// per two-pair check where the 32-pair programs need 210-211 (tools/gen_wave_prog.py miller_c,
// wave_prog64.inc).  The final exponentiation is the 32-pair program; its cyclotomic-squaring runs
// stay on the first wave.  One check on one wave of one SIMD issues at most one VALU instruction
// every ~4.7 cycles and a 64-bit MAD every ~9 (profiles/r06/ubench_issue.txt), so the stage count
// is what sets a lone check's latency; the engine uses this kernel for calls of few checks, where
// the second wave per check costs no occupancy (HBH_AUTO_WAVE2_MAX).
#define WV_NS hbs64
#define WV_PROG hbw64
#define WV_THREADS 128
#define WV_FULL 0
#include "wave_prog64.inc"
#include "k_wave.hpp"

namespace hbl {

size_t wave64_lds_bytes() { return (size_t)hbw64::WP_NSLOTS * hbs64::WV_STRIDE * 4; }

hipError_t wave64_verify(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
                         uint8_t* verdict, uint32_t* value_out) {
  if (n <= 0) return hipSuccess;
  if (flags & ~(WAVE_NEG_P2 | WAVE_CONJ_VALUE)) return hipErrorInvalidValue;  // plain checks only
  hbs64::WaveArgs a = {};
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
  hipLaunchKernelGGL(hbs64::k_wave, dim3((unsigned)n), dim3(128), wave64_lds_bytes(), s, a);
  return hipGetLastError();
}

}  // namespace hbl
