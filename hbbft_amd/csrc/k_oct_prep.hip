// Line tables of shared G2 points on lane octos (the TABLE side of every pairing kernel).
//
// The serial 68-step walk of one shared point (63 doublings + 5 additions of |x|) with the lane-octo
// doubling and addition steps (ofp.hpp: 3 and 5 rounds of four Fp2 products), eight lanes per point;
// pair 0 of each octo writes the table (c0, c1, c4 per step and lane component, PL_Q4 16-byte chunks,
// pair_side.hpp), which every verify kernel reads unchanged.
#include "launch.hpp"
#include "pair_side.hpp"
#include "ofp.hpp"

namespace hbs {

__global__ void __launch_bounds__(256, 1) k_oct_prep(int n, const uint32_t* __restrict__ q, int4* __restrict__ lines,
                                                     uint8_t* __restrict__ qinf) {
  const int j = (int)((blockIdx.x * 256u + threadIdx.x) >> 3);
  if (j >= n) return;  // the eight lanes of an octo leave together
  const uint32_t* w = q + (size_t)j * 48;
  const bool inf = lp_both(words_zero(w + (lp_even() ? 0 : 12), 12) && words_zero(w + (lp_even() ? 24 : 36), 12));
  Fp xQ, yQ;
  h_g2_load(w, xQ, yQ);
  if (inf) {
    xQ = h_one();
    yQ = h_one();
  }
  const bool writer = o_idx() == 0;
  if ((threadIdx.x & 7) == 0) qinf[j] = inf ? 1 : 0;
  HJac T{xQ, yQ, h_one()};
  int4* base = lines + (size_t)j * PAIR_STEPS * 2 * PL_Q4 + (lp_even() ? 0 : PL_Q4);
  int step = 0;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
#pragma unroll 1
    for (int add = 0; add < (((hb::X_ABS >> b) & 1) ? 2 : 1); add++) {
      const HLine l = add ? h_add_step_o(T, xQ, yQ) : h_dbl_step_o(T);
      if (writer) {
        int32_t o[4 * PL_Q4];
#pragma unroll
        for (int k = 0; k < NL; k++) {
          o[k] = l.c0.l[k];
          o[NL + k] = l.c1.l[k];
          o[2 * NL + k] = l.c4.l[k];
        }
        o[3 * NL] = 0;
        o[3 * NL + 1] = 0;
        int4* dst = base + (size_t)step * 2 * PL_Q4;
#pragma unroll
        for (int k = 0; k < PL_Q4; k++) dst[k] = make_int4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
      }
      step++;
    }
  }
}

}  // namespace hbs

namespace hbl {

hipError_t oct_prep(hipStream_t s, int n, const void* q, void* lines, uint8_t* qinf) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hbs::k_oct_prep, dim3((unsigned)((8 * (size_t)n + 255) / 256)), dim3(256), 0, s, n,
                     (const uint32_t*)q, (int4*)lines, qinf);
  return hipGetLastError();
}

}  // namespace hbl
