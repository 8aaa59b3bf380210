// Lane-pair walk of G2 points into the line-table layout of the lane-cooperative and one-thread
// signed implementations (lines.hpp store_line: 68 steps x 21 int4 x pad64(n) points).
//
// k_g2_prepare walks one point per thread: for the few points of a latency-bound call (the master
// check of combine_and_verify_sig, a small drain) that serial walk is the critical path.  Here two
// lanes share a point (pfp.hpp: even lane c0, odd lane c1 of every Fp2), halving the walk's
// latency; each lane stores its own components, reduced to [0, 2p) with non-negative limbs (the
// unsigned-limb contract of fp.hpp: limbs < 2^30, value < 45p).  Same line formulas
// (pairing.hpp dbl_step / add_step), same Montgomery radix R = 2^392.
#define HS_MULFN static __device__ __noinline__
#include "launch.hpp"
#include "pfp.hpp"

namespace hbs {

// [-p, 2p) signed -> [0, 2p) with non-negative normalised limbs
HP_D Fp to_unsigned(const Fp& a) {
  const Fp r = fp_reduce(a);
  Fp rp = fp_addl(r, fp_const(P_L));
  fp_norm(rp);
  return (r.l[NL - 1] < 0) ? rp : r;
}

struct LcPrepSet {
  int n;
  const uint32_t* pts;
  int stride;
  uint32_t* coef;
  uint8_t* inf;
};

__global__ void __launch_bounds__(256, 2) k_lc_prep_pair(LcPrepSet s0, LcPrepSet s1) {
  int j = (int)((blockIdx.x * 256u + threadIdx.x) >> 1);
  const bool first = j < s0.n;
  if (!first) j -= s0.n;
  if (!first && j >= s1.n) return;  // both lanes of a pair leave together
  const LcPrepSet& s = first ? s0 : s1;
  const uint32_t* w = s.pts + (size_t)j * 48;
  const bool inf = lp_both(words_zero(w + (lp_even() ? 0 : 12), 12) && words_zero(w + (lp_even() ? 24 : 36), 12));
  Fp xQ, yQ;
  h_g2_load(w, xQ, yQ);
  if (inf) {  // dummy walk from (1, 1); the pair is masked out by the consumer
    xQ = h_one();
    yQ = h_one();
  }
  if (lp_even()) s.inf[j] = inf ? 1 : 0;
  HJac T{xQ, yQ, h_one()};
  const int comp = lp_even() ? 0 : 1;  // word offset of this lane's Fp2 component: 14 * (2k + comp)
  int step = 0;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
#pragma unroll 1
    for (int add = 0; add < (((hb::X_ABS >> b) & 1) ? 2 : 1); add++) {
      const HLine l = add ? h_add_step(T, xQ, yQ) : h_dbl_step(T);
      const Fp c[3] = {to_unsigned(l.c0), to_unsigned(l.c1), to_unsigned(l.c4)};
#pragma unroll
      for (int k = 0; k < 3; k++) {
#pragma unroll
        for (int i = 0; i < NL; i++) {
          const int word = (2 * k + comp) * NL + i;  // lines.hpp: c0.c0 c0.c1 c1.c0 c1.c1 c4.c0 c4.c1
          const size_t q = (size_t)step * hbl::LINE_Q4 + word / 4;
          s.coef[(q * s.stride + j) * 4 + word % 4] = (uint32_t)c[k].l[i];
        }
      }
      step++;
    }
  }
}

}  // namespace hbs

namespace hbl {

hipError_t lc_prep_pair(hipStream_t s, int n0, const void* pts0, void* coef0, uint8_t* inf0, int n1, const void* pts1,
                        void* coef1, uint8_t* inf1) {
  if (n0 + n1 <= 0) return hipSuccess;
  hbs::LcPrepSet a{n0, (const uint32_t*)pts0, pad64(n0), (uint32_t*)coef0, inf0};
  hbs::LcPrepSet b{n1, (const uint32_t*)pts1, pad64(n1), (uint32_t*)coef1, inf1};
  const size_t lanes = 2 * ((size_t)n0 + (size_t)n1);
  hipLaunchKernelGGL(hbs::k_lc_prep_pair, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, s, a, b);
  return hipGetLastError();
}

}  // namespace hbl
