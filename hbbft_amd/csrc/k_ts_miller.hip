// HBH_IMPL_THREAD_SIGNED, stage 1: the two-pair Miller loop, one thread per check, signed limbs.
// Same line tables (k_g2_prepare) and the same product as the pairing.hpp Miller loop; the
// accumulator is kept reduced (|.| < 2p) between Fp12 operations instead of canonical-ish < 2p
// unsigned, which removes the conditional subtractions from every Fp addition.
#define HS_MULFN static __device__ __noinline__
#include "launch.hpp"
#include "sthread.hpp"

namespace hbs {

struct SLine { Fp2 c0, c1, c4; };

// line table entry (lines.hpp store_line layout; values normalised, in [0, 2p))
__device__ __forceinline__ SLine ts_load_line(const int4* __restrict__ coef, int stride, int step, int pt) {
  int32_t w[84];
#pragma unroll
  for (int q = 0; q < 21; q++) {
    const int4 v = coef[((size_t)step * 21 + q) * stride + pt];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
  SLine l;
#pragma unroll
  for (int j = 0; j < NL; j++) {
    l.c0.c0.l[j] = w[0 * NL + j];
    l.c0.c1.l[j] = w[1 * NL + j];
    l.c1.c0.l[j] = w[2 * NL + j];
    l.c1.c1.l[j] = w[3 * NL + j];
    l.c4.c0.l[j] = w[4 * NL + j];
    l.c4.c1.l[j] = w[5 * NL + j];
  }
  return l;
}

struct TsPair {
  Fp x, y;
  const int4* coef;
  int stride, q;
  bool act;
};

__device__ __forceinline__ Fp12 ts_line(const Fp12& f, const TsPair& P, int step) {
  const SLine l = ts_load_line(P.coef, P.stride, step, P.q);
  const Fp2 c0 = f2_sel(P.act, l.c0, f2_one());
  const Fp2 c1 = f2_sel(P.act, t2_mul_fp(l.c1, P.x), f2_zero());
  const Fp2 c4 = f2_sel(P.act, t2_mul_fp(l.c4, P.y), f2_zero());
  return f12_mul_014(f, c0, c1, c4);
}

__device__ __forceinline__ TsPair ts_pair(const uint32_t* __restrict__ p, const int4* coef, int stride,
                                          const uint8_t* __restrict__ inf, const uint32_t* __restrict__ idx, int i) {
  TsPair P;
  const uint32_t* w = p + (size_t)i * 24;
  uint32_t o = 0;
  for (int k = 0; k < 24; k++) o |= w[k];
  P.x = fp_from_words(w);
  P.y = fp_from_words(w + 12);
  P.q = idx ? (int)idx[i] : i;
  P.act = o != 0 && !inf[P.q];
  P.coef = coef;
  P.stride = stride;
  return P;
}

// flags: bit 0 negates P2 (pairing equality), bit 1 conjugates f (x < 0; single-pairing values)
__global__ void __launch_bounds__(256) k_ts_miller(int n, const uint32_t* __restrict__ p1, const int4* __restrict__ coef1,
                                                   int stride1, const uint8_t* __restrict__ inf1,
                                                   const uint32_t* __restrict__ idx1, const uint32_t* __restrict__ p2,
                                                   const int4* __restrict__ coef2, int stride2,
                                                   const uint8_t* __restrict__ inf2, const uint32_t* __restrict__ idx2,
                                                   int flags, int4* __restrict__ fout, int sstride) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const TsPair A = ts_pair(p1, coef1, stride1, inf1, idx1, i);
  TsPair B = ts_pair(p2, coef2, stride2, inf2, idx2, i);
  if (flags & 1) B.y = fp_neg(B.y);
  Fp12 f = f12_one();
  int step = 0;
  for (int b = 62; b >= 0; b--) {
    if (b != 62) f = f12_sqr(f);
    f = ts_line(f, A, step);
    f = ts_line(f, B, step);
    step++;
    if ((hb::X_ABS >> b) & 1) {
      f = ts_line(f, A, step);
      f = ts_line(f, B, step);
      step++;
    }
  }
  if (flags & 2) f = f12_conj(f);
  st12(fout, sstride, i, f);
}

}  // namespace hbs

namespace hbl {

hipError_t ts_miller(hipStream_t s, int n, const void* p1, const void* coef1, int nq1, const uint8_t* inf1,
                     const uint32_t* idx1, const void* p2, const void* coef2, int nq2, const uint8_t* inf2,
                     const uint32_t* idx2, int flags, void* st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hbs::k_ts_miller, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, (const uint32_t*)p1,
                     (const int4*)coef1, pad64(nq1), inf1, idx1, (const uint32_t*)p2, (const int4*)coef2, pad64(nq2),
                     inf2, idx2, flags, (int4*)st, pad64(n));
  return hipGetLastError();
}

}  // namespace hbl
