// HBH_IMPL_THREAD_SIGNED, stages 2-5: final exponentiation f^(3 (p^12 - 1) / r), one thread per
// check, signed limbs.  Same chain as hb::final_exp_x3 (pairing.hpp):
//   f2 = f^((p^6 - 1)(p^2 + 1));  a = (f2^(x-1))^(x-1);  b = a^x frob1(a);
//   c = (b^x)^x frob2(b) conj(b);  e = c f2^3.
#define HS_MULFN static __device__ __noinline__
#include "launch.hpp"
#include "sthread.hpp"

namespace hbs {

__global__ void __launch_bounds__(256) k_ts_easy(int n, const int4* __restrict__ fin, int4* __restrict__ fout, int ss) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fp12 f = ld12(fin, ss, i);
  const Fp12 f1 = f12_mul(f12_conj(f), f12_inv(f));
  st12(fout, ss, i, f12_mul(f12_frob2(f1), f1));
}

// conj(f^|x|) = f^x, conj(f^(|x|+1)) = f^(x-1) for f in the cyclotomic subgroup
__global__ void __launch_bounds__(256) k_ts_exp(int n, const int4* __restrict__ fin, int4* __restrict__ fout, int ss,
                                                int plus1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fp12 base = ld12(fin, ss, i);
  const uint64_t e = plus1 ? hb::X_ABS + 1 : hb::X_ABS;
  Fp12 r = base;
  for (int k = 62; k >= 0; k--) {
    r = f12_cyclo_sqr(r);
    if ((e >> k) & 1) r = f12_mul(r, base);
  }
  st12(fout, ss, i, f12_conj(r));
}

// mode 1: t frob1(a);  mode 2: t frob2(a) conj(a)
__global__ void __launch_bounds__(256) k_ts_glue(int n, const int4* __restrict__ t, const int4* __restrict__ a,
                                                 int4* __restrict__ fout, int ss, int mode) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fp12 av = ld12(a, ss, i);
  Fp12 r = f12_mul(ld12(t, ss, i), mode == 1 ? f12_frob1(av) : f12_frob2(av));
  if (mode == 2) r = f12_mul(r, f12_conj(av));
  st12(fout, ss, i, r);
}

// e = c f2^3; verdict = (e == 1), or e as canonical words (tower storage order, 144 words)
__global__ void __launch_bounds__(256) k_ts_verdict(int n, const int4* __restrict__ c, const int4* __restrict__ f2,
                                                    int ss, uint8_t* __restrict__ verdict,
                                                    uint32_t* __restrict__ value_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fp12 g = ld12(f2, ss, i);
  const Fp12 e = f12_mul(ld12(c, ss, i), f12_mul(f12_cyclo_sqr(g), g));
  if (value_out) {
    uint32_t* o = value_out + (size_t)i * 144;
    fp_to_words(e.c0.c0.c0, o + 0);
    fp_to_words(e.c0.c0.c1, o + 12);
    fp_to_words(e.c0.c1.c0, o + 24);
    fp_to_words(e.c0.c1.c1, o + 36);
    fp_to_words(e.c0.c2.c0, o + 48);
    fp_to_words(e.c0.c2.c1, o + 60);
    fp_to_words(e.c1.c0.c0, o + 72);
    fp_to_words(e.c1.c0.c1, o + 84);
    fp_to_words(e.c1.c1.c0, o + 96);
    fp_to_words(e.c1.c1.c1, o + 108);
    fp_to_words(e.c1.c2.c0, o + 120);
    fp_to_words(e.c1.c2.c1, o + 132);
  }
  if (verdict) verdict[i] = f12_is_one(e) ? 1 : 0;
}

}  // namespace hbs

namespace hbl {

size_t ts_state_bytes(int n) { return (size_t)hbs::ST_Q4 * 16 * pad64(n); }

hipError_t ts_final_exp(hipStream_t s, int n, void* w0, void* w1, void* w2, void* w3, uint8_t* verdict,
                        uint32_t* value_out) {
  if (n <= 0) return hipSuccess;
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
  const int ss = pad64(n);
  int4 *f = (int4*)w0, *f2 = (int4*)w1, *x = (int4*)w2, *y = (int4*)w3;
  hipLaunchKernelGGL(hbs::k_ts_easy, g, b, 0, s, n, (const int4*)f, f2, ss);         // f2
  hipLaunchKernelGGL(hbs::k_ts_exp, g, b, 0, s, n, (const int4*)f2, x, ss, 1);       // f2^(x-1)
  hipLaunchKernelGGL(hbs::k_ts_exp, g, b, 0, s, n, (const int4*)x, y, ss, 1);        // a
  hipLaunchKernelGGL(hbs::k_ts_exp, g, b, 0, s, n, (const int4*)y, x, ss, 0);        // a^x
  hipLaunchKernelGGL(hbs::k_ts_glue, g, b, 0, s, n, (const int4*)x, (const int4*)y, f, ss, 1);  // b
  hipLaunchKernelGGL(hbs::k_ts_exp, g, b, 0, s, n, (const int4*)f, x, ss, 0);        // b^x
  hipLaunchKernelGGL(hbs::k_ts_exp, g, b, 0, s, n, (const int4*)x, y, ss, 0);        // b^(x^2)
  hipLaunchKernelGGL(hbs::k_ts_glue, g, b, 0, s, n, (const int4*)y, (const int4*)f, x, ss, 2);  // c
  hipLaunchKernelGGL(hbs::k_ts_verdict, g, b, 0, s, n, (const int4*)x, (const int4*)f2, ss, verdict, value_out);
  return hipGetLastError();
}

}  // namespace hbl
