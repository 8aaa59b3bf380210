// Microbenchmark (round 2): VALU issue on gfx950 for the multi-precision kernels, with the
// occupancy FORCED by a dynamic LDS allocation (160 KiB / waves-per-SIMD per 256-thread block, so
// exactly k blocks fit a CU).  Answers three design questions for the fused pairing kernel:
//   1. how many independent v_mad_u64_u32 chains one wave per SIMD needs to keep the MAD pipe busy;
//   2. the rate of the existing one-chain signed Fp multiplication (hbs::fp_mul_l) against a
//      variant whose a*b column sums are independent of the reduction chain (ILP inside one call);
//   3. the rate of a lazily reduced Fp2 product (5 half-products: 3 Karatsuba products + 2
//      reductions) against three separate Montgomery products.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define HS_MULFN static __device__ __noinline__
#include "../hbbft_amd/csrc/sfp.hpp"

using namespace hbs;

#define CHK(x)                                                                     \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);            \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

// ---------------------------------------------------------------- 1. raw MAD chains
// K independent accumulators, each step acc = acc * x + y through v_mad_u64_u32 (inline asm so the
// compiler cannot fold the chain; the carry-out goes to an SGPR pair the chains do not share).
template <int K>
__global__ void __launch_bounds__(256) k_mad(uint64_t* out, int iters) {
  extern __shared__ uint32_t lds[];
  uint64_t acc[K];
  uint32_t x[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    acc[k] = threadIdx.x + k;
    x[k] = threadIdx.x * 7 + k;
  }
  const uint32_t y = blockIdx.x | 1;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 16; r++)
#pragma unroll
      for (int k = 0; k < K; k++) {
        uint64_t cc;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cc) : "v"(x[k]), "v"(y));
      }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < K; k++) s ^= acc[k];
  if (s == 0x1234567) { lds[0] = 1; out[0] = s + lds[1]; }
}

// ---------------------------------------------------------------- 2. Fp multiplication variants
// 3-accumulator FIPS: column k's a*b sum starts from zero (independent of earlier columns), the
// m*p sum and the carry join it after; same limbs, bounds and output as fp_mul_l.
HS_MULFN Fp fp_mul_l3(HS_P14(x), HS_P14(y)) {
  const Fp a = {{HS_L14(x)}};
  const Fp b = {{HS_L14(y)}};
  int32_t m[NL];
  int64_t carry = 0;
  Fp r;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    int64_t ab = 0, mp = 0;
#pragma unroll
    for (int i = 0; i <= k; i++) ab += (int64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = 0; i < k; i++) mp += (int64_t)m[i] * (int32_t)P_L[k - i];
    int64_t s = ab + mp + carry;
    m[k] = (int32_t)(((uint32_t)s * NP0) & (uint32_t)MASK28);
    s += (int64_t)m[k] * (int32_t)P_L[0];
    carry = s >> 28;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    int64_t ab = 0, mp = 0;
#pragma unroll
    for (int i = k - NL + 1; i < NL; i++) {
      ab += (int64_t)a.l[i] * b.l[k - i];
      mp += (int64_t)m[i] * (int32_t)P_L[k - i];
    }
    const int64_t s = ab + mp + carry;
    r.l[k - NL] = (int32_t)s & MASK28;
    carry = s >> 28;
  }
  r.l[NL - 1] = (int32_t)carry;
  return r;
}

template <int V, int ILP>
__global__ void __launch_bounds__(256) k_fpmul(uint32_t* out, const uint32_t* in, int iters) {
  extern __shared__ uint32_t lds[];
  Fp a[ILP], b;
#pragma unroll
  for (int j = 0; j < NL; j++) {
    b.l[j] = (int32_t)in[(NL + j) * 64 + (threadIdx.x & 63)];
#pragma unroll
    for (int k = 0; k < ILP; k++) a[k].l[j] = (int32_t)in[j * 64 + ((threadIdx.x + k) & 63)];
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < ILP; k++) a[k] = (V == 0) ? fp_mul_l(HS_E14(a[k]), HS_E14(b)) : fp_mul_l3(HS_E14(a[k]), HS_E14(b));
  }
#pragma unroll
  for (int k = 1; k < ILP; k++)
#pragma unroll
    for (int j = 0; j < NL; j++) a[0].l[j] ^= a[k].l[j];
  if (a[0].l[3] == 0x1234567) lds[0] = 1;
  if (blockIdx.x == 0 && threadIdx.x < 64)
#pragma unroll
    for (int j = 0; j < NL; j++) out[j * 64 + threadIdx.x] = (uint32_t)a[0].l[j] + lds[1] * 0;
}

// ---------------------------------------------------------------- 3. lazy Fp2 product
// (a0 + a1 u)(b0 + b1 u): P0 = a0 b0, P1 = a1 b1, P2 = (a0 + a1)(b0 + b1) as column sums, then
// c0 = P0 - P1 and c1 = P2 - P0 - P1 reduced once each (Montgomery, two interleaved m chains).
// Inputs normalised (limbs 0..12 in [0, 2^28)); b is read from this lane's LDS slot (the AMDGPU
// calling convention passes only 32 VGPR arguments).
struct Fp2r { Fp c0, c1; };
HS_MULFN Fp2r f2_mul_lazy(HS_P14(x), HS_P14(z), const int4* __restrict__ slot) {
  const Fp a0 = {{HS_L14(x)}};
  const Fp a1 = {{HS_L14(z)}};
  Fp b0, b1;
  {
    int32_t w[28];
#pragma unroll
    for (int q = 0; q < 7; q++) {
      const int4 v = slot[q];
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < NL; j++) { b0.l[j] = w[j]; b1.l[j] = w[NL + j]; }
  }
  int32_t sa[NL], sb[NL];
#pragma unroll
  for (int j = 0; j < NL; j++) { sa[j] = a0.l[j] + a1.l[j]; sb[j] = b0.l[j] + b1.l[j]; }
  int32_t m0[NL], m1[NL];
  int64_t c0 = 0, c1 = 0;
  Fp2r r;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; k++) {
    const int lo = k < NL ? 0 : k - NL + 1, hi = k < NL ? k : NL - 1;
    int64_t p0 = 0, p1 = 0, p2 = 0, q0 = 0, q1 = 0;
#pragma unroll
    for (int i = lo; i <= hi; i++) {
      p0 += (int64_t)a0.l[i] * b0.l[k - i];
      p1 += (int64_t)a1.l[i] * b1.l[k - i];
      p2 += (int64_t)sa[i] * sb[k - i];
    }
#pragma unroll
    for (int i = lo; i <= (k < NL ? k - 1 : NL - 1); i++) {
      q0 += (int64_t)m0[i] * (int32_t)P_L[k - i];
      q1 += (int64_t)m1[i] * (int32_t)P_L[k - i];
    }
    int64_t s0 = p0 - p1 + q0 + c0;
    int64_t s1 = p2 - p0 - p1 + q1 + c1;
    if (k < NL) {
      m0[k] = (int32_t)(((uint32_t)s0 * NP0) & (uint32_t)MASK28);
      m1[k] = (int32_t)(((uint32_t)s1 * NP0) & (uint32_t)MASK28);
      s0 += (int64_t)m0[k] * (int32_t)P_L[0];
      s1 += (int64_t)m1[k] * (int32_t)P_L[0];
    } else {
      r.c0.l[k - NL] = (int32_t)s0 & MASK28;
      r.c1.l[k - NL] = (int32_t)s1 & MASK28;
    }
    c0 = s0 >> 28;
    c1 = s1 >> 28;
  }
  r.c0.l[NL - 1] = (int32_t)c0;
  r.c1.l[NL - 1] = (int32_t)c1;
  return r;
}

// V = 0: f2_mul (three fp_mul_l), V = 1: f2_mul_lazy
template <int V>
__global__ void __launch_bounds__(256) k_f2mul(uint32_t* out, const uint32_t* in, int iters) {
  extern __shared__ int4 slds[];
  Fp2 a, b;
#pragma unroll
  for (int j = 0; j < NL; j++) {
    a.c0.l[j] = (int32_t)in[j * 64 + (threadIdx.x & 63)];
    a.c1.l[j] = (int32_t)in[(NL + j) * 64 + (threadIdx.x & 63)];
    b.c0.l[j] = (int32_t)in[j * 64 + ((threadIdx.x + 5) & 63)];
    b.c1.l[j] = (int32_t)in[(NL + j) * 64 + ((threadIdx.x + 9) & 63)];
  }
  int4* slot = slds + threadIdx.x * 7;
  {
    int32_t w[28];
#pragma unroll
    for (int j = 0; j < NL; j++) { w[j] = b.c0.l[j]; w[NL + j] = b.c1.l[j]; }
#pragma unroll
    for (int q = 0; q < 7; q++) slot[q] = make_int4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
  for (int it = 0; it < iters; it++) {
    if (V == 0) {
      a = f2_mul(a, b);
    } else {
      Fp2r r = f2_mul_lazy(HS_E14(a.c0), HS_E14(a.c1), slot);
      a.c0 = r.c0;
      a.c1 = r.c1;
    }
    fp_norm(a.c0);  // keep the chain's inputs normalised (f2_mul's c0 is fp_sub'ed already)
    fp_norm(a.c1);
  }
  if (blockIdx.x == 0 && threadIdx.x < 64)
#pragma unroll
    for (int j = 0; j < NL; j++) {
      out[j * 64 + threadIdx.x] = (uint32_t)a.c0.l[j];
      out[(NL + j) * 64 + threadIdx.x] = (uint32_t)a.c1.l[j];
    }
}

// ---------------------------------------------------------------- driver
template <typename K, typename... A>
static float run(K kern, int wps, int rounds, A... args) {
  const int cus = 256;
  const size_t lds = (160 * 1024) / wps - 1024;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(cus * wps * rounds), dim3(256), lds, 0, args...);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(cus * wps * rounds), dim3(256), lds, 0, args...);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs %d\n", p.gcnArchName, p.multiProcessorCount);
  uint32_t hin[28 * 64];
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < 28 * 64; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    hin[i] = (uint32_t)s & 0x0fffffffu;
  }
  for (int l = 0; l < 64; l++) { hin[13 * 64 + l] &= 0xffff; hin[27 * 64 + l] &= 0xffff; }
  uint32_t *din, *dout;
  uint64_t* d64;
  CHK(hipMalloc(&din, sizeof(hin)));
  CHK(hipMalloc(&dout, 64 * 64 * 4));
  CHK(hipMalloc(&d64, 64));
  CHK(hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice));
  const int rounds = 4;
  for (int wps : {1, 2, 4, 8}) {
    const double lanes = 256.0 * wps * rounds * 256;
    const int it = 512;
    float ms = run(k_mad<1>, wps, rounds, d64, it);
    printf("mad chains=1 wps=%d: %7.3f ms %6.2f T mad/s\n", wps, ms, lanes * it * 16 * 1 / ms / 1e9);
    ms = run(k_mad<2>, wps, rounds, d64, it);
    printf("mad chains=2 wps=%d: %7.3f ms %6.2f T mad/s\n", wps, ms, lanes * it * 16 * 2 / ms / 1e9);
    ms = run(k_mad<4>, wps, rounds, d64, it);
    printf("mad chains=4 wps=%d: %7.3f ms %6.2f T mad/s\n", wps, ms, lanes * it * 16 * 4 / ms / 1e9);
    ms = run(k_mad<8>, wps, rounds, d64, it);
    printf("mad chains=8 wps=%d: %7.3f ms %6.2f T mad/s\n", wps, ms, lanes * it * 16 * 8 / ms / 1e9);
  }
  for (int wps : {1, 2, 4}) {
    const double lanes = 256.0 * wps * rounds * 256;
    const int it = 200;
    float ms = run(k_fpmul<0, 1>, wps, rounds, dout, din, it);
    printf("fp_mul_l  ILP1 wps=%d: %7.3f ms %6.2f G Fp-mul/s\n", wps, ms, lanes * it / ms / 1e6);
    ms = run(k_fpmul<0, 2>, wps, rounds, dout, din, it);
    printf("fp_mul_l  ILP2 wps=%d: %7.3f ms %6.2f G Fp-mul/s\n", wps, ms, lanes * it * 2 / ms / 1e6);
    ms = run(k_fpmul<1, 1>, wps, rounds, dout, din, it);
    printf("fp_mul_l3 ILP1 wps=%d: %7.3f ms %6.2f G Fp-mul/s\n", wps, ms, lanes * it / ms / 1e6);
    ms = run(k_fpmul<1, 2>, wps, rounds, dout, din, it);
    printf("fp_mul_l3 ILP2 wps=%d: %7.3f ms %6.2f G Fp-mul/s\n", wps, ms, lanes * it * 2 / ms / 1e6);
    ms = run(k_f2mul<0>, wps, rounds, dout, din, it);
    printf("f2_mul (3 fp_mul) wps=%d: %7.3f ms %6.2f G Fp2-mul/s\n", wps, ms, lanes * it / ms / 1e6);
    ms = run(k_f2mul<1>, wps, rounds, dout, din, it);
    printf("f2_mul_lazy       wps=%d: %7.3f ms %6.2f G Fp2-mul/s\n", wps, ms, lanes * it / ms / 1e6);
  }
  // correctness cross-check of the variants on lane 0..63 (the host compares the dumps)
  uint32_t h0[28 * 64], h1[28 * 64];
  run(k_fpmul<0, 1>, 1, 1, dout, din, 3);
  CHK(hipMemcpy(h0, dout, 14 * 64 * 4, hipMemcpyDeviceToHost));
  run(k_fpmul<1, 1>, 1, 1, dout, din, 3);
  CHK(hipMemcpy(h1, dout, 14 * 64 * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < 14 * 64; i++) bad += h0[i] != h1[i];
  printf("CHECK fp_mul_l3 vs fp_mul_l: %d differing words\n", bad);
  run(k_f2mul<0>, 1, 1, dout, din, 3);
  CHK(hipMemcpy(h0, dout, 28 * 64 * 4, hipMemcpyDeviceToHost));
  run(k_f2mul<1>, 1, 1, dout, din, 3);
  CHK(hipMemcpy(h1, dout, 28 * 64 * 4, hipMemcpyDeviceToHost));
  // values may differ by a multiple of p (different reduction paths): compare mod p on the host
  printf("DUMP f2 first lane c0: ");
  for (int j = 0; j < 14; j++) printf("%08x/%08x ", h0[j * 64], h1[j * 64]);
  printf("\n");
  return 0;
}
