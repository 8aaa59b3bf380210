// Microbenchmark (round 6): what one wave per SIMD can issue on gfx950 -- the latency kernels
// (k_wave, the decoders) run there.  v_mad_u64_u32 at one wave per SIMD reaches ~17.5 T MAD/s
// (profiles/r02/ubench_v2_mad.txt: ~9 cycles per wave instruction) against ~38 T at 8 waves; the
// question here is whether other VALU work (adds, logic, 32-bit multiplies) and LDS-crossbar
// shuffles issue in the MAD gaps for free, i.e. whether a latency kernel's cost is its MAD count or
// its instruction count.  Occupancy is forced to one wave per SIMD with a 40 KiB dynamic LDS
// allocation per 64-thread block (4 blocks per CU, one per SIMD); 1,024 blocks.
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench_issue tools/ubench_issue.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHK(x)                                                                \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);       \
      return 1;                                                               \
    }                                                                         \
  } while (0)

// NM MAD chains and NA independent add chains, interleaved: per round every MAD chain takes one
// v_mad_u64_u32 and every add chain NPER v_add_u32 (or v_xor / v_mul_lo / ds_bpermute by KIND).
template <int NM, int NA, int NPER, int KIND>
__global__ void __launch_bounds__(64) k_mix(uint64_t* out, int iters) {
  extern __shared__ uint32_t lds[];
  uint64_t acc[NM > 0 ? NM : 1];
  uint32_t x[NM > 0 ? NM : 1];
  uint32_t a[NA > 0 ? NA : 1];
#pragma unroll
  for (int k = 0; k < NM; k++) {
    acc[k] = threadIdx.x + k;
    x[k] = threadIdx.x * 7 + k;
  }
#pragma unroll
  for (int k = 0; k < NA; k++) a[k] = threadIdx.x * 3 + k;
  const uint32_t y = blockIdx.x | 1;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
#pragma unroll
      for (int k = 0; k < NM; k++) {
        uint64_t cc;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cc) : "v"(x[k]), "v"(y));
      }
#pragma unroll
      for (int k = 0; k < NA; k++)
#pragma unroll
        for (int q = 0; q < NPER; q++) {
          if (KIND == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(y));
          if (KIND == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[k]) : "v"(y));
          if (KIND == 2) asm volatile("ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)" : "+v"(a[k]) : "v"(y));
          if (KIND == 3) asm volatile("ds_bpermute_b32 %0, %1, %0" : "+v"(a[k]) : "v"(y));
          if (KIND == 4) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(acc[k % (NM > 0 ? NM : 1)]));
        }
    }
    if (KIND == 3) asm volatile("s_waitcnt lgkmcnt(0)");
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < NM; k++) s ^= acc[k];
#pragma unroll
  for (int k = 0; k < NA; k++) s ^= a[k];
  if (s == 0x1234567) {
    lds[0] = 1;
    out[0] = s + lds[1];
  }
}

template <int NM, int NA, int NPER, int KIND>
int run(const char* name, uint64_t* d, int iters) {
  const size_t lds = 40 * 1024;
  hipLaunchKernelGGL((k_mix<NM, NA, NPER, KIND>), dim3(1024), dim3(64), lds, 0, d, 2);
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL((k_mix<NM, NA, NPER, KIND>), dim3(1024), dim3(64), lds, 0, d, iters);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  const double rounds = (double)iters * 16;
  const double ns_per_round = ms * 1e6 / rounds;
  // wave instructions per round: NM MADs + NA * NPER others
  printf("%-44s %8.3f ms  %7.2f ns/round  %6.2f ns per instr  (%d MAD + %d other per round)\n", name, ms, ns_per_round,
         ns_per_round / (NM + NA * NPER), NM, NA * NPER);
  return 0;
}

int main() {
  uint64_t* d;
  CHK(hipMalloc(&d, 64));
  const int it = 20000;
  run<8, 0, 1, 0>("8 MAD chains", d, it);
  run<1, 0, 1, 0>("1 MAD chain", d, it);
  run<0, 8, 1, 0>("8 add chains", d, it);
  run<0, 1, 1, 0>("1 add chain", d, it);
  run<8, 8, 1, 0>("8 MAD + 8 add (1 each)", d, it);
  run<8, 8, 2, 0>("8 MAD + 16 add (2 per chain)", d, it);
  run<8, 4, 1, 0>("8 MAD + 4 add", d, it);
  run<8, 8, 1, 1>("8 MAD + 8 mul_lo", d, it);
  run<0, 8, 1, 1>("8 mul_lo chains", d, it);
  run<8, 8, 1, 4>("8 MAD + 8 lshl_b64", d, it);
  run<0, 8, 1, 3>("8 bpermute (batched wait)", d, it);
  run<8, 8, 1, 3>("8 MAD + 8 bpermute (batched wait)", d, it);
  run<0, 1, 1, 2>("1 bpermute + wait (latency)", d, it / 4);
  return 0;
}
