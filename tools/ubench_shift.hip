// Microbenchmark (round 4): issue cost of the 64-bit arithmetic shift that carries a product column
// (acc >>= 28 -> v_ashrrev_i64) against the two 32-bit instructions that could replace it
// (v_alignbit_b32 for the low word, v_ashrrev_i32 for the high word) and a full-rate v_and_b32,
// 8 independent chains per wave, 2 and 4 waves per SIMD (occupancy forced by LDS).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);          \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

template <int OP>
__global__ void __launch_bounds__(256) k(uint64_t* out, int iters) {
  extern __shared__ uint32_t lds[];
  uint64_t v[8];
#pragma unroll
  for (int c = 0; c < 8; c++) v[c] = ((uint64_t)threadIdx.x << 40) | (blockIdx.x + c);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 16; r++)
#pragma unroll
      for (int c = 0; c < 8; c++) {
        if (OP == 0) {
          asm volatile("v_ashrrev_i64 %0, 28, %0" : "+v"(v[c]));
        } else if (OP == 1) {
          uint32_t lo = (uint32_t)v[c], hi = (uint32_t)(v[c] >> 32);
          asm volatile("v_alignbit_b32 %0, %1, %0, 28\n\tv_ashrrev_i32 %1, 28, %1" : "+v"(lo), "+v"(hi));
          v[c] = ((uint64_t)hi << 32) | lo;
        } else {
          uint32_t lo = (uint32_t)v[c];
          asm volatile("v_and_b32 %0, 0x7fffffff, %0" : "+v"(lo));
          v[c] = (v[c] & 0xffffffff00000000ull) | lo;
        }
      }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < 8; c++) s ^= v[c];
  if (s == 0x1234567) { lds[0] = 1; out[0] = s + lds[1]; }
}

template <int OP>
int run(const char* name, int wps, int ninst) {
  uint64_t* out;
  CHK(hipMalloc(&out, 64));
  const int iters = 2000;
  const size_t lds = 160 * 1024 / (wps * 4) * 4 / 4;  // (waves per SIMD) blocks of 4 waves per CU
  const int blocks = 256 * wps;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), lds, 0, out, 10);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), lds, 0, out, iters);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  const double winst = (double)blocks * 4 * iters * 16 * 8 * ninst;  // wave instructions
  // cycles per wave-instruction per SIMD at 2.4 GHz: 1,024 SIMDs
  printf("%-28s wps=%d  %.3f ms  %.2f cycles per wave-instruction per SIMD\n", name, wps, ms,
         ms * 1e-3 * 2.4e9 * 1024 / winst);
  CHK(hipFree(out));
  return 0;
}

int main() {
  for (int w : {2, 4}) {
    if (run<0>("v_ashrrev_i64 (1 instr)", w, 1)) return 1;
    if (run<1>("v_alignbit + v_ashrrev_i32", w, 2)) return 1;
    if (run<2>("v_and_b32 (1 instr)", w, 1)) return 1;
  }
  return 0;
}
