// Issue rate of v_mul_lo_u32 vs v_mad_u64_u32 on gfx950: 8 independent chains per lane, 8 waves per
// SIMD; a quarter-rate instruction shows as 1/4 of the full-rate throughput.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void __launch_bounds__(256) k_mullo(uint32_t* out, int iters, uint32_t c) {
  uint32_t x[8];
  for (int k = 0; k < 8; k++) x[k] = threadIdx.x + k;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[k]) : "s"(c));
  }
  uint32_t s = 0;
  for (int k = 0; k < 8; k++) s ^= x[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_madlo(uint32_t* out, int iters, uint32_t c) {
  uint64_t x[8];
  for (int k = 0; k < 8; k++) x[k] = threadIdx.x + k;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      uint32_t lo = (uint32_t)x[k];
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(x[k]), "=s"(cc) : "v"(lo), "s"(c));
    }
  }
  uint32_t s = 0;
  for (int k = 0; k < 8; k++) s ^= (uint32_t)x[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  uint32_t* d;
  const int blocks = 256 * 4 * 8 / 4;  // 8 waves per SIMD (4 waves per block of 256)
  hipMalloc(&d, (size_t)blocks * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 4096;
  for (int rep = 0; rep < 2; rep++) {
    for (int kind = 0; kind < 2; kind++) {
      hipEventRecord(a);
      if (kind == 0) hipLaunchKernelGGL(k_mullo, dim3(blocks), dim3(256), 0, 0, d, iters, 0x9E3779B9u);
      else hipLaunchKernelGGL(k_madlo, dim3(blocks), dim3(256), 0, 0, d, iters, 0x9E3779B9u);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double ops = (double)blocks * 256 * iters * 8;
      printf("%s: %.3f ms  %.2f T ops/s\n", kind ? "v_mad_u64_u32" : "v_mul_lo_u32", ms, ops / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
