// Microbenchmark: peak 32x32->64 multiply-add rate on gfx950 (roofline denominator).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

template<int NACC>
__global__ void k_mad64(uint64_t* out, uint32_t a, uint32_t b, int iters) {
  uint64_t acc[NACC];
  #pragma unroll
  for (int i = 0; i < NACC; i++) acc[i] = threadIdx.x + i;
  uint32_t x = a + threadIdx.x, y = b ^ blockIdx.x;
  for (int it = 0; it < iters; it++) {
    #pragma unroll
    for (int i = 0; i < NACC; i++) {
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(x), "v"(y) : "vcc");
    }
  }
  uint64_t s = 0;
  #pragma unroll
  for (int i = 0; i < NACC; i++) s += acc[i];
  if (s == 0x123456789ull) out[0] = s;
}

template<int NACC>
__global__ void k_mullohi(uint64_t* out, uint32_t a, uint32_t b, int iters) {
  uint32_t lo[NACC], hi[NACC];
  #pragma unroll
  for (int i = 0; i < NACC; i++) { lo[i] = threadIdx.x + i; hi[i] = i; }
  uint32_t x = a + threadIdx.x, y = b ^ blockIdx.x;
  for (int it = 0; it < iters; it++) {
    #pragma unroll
    for (int i = 0; i < NACC; i++) {
      asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(lo[i]) : "v"(x), "v"(lo[i]));
      asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(hi[i]) : "v"(y), "v"(hi[i]));
    }
  }
  uint64_t s = 0;
  #pragma unroll
  for (int i = 0; i < NACC; i++) s += lo[i] + hi[i];
  if (s == 0x123456789ull) out[0] = s;
}

template<int NACC>
__global__ void k_fma64(double* out, double a, double b, int iters) {
  double acc[NACC];
  #pragma unroll
  for (int i = 0; i < NACC; i++) acc[i] = threadIdx.x + i;
  double x = a + threadIdx.x, y = b;
  for (int it = 0; it < iters; it++) {
    #pragma unroll
    for (int i = 0; i < NACC; i++) {
      asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(x), "v"(y));
    }
  }
  double s = 0;
  #pragma unroll
  for (int i = 0; i < NACC; i++) s += acc[i];
  if (s == 1234.5) out[0] = s;
}

template<int NACC>
__global__ void k_add32(uint32_t* out, uint32_t a, int iters) {
  uint32_t acc[NACC];
  #pragma unroll
  for (int i = 0; i < NACC; i++) acc[i] = threadIdx.x + i;
  uint32_t x = a + threadIdx.x;
  for (int it = 0; it < iters; it++) {
    #pragma unroll
    for (int i = 0; i < NACC; i++) {
      asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(acc[i]) : "v"(x) : "vcc");
    }
  }
  uint32_t s = 0;
  #pragma unroll
  for (int i = 0; i < NACC; i++) s += acc[i];
  if (s == 0x12345) out[0] = s;
}

template<typename K, typename... A>
double timeit(K kern, int blocks, int threads, A... args) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, args...);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, args...);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 3.0;
}

int main() {
  void* buf; CHK(hipMalloc(&buf, 1024));
  int iters = 4096;
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  int cus = p.multiProcessorCount;
  // waves per SIMD: blocks of 256 threads (4 waves, one per SIMD) x k per CU
  for (int wps : {1, 2, 4, 8}) {
    int blocks = cus * wps;
    double n = (double)blocks * 256 * iters;
    double ms = timeit(k_mad64<8>, blocks, 256, (uint64_t*)buf, 3u, 5u, iters);
    printf("mad_u64_u32  acc=8  waves/SIMD=%d : %.3f ms  %.2f T mad/s\n", wps, ms, n * 8 / ms / 1e9);
    ms = timeit(k_mad64<2>, blocks, 256, (uint64_t*)buf, 3u, 5u, iters);
    printf("mad_u64_u32  acc=2  waves/SIMD=%d : %.3f ms  %.2f T mad/s\n", wps, ms, n * 2 / ms / 1e9);
    ms = timeit(k_mad64<1>, blocks, 256, (uint64_t*)buf, 3u, 5u, iters);
    printf("mad_u64_u32  acc=1  waves/SIMD=%d : %.3f ms  %.2f T mad/s\n", wps, ms, n * 1 / ms / 1e9);
    ms = timeit(k_mullohi<8>, blocks, 256, (uint64_t*)buf, 3u, 5u, iters);
    printf("mul_lo+hi    acc=8  waves/SIMD=%d : %.3f ms  %.2f T pairs/s\n", wps, ms, n * 8 / ms / 1e9);
    ms = timeit(k_fma64<8>, blocks, 256, (double*)buf, 1.0, 0.5, iters);
    printf("fma_f64      acc=8  waves/SIMD=%d : %.3f ms  %.2f T fma/s\n", wps, ms, n * 8 / ms / 1e9);
    ms = timeit(k_add32<8>, blocks, 256, (uint32_t*)buf, 3u, iters);
    printf("add_co_u32   acc=8  waves/SIMD=%d : %.3f ms  %.2f T add/s\n", wps, ms, n * 8 / ms / 1e9);
  }
  return 0;
}
