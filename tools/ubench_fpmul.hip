// Microbenchmark: Montgomery Fp (BLS12-381) multiplication throughput on gfx950 for three
// limb/codegen strategies. Used to choose the field representation.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

static constexpr uint32_t P32[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
#define NP32 0xfffcfffdu
static constexpr uint32_t P28[14] = {0xfffaaabu, 0xfefffffu, 0x3ffffb9u, 0xfffeb15u, 0x6241eabu, 0xa0f6b0fu, 0xf6730d2u, 0xf38512bu, 0x4774b84u, 0x4bacd76u, 0xba7b643u, 0xe69a4b1u, 0x1ea397fu, 0x001a011u};
#define NP28 0xffcfffdu

// (A) CIOS, plain C, 32-bit limbs
__device__ __forceinline__ void mm_cios(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  const int NL = 12;
  uint32_t t[NL + 2];
#pragma unroll
  for (int j = 0; j < NL + 2; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) { c = (uint64_t)a[j] * b[i] + t[j] + (c >> 32); t[j] = (uint32_t)c; }
    c = (uint64_t)t[NL] + (c >> 32); t[NL] = (uint32_t)c; t[NL + 1] = (uint32_t)(c >> 32);
    uint32_t m = t[0] * NP32;
    c = (uint64_t)m * P32[0] + t[0];
#pragma unroll
    for (int j = 1; j < NL; j++) { c = (uint64_t)m * P32[j] + t[j] + (c >> 32); t[j - 1] = (uint32_t)c; }
    c = (uint64_t)t[NL] + (c >> 32); t[NL - 1] = (uint32_t)c; t[NL] = t[NL + 1] + (uint32_t)(c >> 32);
  }
  uint32_t s[NL]; uint64_t br = 0;
#pragma unroll
  for (int j = 0; j < NL; j++) { uint64_t d = (uint64_t)t[j] - P32[j] - br; s[j] = (uint32_t)d; br = (d >> 63); }
  bool ge = t[NL] || !br;
#pragma unroll
  for (int j = 0; j < NL; j++) r[j] = ge ? s[j] : t[j];
}

// (B) FIPS with inline-asm mad carry-out, 32-bit limbs
__device__ __forceinline__ void mac_v(uint64_t& acc, uint32_t& ovf, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(acc), "=s"(cc) : "v"(a), "v"(b), "v"(acc));
  asm("v_addc_co_u32 %0, %1, 0, %2, %3" : "=v"(ovf), "=s"(cc) : "v"(ovf), "s"(cc));
}
__device__ __forceinline__ void mac_s(uint64_t& acc, uint32_t& ovf, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(acc), "=s"(cc) : "v"(a), "s"(b), "v"(acc));
  asm("v_addc_co_u32 %0, %1, 0, %2, %3" : "=v"(ovf), "=s"(cc) : "v"(ovf), "s"(cc));
}
__device__ __forceinline__ void mm_fips(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  const int NL = 12;
  uint32_t m[NL]; uint64_t acc = 0; uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) mac_v(acc, ovf, a[i], b[k - i]);
#pragma unroll
    for (int i = 0; i < k; i++) mac_s(acc, ovf, m[i], P32[k - i]);
    m[k] = (uint32_t)acc * NP32;
    mac_s(acc, ovf, m[k], P32[0]);
    acc = (acc >> 32) | ((uint64_t)ovf << 32); ovf = 0;
  }
  uint32_t t[NL + 1];
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int i = k - NL + 1; i < NL; i++) { mac_v(acc, ovf, a[i], b[k - i]); mac_s(acc, ovf, m[i], P32[k - i]); }
    t[k - NL] = (uint32_t)acc; acc = (acc >> 32) | ((uint64_t)ovf << 32); ovf = 0;
  }
  t[NL - 1] = (uint32_t)acc; t[NL] = (uint32_t)(acc >> 32);
  uint32_t s[NL]; uint64_t br = 0;
#pragma unroll
  for (int j = 0; j < NL; j++) { uint64_t d = (uint64_t)t[j] - P32[j] - br; s[j] = (uint32_t)d; br = (d >> 63); }
  bool ge = t[NL] || !br;
#pragma unroll
  for (int j = 0; j < NL; j++) r[j] = ge ? s[j] : t[j];
}

// (C) FIPS, radix 2^28, 14 limbs, lazy (output < 2p, no final subtraction)
__device__ __forceinline__ void mm28(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  const int NL = 14;
  uint32_t m[NL]; uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc += (uint64_t)a[i] * b[k - i];
#pragma unroll
    for (int i = 0; i < k; i++) acc += (uint64_t)m[i] * P28[k - i];
    m[k] = ((uint32_t)acc * NP28) & 0x0fffffffu;
    acc += (uint64_t)m[k] * P28[0];
    acc >>= 28;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
#pragma unroll
    for (int i = k - NL + 1; i < NL; i++) { acc += (uint64_t)a[i] * b[k - i]; acc += (uint64_t)m[i] * P28[k - i]; }
    r[k - NL] = (uint32_t)acc & 0x0fffffffu; acc >>= 28;
  }
  r[NL - 1] = (uint32_t)acc;
}

// (D) operand-scanning CIOS, radix 2^28, 14 limbs, 64-bit column accumulators: every row is 28
// independent v_mad_u64_u32 (ILP inside one product); only m_i and one carry are serial.
__device__ __forceinline__ void mm28os(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  const int NL = 14;
  uint64_t t[NL];
#pragma unroll
  for (int j = 0; j < NL; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
#pragma unroll
    for (int j = 0; j < NL; j++) t[j] += (uint64_t)a[j] * b[i];
    const uint32_t m = ((uint32_t)t[0] * NP28) & 0x0fffffffu;
    const uint64_t c = (t[0] + (uint64_t)m * P28[0]) >> 28;
#pragma unroll
    for (int j = 1; j < NL; j++) t[j - 1] = t[j] + (uint64_t)m * P28[j];
    t[NL - 1] = 0;
    t[0] += c;
  }
#pragma unroll
  for (int j = 0; j < NL - 1; j++) { t[j + 1] += t[j] >> 28; r[j] = (uint32_t)t[j] & 0x0fffffffu; }
  r[NL - 1] = (uint32_t)t[NL - 1];
}
template <int V, int NL, int ILP>
__global__ void __launch_bounds__(256) kbench(uint32_t* out, const uint32_t* in, int n, int iters) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a[ILP][NL], b[NL];
#pragma unroll
  for (int j = 0; j < NL; j++) {
    b[j] = in[(NL + j) * 64 + (i & 63)];
#pragma unroll
    for (int k = 0; k < ILP; k++) a[k][j] = in[j * 64 + ((i + k) & 63)];
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < ILP; k++) {
      if (V == 0) mm_cios(a[k], a[k], b);
      if (V == 1) mm_fips(a[k], a[k], b);
      if (V == 2) mm28(a[k], a[k], b);
      if (V == 3) mm28os(a[k], a[k], b);
    }
  }
  // every chain feeds the output, otherwise the compiler deletes chains 1..ILP-1
#pragma unroll
  for (int k = 1; k < ILP; k++)
#pragma unroll
    for (int j = 0; j < NL; j++) a[0][j] ^= a[k][j];
  if (i < n) {
#pragma unroll
    for (int j = 0; j < NL; j++) out[j * n + i] = a[0][j];
  }
}

template <int V, int NL, int ILP>
void run(const char* name, uint32_t* dout, uint32_t* din, int cus, int iters) {
  for (int wps : {1, 2, 4, 8}) {
    int blocks = cus * wps, threads = 256;
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((kbench<V, NL, ILP>), dim3(blocks), dim3(threads), 0, 0, dout, din, 64, iters);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((kbench<V, NL, ILP>), dim3(blocks), dim3(threads), 0, 0, dout, din, 64, iters);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    double muls = (double)blocks * threads * iters * ILP;
    printf("%-10s ILP=%d waves/SIMD=%d: %8.3f ms  %7.2f G Fp-mul/s\n", name, ILP, wps, ms, muls / ms / 1e6);
  }
  uint32_t h[14];
  (void)hipMemcpy(h, dout, 4, hipMemcpyDeviceToHost);
  for (int j = 0; j < NL; j++) (void)hipMemcpy(&h[j], dout + j * 64, 4, hipMemcpyDeviceToHost);
  printf("CHECK %s ILP%d", name, ILP);
  for (int j = 0; j < NL; j++) printf(" %08x", h[j]);
  printf("\n");
}

int main() {
  hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
  int cus = p.multiProcessorCount;
  printf("device %s CUs %d\n", p.gcnArchName, cus);
  uint32_t hin[28 * 64];
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < 28 * 64; i++) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; hin[i] = (uint32_t)s & 0x0fffffffu; }
  for (int l = 0; l < 64; l++) { hin[11 * 64 + l] &= 0x00ffffff; hin[23 * 64 + l] &= 0x00ffffff; hin[13*64+l] &= 0xffff; hin[27*64+l] &= 0xffff; }
  FILE* f = fopen("gpurun_out/fpmul_in.txt", "w");
  for (int i = 0; i < 28 * 64; i++) fprintf(f, "%08x\n", hin[i]);
  fclose(f);
  uint32_t *din, *dout;
  (void)hipMalloc(&din, sizeof(hin)); (void)hipMalloc(&dout, 14 * 1024 * 1024 * 4);
  (void)hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice);
  int iters = 1000;
  if (getenv("UB_ALL")) {
    run<0, 12, 1>("cios32", dout, din, cus, iters);
    run<0, 12, 2>("cios32", dout, din, cus, iters);
    run<1, 12, 1>("fips32asm", dout, din, cus, iters);
    run<1, 12, 2>("fips32asm", dout, din, cus, iters);
  }
  run<3, 14, 1>("os28", dout, din, cus, iters);
  run<3, 14, 2>("os28", dout, din, cus, iters);
  run<2, 14, 1>("fips28", dout, din, cus, iters);
  run<2, 14, 2>("fips28", dout, din, cus, iters);
  run<2, 14, 4>("fips28", dout, din, cus, iters);
  return 0;
}
