// One-thread-per-check pairing kernels (HBH_IMPL_THREAD, kernels.hpp) and their host launchers.
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "launch.hpp"

namespace hbl {

static inline dim3 grid_for(int n) { return dim3((unsigned)((n + 255) / 256)); }

hipError_t pairing_eq(hipStream_t s, int n, const void* p1, const void* coef1, int nq1, const uint8_t* inf1,
                      const uint32_t* idx1, const void* p2, const void* coef2, int nq2, const uint8_t* inf2,
                      const uint32_t* idx2, uint8_t* verdict) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_pairing_eq, grid_for(n), dim3(256), 0, s, n, (const uint32_t*)p1, (const uint4*)coef1,
                     pad64(nq1), inf1, idx1, (const uint32_t*)p2, (const uint4*)coef2, pad64(nq2), inf2, idx2, verdict);
  return hipGetLastError();
}

hipError_t pairing_value(hipStream_t s, int n, const void* p, const void* coef, const uint8_t* inf, uint32_t* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb::k_dbg_pairing, grid_for(n), dim3(256), 0, s, n, (const uint32_t*)p, (const uint4*)coef,
                     pad64(n), inf, out);
  return hipGetLastError();
}

}  // namespace hbl
