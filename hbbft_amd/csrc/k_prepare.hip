// G2 line-table walk (k_g2_prepare, lines.hpp) and its host launcher: stage 1 of every pairing
// implementation.
#include <hip/hip_runtime.h>

#include "launch.hpp"
#include "lines.hpp"

namespace hb {

// Walk T over the Miller loop of Q and store its 68 lines.  Two independent point sets share one
// launch (the per-document H table and the per-share G2 points): the small set's latency-bound
// walk then overlaps the large one instead of adding a serial launch.
struct PrepSet {
  int n;
  const uint32_t* pts;
  int stride;
  uint4* coef;
  uint8_t* inf;
};
static __global__ void __launch_bounds__(256) k_g2_prepare(PrepSet s0, PrepSet s1) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool first = i < s0.n;
  if (!first) i -= s0.n;
  if (!first && i >= s1.n) return;
  const uint32_t* pts = first ? s0.pts : s1.pts;
  const int stride = first ? s0.stride : s1.stride;
  uint4* coef = first ? s0.coef : s1.coef;
  uint8_t* inf = first ? s0.inf : s1.inf;
  G2Aff q = g2_from_words(pts + (size_t)i * G2_WORDS);
  inf[i] = q.inf ? 1 : 0;
  if (q.inf) { q.x = f2_one(); q.y = f2_one(); }  // dummy walk; the pair is masked out
  G2Jac T{q.x, q.y, f2_one()};
  int step = 0;
  for (int b = 62; b >= 0; b--) {
    Line l = dbl_step(T);
    store_line(coef, stride, step++, i, l);
    if ((X_ABS >> b) & 1) {
      l = add_step(T, q.x, q.y);
      store_line(coef, stride, step++, i, l);
    }
  }
}

}  // namespace hb

namespace hbl {

static inline dim3 grid_for(int n) { return dim3((unsigned)((n + 255) / 256)); }

hipError_t g2_prepare(hipStream_t s, int n0, const void* pts0, void* coef0, uint8_t* inf0, int n1, const void* pts1,
                      void* coef1, uint8_t* inf1) {
  if (n0 + n1 <= 0) return hipSuccess;
  hb::PrepSet a{n0, (const uint32_t*)pts0, pad64(n0), (uint4*)coef0, inf0};
  hb::PrepSet b{n1, (const uint32_t*)pts1, pad64(n1), (uint4*)coef1, inf1};
  hipLaunchKernelGGL(hb::k_g2_prepare, grid_for(n0 + n1), dim3(256), 0, s, a, b);
  return hipGetLastError();
}

}  // namespace hbl
