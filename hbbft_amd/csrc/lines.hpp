// Miller-loop line tables of G2 points (gfx950): the table layout written by k_g2_prepare
// (k_prepare.hip) and read by the lane-cooperative and one-thread signed pairing kernels.
#pragma once
#include "pairing.hpp"
#include "points.hpp"

namespace hb {

constexpr int LINE_Q4 = LINE_WORDS / 4;  // 21 x 16-byte chunks per line

// Line tables: uint4 coef[(step * LINE_Q4 + q) * stride + point]  -- lanes that walk consecutive
// points read consecutive 16-byte chunks (coalesced); lanes sharing a point (H per document) read
// one broadcast address.
__device__ __forceinline__ void store_line(uint4* __restrict__ coef, int stride, int step, int pt, const Line& l) {
  uint32_t w[LINE_WORDS];
#pragma unroll
  for (int j = 0; j < NL; j++) {
    w[0 * NL + j] = l.c0.c0.l[j];
    w[1 * NL + j] = l.c0.c1.l[j];
    w[2 * NL + j] = l.c1.c0.l[j];
    w[3 * NL + j] = l.c1.c1.l[j];
    w[4 * NL + j] = l.c4.c0.l[j];
    w[5 * NL + j] = l.c4.c1.l[j];
  }
#pragma unroll
  for (int q = 0; q < LINE_Q4; q++)
    coef[((size_t)step * LINE_Q4 + q) * stride + pt] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

__device__ __forceinline__ Line load_line(const uint4* __restrict__ coef, int stride, int step, int pt) {
  uint32_t w[LINE_WORDS];
#pragma unroll
  for (int q = 0; q < LINE_Q4; q++) {
    uint4 v = coef[((size_t)step * LINE_Q4 + q) * stride + pt];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
  Line l;
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

}  // namespace hb
