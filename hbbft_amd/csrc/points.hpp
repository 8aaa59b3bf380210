// Boundary formats <-> device representation.
//
// ABI point format (include/hbbft_hip.h): affine coordinates as canonical little-endian integers,
//   G1: x(48 B) || y(48 B)                      = 24 x uint32
//   G2: x.c0 || x.c1 || y.c0 || y.c1 (48 B each) = 48 x uint32
// The point at infinity is all-zero ((0,0) is on neither curve, so the encoding is unambiguous).
#pragma once
#include "tower.hpp"

namespace hb {

constexpr int G1_WORDS = 24;
constexpr int G2_WORDS = 48;

struct G1Aff { Fp x, y; bool inf; };
struct G2Aff { Fp2 x, y; bool inf; };

HB_HD bool words_all_zero(const uint32_t* w, int n) {
  uint32_t o = 0;
  for (int i = 0; i < n; i++) o |= w[i];
  return o == 0;
}

HB_HD G1Aff g1_from_words(const uint32_t* w) {
  G1Aff p;
  p.x = fp_from_words(w);
  p.y = fp_from_words(w + 12);
  p.inf = words_all_zero(w, G1_WORDS);
  return p;
}

HB_HD G2Aff g2_from_words(const uint32_t* w) {
  G2Aff p;
  p.x.c0 = fp_from_words(w);
  p.x.c1 = fp_from_words(w + 12);
  p.y.c0 = fp_from_words(w + 24);
  p.y.c1 = fp_from_words(w + 36);
  p.inf = words_all_zero(w, G2_WORDS);
  return p;
}

}  // namespace hb
