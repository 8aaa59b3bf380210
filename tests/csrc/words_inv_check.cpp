// CPU check of hbbft_amd/csrc/words.hpp's variable-time inverse: every MODE (runs of even divsteps
// at once, lazily reduced coefficients -- the wave kernels' one inversion) against the per-divstep
// form, and both against y * y^-1 == 1, for the BLS12-381 base field (12 words) and scalar
// field (8 words).  Built and run by tests/test_words_inv.py.
#include <cstdint>
#include <cstdio>
#include <random>

#include "words.hpp"

template <int N>
static bool mul_is_one(const uint32_t* a, const uint32_t* b, const uint32_t* m) {
  // a * b mod m by schoolbook + shift-subtract (slow, test only)
  uint32_t acc[N + 1] = {0};
  for (int bit = 32 * N - 1; bit >= 0; bit--) {
    uint32_t carry = 0;  // acc <<= 1
    for (int i = 0; i <= N; i++) {
      const uint32_t nc = acc[i] >> 31;
      acc[i] = (acc[i] << 1) | carry;
      carry = nc;
    }
    if ((a[bit >> 5] >> (bit & 31)) & 1) {
      uint64_t c = 0;
      for (int i = 0; i < N; i++) {
        c += (uint64_t)acc[i] + b[i];
        acc[i] = (uint32_t)c;
        c >>= 32;
      }
      acc[N] += (uint32_t)c;
    }
    for (int k = 0; k < 3; k++) {
      if (acc[N] == 0 && !hb::words_geq<N>(acc, m)) break;
      const uint32_t br = hb::words_sub<N>(acc, m);
      acc[N] -= br;
    }
  }
  return acc[N] == 0 && hb::words_is_one<N>(acc);
}

template <int N>
static int run(const uint32_t* m, uint32_t topmask, int iters, uint64_t seed) {
  std::mt19937_64 rng(seed);
  int bad = 0;
  for (int it = 0; it < iters; it++) {
    uint32_t y[N];
    for (int i = 0; i < N; i++) y[i] = (uint32_t)rng();
    y[N - 1] &= topmask;
    if (it < 3) {
      for (int i = 0; i < N; i++) y[i] = 0;
      y[0] = (uint32_t)it;  // 0 (no inverse: 0 out), 1, 2
    } else if (it == 3) {
      for (int i = 0; i < N; i++) y[i] = m[i];
      y[0] -= 1;  // m - 1
    }
    uint32_t r0[N], r1[N], r2[N], r3[N];
    hb::words_inv_vartime<N, 0>(y, m, r0);
    hb::words_inv_vartime<N, hb::INV_BATCH>(y, m, r1);
    hb::words_inv_vartime<N, hb::INV_LAZY>(y, m, r2);
    hb::words_inv_vartime<N, hb::INV_BATCH | hb::INV_LAZY>(y, m, r3);
    bool same = true, zero = true;
    for (int i = 0; i < N; i++) {
      same = same && r0[i] == r1[i] && r0[i] == r2[i] && r0[i] == r3[i];
      zero = zero && y[i] == 0;
    }
    const bool ok = same && (zero || (it < 200 ? mul_is_one<N>(y, r1, m) : true));
    if (!ok) bad++;
  }
  return bad;
}

int main() {
  const uint32_t P[12] = {0xffffaaab, 0xb9feffff, 0xb153ffff, 0x1eabfffe, 0xf6b0f624, 0x6730d2a0,
                          0xf38512bf, 0x64774b84, 0x434bacd7, 0x4b1ba7b6, 0x397fe69a, 0x1a0111ea};
  const uint32_t R[8] = {0x00000001, 0xffffffff, 0xfffe5bfe, 0x53bda402,
                         0x09a1d805, 0x3339d808, 0x299d7d48, 0x73eda753};
  const int bp = run<12>(P, 0x0fffffff, 20000, 1);
  const int br = run<8>(R, 0x3fffffff, 20000, 2);
  printf("p: %d bad, r: %d bad\n", bp, br);
  return (bp || br) ? 1 : 0;
}
