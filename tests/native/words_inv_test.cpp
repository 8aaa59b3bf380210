#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include "words.hpp"
// p and r as words
static const uint32_t PW[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
static const uint32_t RW[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u, 0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
// check y * out == 1 mod m via schoolbook multiply + long reduction (slow, fine)
template <int N> bool check(const uint32_t* y, const uint32_t* m, const uint32_t* o) {
  // compute (y*o) mod m using bitwise double-and-add on N words
  uint32_t acc[N + 1] = {0};
  for (int bit = 32 * N - 1; bit >= 0; bit--) {
    // acc = 2 acc mod m
    uint32_t c = 0;
    for (int i = 0; i <= N; i++) { uint32_t nc = acc[i] >> 31; acc[i] = (acc[i] << 1) | c; c = nc; }
    if (acc[N] || hb::words_geq<N>(acc, m)) { uint32_t br = hb::words_sub<N>(acc, m); acc[N] -= br; }
    if ((o[bit >> 5] >> (bit & 31)) & 1) {
      uint64_t cc = 0;
      for (int i = 0; i < N; i++) { cc += (uint64_t)acc[i] + y[i]; acc[i] = (uint32_t)cc; cc >>= 32; }
      acc[N] += (uint32_t)cc;
      if (acc[N] || hb::words_geq<N>(acc, m)) { uint32_t br = hb::words_sub<N>(acc, m); acc[N] -= br; }
    }
  }
  return acc[N] == 0 && hb::words_is_one<N>(acc);
}
template <int N> int run(const uint32_t* m, int trials, std::mt19937_64& g) {
  int bad = 0;
  for (int t = 0; t < trials; t++) {
    uint32_t y[N], o[N];
    for (int i = 0; i < N; i++) y[i] = (uint32_t)g();
    if (t == 0) { memset(y, 0, sizeof y); y[0] = 1; }
    if (t == 1) { memcpy(y, m, sizeof y); y[0] -= 1; }
    if (t == 2) { memset(y, 0, sizeof y); y[0] = 2; }
    if (t == 3) { memset(y, 0, sizeof y); y[N - 1] = 1u << 20; }
    if (t == 4) { memset(y, 0, sizeof y); y[3] = 0xffffffffu; }
    // reduce y mod m roughly: clear the top bits
    y[N - 1] &= (m[N - 1] >> 1);
    if (hb::words_geq<N>(y, m)) hb::words_sub<N>(y, m);
    bool zero = true; for (int i = 0; i < N; i++) zero &= y[i] == 0;
    if (zero) y[0] = 3;
    hb::words_inv_vartime<N>(y, m, o);
    if (!check<N>(y, m, o)) { bad++; if (bad < 5) printf("bad trial %d\n", t); }
  }
  uint32_t z[N] = {0}, o[N];
  hb::words_inv_vartime<N>(z, m, o);
  for (int i = 0; i < N; i++) if (o[i]) { printf("inv(0) != 0\n"); bad++; break; }
  return bad;
}
int main() {
  std::mt19937_64 g(42);
  int b1 = run<12>(PW, 20000, g), b2 = run<8>(RW, 20000, g);
  printf("bad: p %d, r %d\n", b1, b2);
  return b1 || b2;
}
