// Host launcher of the wire-format kernels (k_wire.hip).  Kept out of launch.hpp so that the
// pairing translation units do not depend on it.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace hbl {

// per-point flags prepared by the host from the compressed encoding's top bits
constexpr uint8_t WIRE_INFINITY = 1;  // valid encoding of the point at infinity
constexpr uint8_t WIRE_GREATEST = 2;  // the "y is the larger root" bit
constexpr uint8_t WIRE_REJECT = 4;    // malformed flags (not compressed, bad infinity encoding)

// G1Compressed::into_affine for n points: xw = 12 canonical LE words of x per point (flag bits
// cleared); out = ABI G1 points (all-zero when ok[i] == 0 or for infinity); ok[i] = 1 iff the
// encoding decodes to a point of the prime-order subgroup.
hipError_t g1_decompress(hipStream_t s, int n, const uint32_t* xw, const uint8_t* flags, void* out, uint8_t* ok);
// G2Compressed::into_affine: xw = 24 words per point (x.c0 then x.c1), out = ABI G2 points.
hipError_t g2_decompress(hipStream_t s, int n, const uint32_t* xw, const uint8_t* flags, void* out, uint8_t* ok);

// Device-side flag parsing + word reversal of n encodings (nfe = 1 for G1, 2 for G2) already in
// device memory: xw = 12 * nfe words per point, flags as above.
hipError_t wire_parse(hipStream_t s, int n, int nfe, const uint8_t* in, uint32_t* xw, uint8_t* flags);

}  // namespace hbl
