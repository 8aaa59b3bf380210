// Latency form of the G2 combine (threshold_crypto interpolate at 0 for a few combines):
//   interp_digits (k_curve.hip): the four 64-bit GLS digits of each lambda_k(0);
//   interp_g2_pair (k_interp_pair.hip): the curve work on lane pairs (pfp.hpp Fp2 arithmetic).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace hbl {
// digits[(c*m + k)*4 + j]; status[c] = HBL_DUPLICATE (and zero digits) on a repeated x
// g1: the two 128-bit GLV digits of G1 (phi = [-x^2]) as 4 u64 words per sample (d0 lo, d0 hi, d1 lo, d1 hi)
hipError_t interp_digits(hipStream_t s, int ncomb, int m, const uint32_t* xs, uint64_t* digits, int* status,
                         bool g1 = false);
// out[c] = sum_k lambda_k(0) P[c][k] on G1 (ABI G1 words) from the G1 digits; four workgroups (32-bit
// chunks) per combine on lane quads (k_g1quad.hip) and a join; part: interp_g1_quad_part_bytes(ncomb)
size_t interp_g1_quad_part_bytes(int ncomb);
hipError_t interp_g1_quad(hipStream_t s, int ncomb, int m, const uint64_t* digits, const void* pts, void* part,
                          void* out);
// out[c] = sum_k lambda_k(0) P[c][k] (ABI G2 words) from the digits; one workgroup per (combine,
// 32-bit digit chunk) and a join kernel; part: interp_g2_pair_part_bytes(ncomb) of device scratch
size_t interp_g2_pair_part_bytes(int ncomb);
hipError_t interp_g2_pair(hipStream_t s, int ncomb, int m, const uint64_t* digits, const void* pts, void* part,
                          void* out);
// true when interp_g2_pair handles m samples per combine
bool interp_g2_pair_fits(int m);
}  // namespace hbl
