// Latency form of the G2 combine (threshold_crypto interpolate at 0 for a few combines):
//   interp_digits (k_curve.hip): the four 64-bit GLS digits of each lambda_k(0);
//   interp_g2_pair (k_interp_pair.hip): the curve work on lane pairs (pfp.hpp Fp2 arithmetic).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace hbl {
// digits[(c*m + k)*4 + j]; status[c] = HBL_DUPLICATE (and zero digits) on a repeated x
hipError_t interp_digits(hipStream_t s, int ncomb, int m, const uint32_t* xs, uint64_t* digits, int* status);
// out[c] = sum_k lambda_k(0) P[c][k] (ABI G2 words) from the digits; one workgroup per (combine,
// 32-bit digit chunk) and a join kernel; part: interp_g2_pair_part_bytes(ncomb) of device scratch
size_t interp_g2_pair_part_bytes(int ncomb);
hipError_t interp_g2_pair(hipStream_t s, int ncomb, int m, const uint64_t* digits, const void* pts, void* part,
                          void* out);
// true when interp_g2_pair handles m samples per combine
bool interp_g2_pair_fits(int m);
}  // namespace hbl
