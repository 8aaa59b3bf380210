// Host launcher of k_lc_prep_pair (k_lcprep.hip): lane-pair walk of up to two G2 point sets into
// the line-table layout of lines.hpp (LINE_Q4 int4 per step, pad64(n) points per row).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace hbl {
hipError_t lc_prep_pair(hipStream_t s, int n0, const void* pts0, void* coef0, uint8_t* inf0, int n1, const void* pts1,
                        void* coef1, uint8_t* inf1);
}  // namespace hbl
