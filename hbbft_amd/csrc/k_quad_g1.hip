// HBH_IMPL_QUAD, generator mode 1 (P1 is the generator; k_quad.hpp).
#define HS_MULFN static __device__ __noinline__
#include "k_quad.hpp"

namespace hbl {

hipError_t quad_verify_g1(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
                          uint8_t* verdict, uint32_t* value_out) {
  return quad_launch<1>(s, n, d1, d2, flags, verdict, value_out);
}

}  // namespace hbl
