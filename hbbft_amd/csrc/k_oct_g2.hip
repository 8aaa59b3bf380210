// HBH_IMPL_OCT, generator mode 2 (P2 is the generator; k_oct.hpp).
#define HS_MULFN static __device__ __noinline__
#include "k_oct.hpp"

namespace hbl {

hipError_t oct_verify_g2(hipStream_t s, int n, const PairSideDesc& d1, const PairSideDesc& d2, int flags,
                          uint8_t* verdict, uint32_t* value_out) {
  return oct_launch<2>(s, n, d1, d2, flags, verdict, value_out);
}

}  // namespace hbl
