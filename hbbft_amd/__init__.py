"""hbbft_amd -- MI355X (gfx950) batch engine for hbbft's BLS12-381 threshold-crypto hot path.

The product is the C ABI in include/hbbft_hip.h (libhbbft_hip.so, hand-written HIP kernels);
this package is its host-side binding.  There is no CPU fallback: without the built library or
a GPU the calls raise.
"""
from ._lib import G1_BYTES, G2_BYTES, FR_BYTES, HbhError, lib  # noqa: F401
