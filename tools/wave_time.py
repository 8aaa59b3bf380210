"""Device time of single-check wave-kernel calls (HBBFT_HIP_LIB selects the build); no verdict check."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12_381 as C  # noqa: E402
from oracle import cbls  # noqa: E402
from hbbft_amd.engine import Engine, g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a  # noqa: E402
from hbbft_amd._lib import IMPL_WAVE  # noqa: E402

eng = Engine(0)
g1, g2 = g1a(C.g1_uncompressed(C.G1_GEN)), g2a(C.g2_uncompressed(C.G2_GEN))
h = cbls.g2_mul(g2, 12345)
pk, sig = cbls.g1_mul(g1, 77), cbls.g2_mul(h, 77)
eng.set_pairing_impl(IMPL_WAVE)
eng.verify_sig_shares([pk], [sig], [h], [0])
eng.set_profiling(True)
for _ in range(5):
    v = eng.verify_sig_shares([pk], [sig], [h], [0])
tot, cnt = eng.stage_time(1)
print(os.path.basename(os.environ.get("HBBFT_HIP_LIB", "default")), "one check %.3f ms" % (tot / cnt), "verdict", v.hex())
