"""Per-stage-kind core-cycle profile of k_wave / k_wave64 (round 6): run with a library built with
-DWV_STAGE_CLOCK (timing only; block 0's lane 0 prints one STAGECLK line per stage program it runs).
  HBBFT_HIP_LIB=ab_libs/clk.so python tools/stage_clock.py"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12_381 as C  # noqa: E402
from oracle import cbls  # noqa: E402
from hbbft_amd.engine import Engine, g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a  # noqa: E402
from hbbft_amd._lib import IMPL_WAVE, IMPL_WAVE2  # noqa: E402

eng = Engine(0)
rng = random.Random(5)
g1, g2 = g1a(C.g1_uncompressed(C.G1_GEN)), g2a(C.g2_uncompressed(C.G2_GEN))
h = cbls.g2_mul(g2, rng.randrange(1, C.R))
sk = rng.randrange(1, C.R)
pk, sig = cbls.g1_mul(g1, sk), cbls.g2_mul(h, sk)
for name, impl in (("wave", IMPL_WAVE), ("wave2", IMPL_WAVE2)):
    eng.set_pairing_impl(impl)
    for _ in range(2):
        print("== %s single check" % name, flush=True)
        assert eng.verify_sig_shares([pk], [sig], [h], [0]) == b"\x01"
        eng.synchronize() if hasattr(eng, "synchronize") else None
# one combine (t = 21): the split master check's W1J Miller waves, the tree and the final exponentiation
t = 21
coeffs = [rng.randrange(1, C.R) for _ in range(t + 1)]
ids = list(range(t + 1))
shares = [cbls.g2_mul(h, sum(c * pow(i + 1, k, C.R) for k, c in enumerate(coeffs)) % C.R) for i in ids]
mpk = cbls.g1_mul(g1, coeffs[0])
for _ in range(2):
    print("== combine t=21", flush=True)
    out, st, v = eng.combine_verify_g2(t, [ids], [shares], mpk, [h])
    assert st == [0] and v == b"\x01"
