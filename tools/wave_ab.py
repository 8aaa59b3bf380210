"""A/B timing of the wave-per-check kernel (HBBFT_HIP_LIB selects the build): device ms per call
at n = 1 .. 2048 checks, plus a verdict check against the lane-pair kernel."""
import os
import sys
import random

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12_381 as C  # noqa: E402
from oracle import cbls  # noqa: E402
from hbbft_amd.engine import Engine, g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a  # noqa: E402
from hbbft_amd._lib import IMPL_PAIR, IMPL_WAVE  # noqa: E402

eng = Engine(0)
rng = random.Random(5)
g1, g2 = g1a(C.g1_uncompressed(C.G1_GEN)), g2a(C.g2_uncompressed(C.G2_GEN))
hs = [cbls.g2_mul(g2, rng.randrange(1, C.R)) for _ in range(3)]
sk = [rng.randrange(1, C.R) for _ in range(7)]
pks = [cbls.g1_mul(g1, k) for k in sk]
base = []
for i in range(64):
    d, j = i % 3, i % 7
    pk, sig = pks[j], cbls.g2_mul(hs[d], sk[j])
    if i % 11 == 3:
        sig = cbls.g2_mul(hs[(d + 1) % 3], sk[j])
    elif i % 11 == 7:
        pk, sig = bytes(96), bytes(192)
    base.append((pk, sig, d))
args = ([b[0] for b in base], [b[1] for b in base], hs, [b[2] for b in base])
eng.set_pairing_impl(IMPL_PAIR)
ref = eng.verify_sig_shares(*args)
eng.set_pairing_impl(IMPL_WAVE)
assert eng.verify_sig_shares(*args) == ref
tag = os.path.basename(os.environ.get("HBBFT_HIP_LIB", "default"))
row = [tag]
for n in [1, 256, 1024, 2048]:
    bb = (base * ((n + 63) // 64))[:n]
    a = ([b[0] for b in bb], [b[1] for b in bb], hs, [b[2] for b in bb])
    eng.verify_sig_shares(*a)
    eng.set_profiling(True)
    for _ in range(3):
        eng.verify_sig_shares(*a)
    tot, cnt = eng.stage_time(1)
    row.append("n=%d %.3f ms" % (n, tot / cnt))
print(*row, flush=True)
