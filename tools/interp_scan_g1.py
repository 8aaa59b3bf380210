"""Device time of hbh_interpolate_g1 for ncomb = 1 .. 1024 combines of t = 21 (HBBFT_HIP_LIB selects the
build), and byte equality of the two forms on the 100-combine batch."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hbbft_amd._lib import STAGE_CURVE  # noqa: E402
from hbbft_amd.engine import Engine, g1_abi_from_uncompressed as g1a  # noqa: E402
from oracle import bls12_381 as C  # noqa: E402

eng = Engine(0)
rng = random.Random(1)
t = 21
G1 = g1a(C.g1_uncompressed(C.G1_GEN))
base = eng.g1_mul([G1] * 64, [rng.randrange(1, C.R) for _ in range(64)])
row = [os.path.basename(os.environ.get("HBBFT_HIP_LIB", "default"))]
for nc in (1, 16, 100, 256, 1024):
    idx = [[(c + k) % 64 for k in range(t + 1)] for c in range(nc)]
    pts = [[base[i] for i in ix] for ix in idx]
    out = eng.interpolate_g1(t, idx, pts)
    eng.set_profiling(True)
    for _ in range(3):
        out = eng.interpolate_g1(t, idx, pts)
    tot, cnt = eng.stage_time(STAGE_CURVE)
    eng.set_profiling(False)
    row.append("%d: %.2f ms" % (nc, tot / cnt))
print(*row, flush=True)
