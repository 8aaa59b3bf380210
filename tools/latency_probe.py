"""Device ms per share-check call by size and implementation (HBBFT_HIP_LIB selects the build), verdicts
compared with the lane-pair kernel at every size.  usage: latency_probe.py [N ...] (default 1 1024 4096 8192)"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12_381 as C  # noqa: E402
from oracle import cbls  # noqa: E402
from hbbft_amd.engine import Engine, g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a  # noqa: E402
from hbbft_amd._lib import IMPL_PAIR, IMPL_WAVE, IMPL_OCT, IMPL_AUTO, IMPL_WAVE2  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [1, 1024, 4096, 8192]
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
for n in sizes:
    bb = (base * ((n + 63) // 64))[:n]
    a = ([b[0] for b in bb], [b[1] for b in bb], hs, [b[2] for b in bb])
    eng.set_pairing_impl(IMPL_PAIR)
    ref = eng.verify_sig_shares(*a)
    row = ["n=%d" % n]
    for name, impl in (("wave2", IMPL_WAVE2), ("wave", IMPL_WAVE), ("oct", IMPL_OCT), ("auto", IMPL_AUTO)):
        if impl in (IMPL_WAVE, IMPL_WAVE2) and n > 4096:
            continue
        eng.set_pairing_impl(impl)
        if not os.environ.get("HBH_PROBE_NOCHECK"):  # timing-only A/B libraries give wrong verdicts
            assert eng.verify_sig_shares(*a) == ref, (name, n)
        eng.set_profiling(True)
        for _ in range(3):
            eng.verify_sig_shares(*a)
        tot, cnt = eng.stage_time(1)
        eng.set_profiling(False)
        row.append("%s %.3f ms" % (name, tot / cnt))
    print(*row, flush=True)
