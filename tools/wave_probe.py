"""GPU probe of the wave-per-check kernel: correctness against the lane-pair kernel on small batches
and device time per call for n = 1 .. 8192 checks (WAVE vs LANE_COOP vs PAIR)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import bls12_381 as C  # noqa: E402
from oracle import cbls  # noqa: E402
from hbbft_amd.engine import Engine, g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a  # noqa: E402
from hbbft_amd._lib import IMPL_LANE_COOP, IMPL_PAIR, IMPL_WAVE, IMPL_AUTO  # noqa: E402
import random  # noqa: E402

eng = Engine(0)
rng = random.Random(5)
g1, g2 = g1a(C.g1_uncompressed(C.G1_GEN)), g2a(C.g2_uncompressed(C.G2_GEN))
P = [C.g1_mul(C.G1_GEN, k) for k in (1, 5, 12345)]
Q = [C.g2_mul(C.G2_GEN, k) for k in (1, 7, 999)]
eng.set_pairing_impl(IMPL_WAVE)
out = eng.dbg_pairing([g1a(C.g1_uncompressed(p)) for p in P], [g2a(C.g2_uncompressed(q)) for q in Q])


def f12_bytes(e):
    return b"".join(c.to_bytes(48, "little") for six in e for f2 in six for c in f2)


for k in range(3):
    print("value", k, out[k] == f12_bytes(C.f12_pow(C.pairing(P[k], Q[k]), 3)), flush=True)
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
for impl in (IMPL_PAIR, IMPL_WAVE):
    eng.set_pairing_impl(impl)
    v = eng.verify_sig_shares([b[0] for b in base], [b[1] for b in base], hs, [b[2] for b in base])
    print("impl", impl, "verdicts", bytes(v).hex(), flush=True)
eng.set_profiling(True)
for n in [1, 2, 16, 256, 1024, 2048, 4096, 8192]:
    reps = (n + len(base) - 1) // len(base)
    bb = (base * reps)[:n]
    row = [n]
    for impl in (IMPL_WAVE, IMPL_LANE_COOP, IMPL_PAIR):
        eng.set_pairing_impl(impl)
        eng.verify_sig_shares([b[0] for b in bb], [b[1] for b in bb], hs, [b[2] for b in bb])
        eng.set_profiling(True)
        t0 = time.perf_counter()
        for _ in range(3):
            eng.verify_sig_shares([b[0] for b in bb], [b[1] for b in bb], hs, [b[2] for b in bb])
        wall = (time.perf_counter() - t0) / 3 * 1e3
        tot, cnt = eng.stage_time(1)
        tp, cp = eng.stage_time(0)
        row.append("impl%d dev %.3f ms (prep %.3f) wall %.3f" % (impl, tot / max(cnt, 1), tp / max(cp, 1), wall))
    print(*row, flush=True)
