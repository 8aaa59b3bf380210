"""Latency probe of combine_and_verify_sig for one document (N=64, t=21): host-to-host per impl,
and the device stage split (interpolation vs pairing) -- run under rocprofv3 --kernel-trace for
per-kernel times."""
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hbbft_amd._lib import IMPL_AUTO, IMPL_LANE_COOP, IMPL_PAIR, STAGE_CURVE, STAGE_PAIRING, STAGE_PREPARE  # noqa
from hbbft_amd.engine import Engine, g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a  # noqa
from oracle import bls12_381 as C  # noqa

R = C.R
eng = Engine(0)
rng = random.Random(1)
t, n = 21, 64
G1 = g1a(C.g1_uncompressed(C.G1_GEN))
G2 = g2a(C.g2_uncompressed(C.G2_GEN))
coeffs = [rng.randrange(1, R) for _ in range(t + 1)]


def pe(x):
    r = 0
    for c in reversed(coeffs):
        r = (r * x + c) % R
    return r


sks = [pe(i + 1) for i in range(n)]
mpk = eng.g1_mul([G1], [coeffs[0]])[0]
h = eng.g2_mul([G2], [rng.randrange(1, R)])[0]
idx = list(range(3, 3 + t + 1))
sig = eng.g2_mul([h] * (t + 1), [sks[i] for i in idx])
out = {}
for name, impl in (("auto", IMPL_AUTO), ("lane_coop", IMPL_LANE_COOP)):
    eng.set_pairing_impl(impl)
    for _ in range(2):
        eng.combine_verify_g2(t, [idx], [sig], mpk, [h])
    ts = []
    eng.set_profiling(True)
    for _ in range(7):
        t0 = time.perf_counter()
        o, st, v = eng.combine_verify_g2(t, [idx], [sig], mpk, [h])
        ts.append((time.perf_counter() - t0) * 1e3)
        assert st == [0] and v == b"\x01"
    out[name] = {"host_ms": statistics.median(ts),
                 "curve_dev_ms": eng.stage_time(STAGE_CURVE)[0] / 7,
                 "prep_dev_ms": eng.stage_time(STAGE_PREPARE)[0] / 7,
                 "pair_dev_ms": eng.stage_time(STAGE_PAIRING)[0] / 7}
    eng.set_profiling(False)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        eng.verify_sig_shares([mpk], [o[0]], [h], [0])
        ts.append((time.perf_counter() - t0) * 1e3)
    out[name]["verify1_host_ms"] = statistics.median(ts)
eng.set_pairing_impl(IMPL_AUTO)
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    eng.interpolate_g2(t, [idx], [sig])
    ts.append((time.perf_counter() - t0) * 1e3)
out["interp_g2_host_ms"] = statistics.median(ts)
print(json.dumps(out, indent=1))
