"""Latency of combine_and_verify_sig for one document (N=64, t=21), host-to-host, with the split
master check (default) or interpolate-then-verify (HBH_SPLIT_CHECK=0 in the environment), plus the
device stage times; run under rocprofv3 --kernel-trace for per-kernel times."""
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hbbft_amd._lib import STAGE_CURVE, STAGE_PAIRING  # noqa
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
reps = int(os.environ.get("PROBE_REPS", "15"))
for _ in range(3):
    eng.combine_verify_g2(t, [idx], [sig], mpk, [h])
ts = []
eng.set_profiling(True)
for _ in range(reps):
    t0 = time.perf_counter()
    o, st, v = eng.combine_verify_g2(t, [idx], [sig], mpk, [h])
    ts.append((time.perf_counter() - t0) * 1e3)
    assert st == [0] and v == b"\x01"
out = {"split": os.environ.get("HBH_SPLIT_CHECK", "1") != "0", "host_ms_median": statistics.median(ts),
       "host_ms_min": min(ts), "curve_dev_ms": eng.stage_time(STAGE_CURVE)[0] / reps,
       "pair_dev_ms": eng.stage_time(STAGE_PAIRING)[0] / reps}
eng.set_profiling(False)
o2, st2, v2 = eng.combine_verify_g2(t, [idx], [sig], mpk, [eng.g2_mul([G2], [5])[0]])
out["wrong_doc_verdict"] = v2[0]
print(json.dumps(out))
