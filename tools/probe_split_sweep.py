"""combine_and_verify_sig host-to-host latency per call by batch size (ncomb combines of t + 1 shares),
split master check vs interpolate-then-verify; the engine reads HBH_SPLIT_MAX / HBH_SPLIT_CHECK at
creation, so each mode gets its own engine.  usage: probe_split_sweep.py T NCOMB [NCOMB ...]"""
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hbbft_amd.engine import Engine, g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a  # noqa
from oracle import bls12_381 as C  # noqa

t = int(sys.argv[1])
sizes = [int(x) for x in sys.argv[2:]]
R = C.R
rng = random.Random(5)
G1 = g1a(C.g1_uncompressed(C.G1_GEN))
G2 = g2a(C.g2_uncompressed(C.G2_GEN))
coeffs = [rng.randrange(1, R) for _ in range(t + 1)]


def pe(x):
    r = 0
    for c in reversed(coeffs):
        r = (r * x + c) % R
    return r


n = 3 * t + 1
modes = {"split": ("1", "100000"), "unsplit": ("0", "0"), "auto": ("1", "0")}
engines = {}
for name, (chk, mx) in modes.items():
    os.environ["HBH_SPLIT_CHECK"], os.environ["HBH_SPLIT_MAX"] = chk, mx
    engines[name] = Engine(0)
eng = engines["split"]
mpk = eng.g1_mul([G1], [coeffs[0]])[0]
nd = max(sizes)
hs = eng.g2_mul([G2] * nd, [rng.randrange(1, R) for _ in range(nd)])
idxs, sigs = [], []
for c in range(nd):
    idx = sorted(rng.sample(range(n), t + 1))
    idxs.append(idx)
    sigs.append(eng.g2_mul([hs[c]] * (t + 1), [pe(i + 1) for i in idx]))
for nc in sizes:
    res = {"t": t, "ncomb": nc}
    outs = {}
    for name, e in engines.items():
        args = (t, idxs[:nc], sigs[:nc], mpk, hs[:nc])
        for _ in range(2):
            e.combine_verify_g2(*args)
        ts = []
        for _ in range(7):
            t0 = time.perf_counter()
            outs[name] = e.combine_verify_g2(*args)
            ts.append((time.perf_counter() - t0) * 1e3)
        res[name + "_ms"] = round(statistics.median(ts), 3)
        assert list(outs[name][1]) == [0] * nc and bytes(outs[name][2]) == b"\x01" * nc, name
    assert outs["split"] == outs["unsplit"] == outs["auto"]
    print(json.dumps(res), flush=True)
