"""Latency probe for the combine path on one GPU (tool, not product): host-to-host wall time of
interpolate_g2 for one combine of t+1 = 22 shares and of one master verify_g2 per pairing
implementation, plus the device stage times the engine records.  Prints one JSON line."""
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from hbbft_amd._lib import STAGE_CURVE, STAGE_PAIRING, STAGE_PREPARE  # noqa: E402
from hbbft_amd.engine import Engine  # noqa: E402


def med(f, reps=7):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(ts)


def main():
    eng = Engine(0)
    w = bench.Workload(eng, 64 * 4, seed=7)
    T = bench.T
    idx = [k for k in range(64) if w.expected[k]][: T + 1]
    pts = [w.sigs[k] for k in idx]
    out = {}
    out["interp_g2_1_ms"] = med(lambda: eng.interpolate_g2(T, [idx], [pts]))
    sig = eng.interpolate_g2(T, [idx], [pts])[0][0]
    eng.set_profiling(True)
    eng.interpolate_g2(T, [idx], [pts])
    out["interp_g2_1_dev_ms"] = eng.stage_time(STAGE_CURVE)[0]
    eng.set_profiling(False)
    out["interp_g1_1_ms"] = med(lambda: eng.interpolate_g1(T, [idx], [w.pks[k] for k in idx]))
    for name, impl in bench.IMPLS.items():
        eng.set_pairing_impl(impl)
        v = eng.verify_sig_shares([w.master_pk], [sig], [w.hashes[0]], [0])
        assert v == b"\x01", name
        out["verify1_%s_ms" % name] = med(lambda: eng.verify_sig_shares([w.master_pk], [sig], [w.hashes[0]], [0]))
        eng.set_profiling(True)
        eng.verify_sig_shares([w.master_pk], [sig], [w.hashes[0]], [0])
        out["verify1_%s_prep_dev_ms" % name] = eng.stage_time(STAGE_PREPARE)[0]
        out["verify1_%s_pair_dev_ms" % name] = eng.stage_time(STAGE_PAIRING)[0]
        eng.set_profiling(False)
    rng = random.Random(1)
    out["g2_mul_1_ms"] = med(lambda: eng.g2_mul([w.g2], [rng.randrange(1, bench.R_ORDER)]))
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
