"""Host-to-host time of the epoch's engine calls (combine_verify_g2 of 10 / 100 coin-sized combines,
t = 33; verify_sig_shares of 100 / 1,000 / 5,000 checks), for A/B between trees: run it from a tree's
root (the hbbft_amd package of the current directory is imported)."""
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.getcwd())
from hbbft_amd.engine import Engine  # noqa: E402
from hbbft_amd.honey_badger import NetworkKeys  # noqa: E402
from hbbft_amd.sync_key_gen import G2_GEN, R_ORDER  # noqa: E402

eng = Engine(0)
rng = random.Random(7)
n, t = 100, 33
keys = NetworkKeys(eng, n, t, rng)
hs = eng.g2_mul([G2_GEN] * 100, [rng.randrange(1, R_ORDER) for _ in range(100)])
row = [os.path.basename(os.getcwd())]
# shares of document c by every node
for ncomb in (10, 100):
    idx, pts = [], []
    for c in range(ncomb):
        ids = sorted(rng.sample(range(n), t + 1))
        sh = eng.g2_mul([hs[c]] * (t + 1), [keys.sks[i] for i in ids])
        idx.append(ids)
        pts.append(sh)
    eng.combine_verify_g2(t, idx, pts, keys.master_pk, hs[:ncomb])
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        out, st, v = eng.combine_verify_g2(t, idx, pts, keys.master_pk, hs[:ncomb])
        ts.append((time.perf_counter() - t0) * 1e3)
        assert all(s == 0 for s in st) and all(v)
    row.append("combine%d %.2f ms" % (ncomb, statistics.median(ts)))
for nchk in (100, 1000, 5000):
    docs = [k % 100 for k in range(nchk)]
    nodes = [k % n for k in range(nchk)]
    sh = eng.g2_mul([hs[d] for d in docs], [keys.sks[j] for j in nodes])
    pk = [keys.pks[j] for j in nodes]
    eng.verify_sig_shares(pk, sh, hs, docs)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        v = eng.verify_sig_shares(pk, sh, hs, docs)
        ts.append((time.perf_counter() - t0) * 1e3)
        assert all(v)
    row.append("verify%d %.2f ms" % (nchk, statistics.median(ts)))
print(*row, flush=True)
