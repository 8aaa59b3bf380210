"""cProfile of the epoch workload's host side (GPU box): where the non-kernel time of run_epoch goes."""
import cProfile
import os
import pstats
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hbbft_amd.engine import Engine  # noqa: E402
from hbbft_amd.honey_badger import EpochTrace, NetworkKeys, run_epoch  # noqa: E402

eng = Engine(0)
rng = random.Random(3)
keys = NetworkKeys(eng, 100, 33, rng)
traces = [EpochTrace.generate(eng, keys, rng, hb_epoch=e, proposal_bytes=1000) for e in range(3)]
run_epoch(eng, keys, traces[0], window=4096)
t0 = time.perf_counter()
run_epoch(eng, keys, traces[1], window=4096)
print("epoch wall ms", (time.perf_counter() - t0) * 1e3)
pr = cProfile.Profile()
pr.enable()
run_epoch(eng, keys, traces[2], window=4096)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
