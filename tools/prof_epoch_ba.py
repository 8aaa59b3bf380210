"""Host profile of one N=100 epoch on the GPU box, BA-driven coins vs the synthetic coin set
(cProfile; the engine calls are real)."""
import cProfile
import pstats
import random
import sys
import time

sys.path.insert(0, ".")
from hbbft_amd.engine import Engine  # noqa: E402
from hbbft_amd.honey_badger import EpochTrace, NetworkKeys, run_epoch  # noqa: E402

eng = Engine(0)
rng = random.Random(5)
keys = NetworkKeys(eng, 100, 33, rng)
for mode in ("synthetic", "ba", "synthetic", "ba"):
    tr = EpochTrace.generate(eng, keys, rng, hb_epoch=0, proposal_bytes=1000)
    if mode == "ba":
        tr.with_ba(eng, rng)
    run_epoch(eng, keys, tr, window=4096)  # warm
    tr = EpochTrace.generate(eng, keys, rng, hb_epoch=1, proposal_bytes=1000)
    if mode == "ba":
        tr.with_ba(eng, rng)
    pr = cProfile.Profile()
    t = time.time()
    pr.enable()
    res = run_epoch(eng, keys, tr, window=4096)
    pr.disable()
    print(mode, "epoch %.1f ms" % ((time.time() - t) * 1e3), {k: round(v * 1e3, 1) for k, v in res.timing.items()},
          "calls", res.engine_calls, flush=True)
    if mode == "ba":
        pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
