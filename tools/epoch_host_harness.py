"""CPU harness for the HoneyBadger epoch's HOST side (configs[4]): the same run_epoch flows, with an
engine stand-in whose curve arithmetic runs on the host stage (hbh_host_g1_mul / g2_mul) and whose
verdicts come from the trace's construction (which shares were forged), so the Python flows can be
profiled and tuned without a GPU.  Test and tuning infrastructure only: never used by the product
path (bench.py's epoch line runs the real engine).

usage: python3 tools/epoch_host_harness.py [--profile] [--reps N]"""
import argparse
import cProfile
import os
import pickle
import pstats
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hbbft_amd import hoststage  # noqa: E402
from hbbft_amd.honey_badger import EpochTrace, NetworkKeys, prefetch_coins, run_epoch  # noqa: E402


class HostEngine:
    """Engine stand-in: scalar multiplications on the host stage; pairing verdicts from a table of
    the valid (public key, share) pairs the trace was built from; combines from the master key."""

    def __init__(self, threads=8):
        self.threads = threads
        self.valid = set()      # (pk bytes, share bytes) known valid
        self.msk = None
        self.u_of_share = {}    # decryption share -> U of its ciphertext

    # curve arithmetic used to build traces
    def g1_mul(self, pts, scalars):
        return hoststage.g1_mul(list(pts), list(scalars), threads=self.threads)

    def g2_mul(self, pts, scalars):
        return hoststage.g2_mul(list(pts), list(scalars), threads=self.threads)

    # verdicts
    sleep_base, sleep_per = 0.0, 0.0  # emulated device time per call (time.sleep releases the GIL)

    def _device(self, n):
        if self.sleep_base or self.sleep_per:
            time.sleep(self.sleep_base + n * self.sleep_per)

    def verify_sig_shares(self, pks, sigs, hashes, doc_idx):
        self._device(len(pks))
        return bytes(1 if (bytes(p), bytes(s)) in self.valid else 0 for p, s in zip(pks, sigs))

    def verify_dec_shares(self, shares, pks, huv, w, ct_idx):
        self._device(len(pks))
        return bytes(1 if (bytes(p), bytes(s)) in self.valid else 0 for s, p in zip(shares, pks))

    def verify_ciphertexts(self, us, ws, huv):
        return bytes(1 for _ in us)

    def combine_verify_g2(self, t, idx, shares, master_pk, hashes):
        sigs = hoststage.g2_mul([bytes(h) for h in hashes], [self.msk] * len(hashes), threads=self.threads)
        st = [5 if len(set(i)) != len(i) else 0 for i in idx]
        return sigs, st, bytes(1 for _ in idx)

    def interpolate_g1(self, t, idx, shares):
        us = [self.u_of_share[bytes(s[0])] for s in shares]
        return hoststage.g1_mul(us, [self.msk] * len(us), threads=self.threads), [0] * len(idx)


def build(eng, seed=5, n=100, t=33):
    rng = random.Random(seed)
    keys = NetworkKeys(eng, n, t, rng)
    tr = EpochTrace.generate(eng, keys, rng, hb_epoch=1, proposal_bytes=1000)
    tr.with_ba(eng, rng)
    return keys, tr


def teach(eng, keys, tr):
    """Fill the stand-in's verdict table from the trace's construction."""
    eng.msk = keys.msk
    bad = set(tr.bad) | set(tr.ba.bad)
    for (p, j), s in tr.dec_shares.items():
        eng.u_of_share[bytes(s)] = tr.cts[p][0]
        if ("dec", p, j) not in bad:
            eng.valid.add((bytes(keys.pks[j]), bytes(s)))
    from hbbft_amd.sync_key_gen import G1_GEN
    for p in tr.cts:  # a ciphertext check as a share-check row (honey_badger._one_call): (g1, U)
        eng.valid.add((bytes(G1_GEN), bytes(tr.cts[p][0])))
    for (p, e, j), s in tr.ba.shares.items():
        if ("coin", p, j) not in bad:
            eng.valid.add((bytes(keys.pks[j]), bytes(s)))
    # our own coin shares and decryption shares (signed / computed by the flows on the host)
    ps = sorted(tr.cts)
    for p, s in zip(ps, hoststage.g1_mul([tr.cts[p][0] for p in ps], [keys.sks[0]] * len(ps))):
        eng.u_of_share[bytes(s)] = tr.cts[p][0]
    hs = [tr.ba.hashes[k] for k in sorted(tr.ba.hashes)]
    for s in hoststage.g2_mul(hs, [keys.sks[0]] * len(hs)):
        eng.valid.add((bytes(keys.pks[0]), bytes(s)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--prefetch", action="store_true", help="coin documents prefetched (here: same epoch)")
    ap.add_argument("--pipeline", action="store_true")
    ap.add_argument("--no-preverify", action="store_true")
    ap.add_argument("--window", type=int, default=6144)
    ap.add_argument("--device-ms", default="0,0", help="emulated device time per drain: base ms, ms per check")
    ap.add_argument("--dump", default=None, metavar="FILE",
                    help="write a digest of the last epoch's outputs (decisions, coins, plaintexts, faults, errors) "
                         "to compare two versions of the flows")
    args = ap.parse_args()
    eng = HostEngine()
    b, per = (float(x) for x in args.device_ms.split(","))
    eng.sleep_base, eng.sleep_per = b / 1e3, per / 1e3
    cache = os.path.join("/tmp", "epoch_host_trace.pkl")
    if os.path.exists(cache):
        with open(cache, "rb") as f:
            keys_state, tr = pickle.load(f)
        keys = NetworkKeys.__new__(NetworkKeys)
        keys.__dict__.update(keys_state)
    else:
        t0 = time.time()
        keys, tr = build(eng)
        print("trace built in %.1f s" % (time.time() - t0), flush=True)
        with open(cache, "wb") as f:
            pickle.dump((keys.__dict__, tr), f)
    teach(eng, keys, tr)
    # the second engine of decryption-share pre-verification / pipelined combines: the same stand-in
    import hbbft_amd.honey_badger as hb
    eng.device = 0
    hb._COMBINE_ENGINES[id(eng)] = (eng, eng)
    for r in range(args.reps):
        pr = cProfile.Profile() if args.profile and r == args.reps - 1 else None
        t0 = time.perf_counter()
        if pr:
            pr.enable()
        pf = prefetch_coins(keys, tr.hb_epoch, range(keys.n)) if args.prefetch else None
        res = run_epoch(eng, keys, tr, window=args.window, coin_prefetch=pf, pipelined=args.pipeline,
                        preverify=not args.no_preverify)
        if pr:
            pr.disable()
        ms = (time.perf_counter() - t0) * 1e3
        print("epoch %.1f ms" % ms, {k: round(v * 1e3, 1) for k, v in res.timing.items()},
              "wait", {k: round(v * 1e3, 1) for k, v in res.wait.items()},
              "calls", res.engine_calls, "coins", len(res.coins), "plaintexts", len(res.plaintexts),
              "faults", len(res.faults), "errors", len(res.errors), flush=True)
        if pr:
            pstats.Stats(pr).sort_stats("tottime").print_stats(30)
    if args.dump:
        with open(args.dump, "w") as f:
            f.write(digest(res))


def digest(res):
    """Canonical text of an epoch's observable outputs."""
    import hashlib
    lines = ["decisions %r" % sorted(res.ba_decisions.items()),
             "ba_coins %r" % sorted((p, sorted(c.items())) for p, c in res.ba_coins.items()),
             "coins %r" % sorted(res.coins.items()),
             "signatures %s" % hashlib.sha256(b"".join(bytes(res.signatures[p]) for p in sorted(res.signatures))).hexdigest(),
             "plaintexts %s" % hashlib.sha256(b"".join(bytes(res.plaintexts[p]) for p in sorted(res.plaintexts))).hexdigest(),
             "faults %r" % sorted(repr(f) for f in res.faults),
             "errors %r" % sorted(repr(e) for e in res.errors),
             "ba_queued %r" % res.ba_queued]
    return "\n".join(lines) + "\n"


if __name__ == "__main__":
    main()
