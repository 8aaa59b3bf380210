"""Engine pool (hbh_pool_*, multi-device fan-out inside the ABI): two shards on device 0 -- two
engines, two streams, two host threads -- split every batch by instance and gather the outputs in
the caller's order, byte-identical to the single-engine call.  Instances are interleaved in the
batch (not sorted) so the split/scatter is exercised; both shards must have launched work."""
import random

import pytest

from oracle import bls12_381 as C
from oracle import tc
from hbbft_amd._lib import STAGE_CURVE, STAGE_PAIRING, HbhError
from hbbft_amd.engine import Pool, g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a

pytestmark = pytest.mark.gpu
R = C.R
G1 = g1a(C.g1_uncompressed(C.G1_GEN))
G2 = g2a(C.g2_uncompressed(C.G2_GEN))


@pytest.fixture(scope="module")
def pool():
    p = Pool([0, 0])
    yield p
    p.close()


def shard_launches(pool, stage):
    return [pool.shard_engine(s).stage_time(stage)[1] for s in range(pool.shards)]


def profiling(pool, on):
    for s in range(pool.shards):
        pool.shard_engine(s).set_profiling(on)


def test_pool_sig_and_dec_shares(engine, pool):
    rng = random.Random(9)
    n_nodes, t, ndocs = 16, 5, 12
    coeffs = [rng.randrange(1, R) for _ in range(t + 1)]
    sks = [tc.poly_eval(coeffs, i + 1) for i in range(n_nodes)]
    pks = engine.g1_mul([G1] * n_nodes, sks)
    hashes = engine.g2_mul([G2] * ndocs, [rng.randrange(1, R) for _ in range(ndocs)])
    items = [(m, j) for m in range(ndocs) for j in range(n_nodes)]
    rng.shuffle(items)  # instances interleaved
    bad = set(rng.sample(range(len(items)), 9))
    sigs = engine.g2_mul([hashes[m] for m, _ in items],
                         [rng.randrange(1, R) if k in bad else sks[j] for k, (m, j) in enumerate(items)])
    args = ([pks[j] for _, j in items], sigs, hashes, [m for m, _ in items])
    profiling(pool, True)
    v = pool.verify_sig_shares(*args)
    assert all(k > 0 for k in shard_launches(pool, STAGE_PAIRING))  # both shards ran
    profiling(pool, False)
    assert v == engine.verify_sig_shares(*args)
    assert v == bytes(0 if k in bad else 1 for k in range(len(items)))
    # decryption shares over ciphertexts (U = g1 r, W = H r)
    rs = [rng.randrange(1, R) for _ in range(ndocs)]
    us = engine.g1_mul([G1] * ndocs, rs)
    ws = engine.g2_mul(hashes, rs)
    shares = engine.g1_mul([us[m] for m, _ in items],
                           [rng.randrange(1, R) if k in bad else sks[j] for k, (m, j) in enumerate(items)])
    dargs = (shares, [pks[j] for _, j in items], hashes, ws, [m for m, _ in items])
    assert pool.verify_dec_shares(*dargs) == engine.verify_dec_shares(*dargs)
    # combines: one per document, first t+1 valid shares
    idx, pts, gidx, gpts = [], [], [], []
    for m in range(ndocs):
        ks = [k for k, (mm, _) in enumerate(items) if mm == m and k not in bad][: t + 1]
        idx.append([items[k][1] for k in ks])
        pts.append([sigs[k] for k in ks])
        gpts.append([shares[k] for k in ks])
    mpk = engine.g1_mul([G1], [coeffs[0]])[0]
    assert pool.combine_verify_g2(t, idx, pts, mpk, hashes) == engine.combine_verify_g2(t, idx, pts, mpk, hashes)
    out, st = pool.interpolate_g1(t, idx, gpts)
    assert (out, st) == engine.interpolate_g1(t, idx, gpts)
    assert out == engine.g1_mul(us, [coeffs[0]] * ndocs)


def test_pool_bivar_ack_check(engine, pool):
    rng = random.Random(4)
    t, nparts = 2, 5
    npos = (t + 1) * (t + 2) // 2
    coefs = [[rng.randrange(1, R) for _ in range(npos)] for _ in range(nparts)]
    flat = engine.g1_mul([G1] * (nparts * npos), [c for cs in coefs for c in cs])
    parts = [flat[p * npos:(p + 1) * npos] for p in range(nparts)]
    acks = [(p, x, y) for p in range(nparts) for x in (1, 3) for y in range(1, 7)]
    rng.shuffle(acks)
    vals = [rng.randrange(0, R) for _ in acks]
    a = (t, parts, [p for p, _, _ in acks], [x for _, x, _ in acks], [y for _, _, y in acks], vals)
    profiling(pool, True)
    got = pool.bivar_ack_check(*a)
    assert all(k > 0 for k in shard_launches(pool, STAGE_CURVE))
    profiling(pool, False)
    assert got == engine.bivar_ack_check(*a)


def test_pool_errors(pool):
    with pytest.raises(HbhError, match="instance index out of range"):
        pool.verify_sig_shares([G1], [G2], [G2], [3])
    with pytest.raises(AttributeError):
        pool.g1_mul([G1], [1])
    assert pool.shards == 2
