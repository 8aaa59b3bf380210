"""BASELINE.json configs[1]-[3] at full size on the GPU, checked against the construction and, on a
sample, against the C oracle (oracle/c/bls_cpu.c, the pairing 0.14 restatement):

* configs[1]: 65,536 ThresholdSign share checks (N=64, f=21, 1,024 documents, 1/64 forged), AUTO
  (the lane-pair kernel) and WAVE (one wave per check), verdicts equal to each other and to the
  construction;
  256 sampled verdicts recomputed by the C oracle; 1,024 combines + master verify.
* configs[2]: 65,536 decryption-share checks over 1,024 ciphertexts + 1,024 G1 combines, each equal
  to U * msk (C oracle).
* configs[3]: the 10,000 Ack checks (t=33) of one SyncKeyGen node over 100 Parts with 595-point
  commitments, verdicts equal to the construction; a C-oracle sample of BivarCommitment::evaluate.
"""
import random

import numpy as np
import pytest

from oracle import bls12_381 as C
from oracle import cbls, tc
from hbbft_amd._lib import IMPL_AUTO, IMPL_OCT, IMPL_QUAD, IMPL_WAVE, IMPL_WAVE2
from hbbft_amd.engine import g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a

pytestmark = pytest.mark.gpu
R = C.R
G1 = g1a(C.g1_uncompressed(C.G1_GEN))
G2 = g2a(C.g2_uncompressed(C.G2_GEN))
N, T, NDOCS = 64, 21, 1024


def keyset(engine, rng, n, t):
    coeffs = [rng.randrange(1, R) for _ in range(t + 1)]
    sks = [tc.poly_eval(coeffs, i + 1) for i in range(n)]
    pts = engine.g1_mul([G1] * (n + 1), sks + [coeffs[0]])
    return coeffs, sks, pts[:n], pts[n]


@pytest.fixture(scope="module")
def sign_batch(engine):
    rng = random.Random(65536)
    coeffs, sks, pks, mpk = keyset(engine, rng, N, T)
    hashes = engine.g2_mul([G2] * NDOCS, [rng.randrange(1, R) for _ in range(NDOCS)])
    bad = {m * N + (m * 37) % N for m in range(NDOCS)}
    bases, scal = [], []
    for i in range(NDOCS * N):
        m, j = divmod(i, N)
        if i in bad:
            bases.append(G2 if m % 2 else hashes[(m + 1) % NDOCS])  # random point / another document's share
            scal.append(rng.randrange(1, R) if m % 2 else sks[j])
        else:
            bases.append(hashes[m])
            scal.append(sks[j])
    sigs = engine.g2_mul(bases, scal)
    expected = bytes(0 if i in bad else 1 for i in range(NDOCS * N))
    return dict(coeffs=coeffs, sks=sks, pks=pks, mpk=mpk, hashes=hashes, sigs=sigs, expected=expected)


@pytest.mark.parametrize("impl", [IMPL_AUTO, IMPL_WAVE, IMPL_QUAD, IMPL_OCT, IMPL_WAVE2],
                         ids=["auto", "wave", "quad", "oct", "wave2"])
def test_config1_65536_sig_shares(engine, sign_batch, impl):
    b = sign_batch
    n = NDOCS * N
    engine.set_pairing_impl(impl)
    try:
        v = engine.verify_sig_shares([b["pks"][i % N] for i in range(n)], b["sigs"], b["hashes"],
                                     [i // N for i in range(n)])
    finally:
        engine.set_pairing_impl(IMPL_AUTO)
    assert v == b["expected"]
    rng = random.Random(7)
    sample = sorted(rng.sample(range(n), 256)) + [m * N + (m * 37) % N for m in range(4)]
    for i in sample:
        assert cbls.verify_g2(b["pks"][i % N], b["sigs"][i], b["hashes"][i // N]) == bool(v[i]), i


@pytest.mark.parametrize("n", [512, 576, 4096, 4160, 8192, 8256, 16384, 16448, 32768, 32832, 49152, 49216],
                         ids=["wave2_max", "wave_min", "wave_max", "oct_min", "oct_max", "quad_min", "quad_max",
                              "pair_min", "split_lo", "split_min", "split_max", "pair2_min"])
def test_config1_at_auto_thresholds(engine, sign_batch, n):
    """Every kernel on both sides of the AUTO boundaries (HBH_AUTO_WAVE_MAX = 4,096 checks, 64
    documents of configs[1]; HBH_AUTO_OCT_MAX = 8,192, 128 documents; HBH_AUTO_QUAD_MAX = 16,384, 256
    documents; the PAIR + rest split of (32,768, 49,152]; one more document past each): WAVE walks both
    G2 sides, OCT, QUAD and PAIR read H's line table; verdicts equal the construction."""
    b = sign_batch
    from hbbft_amd._lib import IMPL_PAIR, IMPL_QUAD
    for impl in (IMPL_WAVE2, IMPL_WAVE, IMPL_OCT, IMPL_QUAD, IMPL_PAIR, IMPL_AUTO):
        engine.set_pairing_impl(impl)
        try:
            v = engine.verify_sig_shares([b["pks"][i % N] for i in range(n)], b["sigs"][:n], b["hashes"][:n // N],
                                         [i // N for i in range(n)])
        finally:
            engine.set_pairing_impl(IMPL_AUTO)
        assert v == b["expected"][:n], impl


@pytest.mark.parametrize("extra", [4096, 8192, 16384, 40960], ids=["wave_rest", "oct_rest", "quad_rest", "split_rest"])
def test_config1_auto_beyond_one_round(engine, sign_batch, extra):
    """AUTO above 49,152 checks: one round of 65,536 on PAIR, then the remainder by size (WAVE /
    OCT / QUAD / PAIR + rest) on the same stream -- the batch is configs[1] followed by its first `extra`
    checks again; verdicts equal the construction's."""
    b = sign_batch
    n = NDOCS * N
    idx = list(range(n)) + list(range(extra))
    v = engine.verify_sig_shares([b["pks"][i % N] for i in idx], [b["sigs"][i] for i in idx], b["hashes"],
                                 [i // N for i in idx])
    assert v == b["expected"] + b["expected"][:extra]


def test_config1_combines(engine, sign_batch):
    """combine_and_verify_sig for all 1,024 documents (first 22 valid shares) in one call."""
    b = sign_batch
    idx, pts = [], []
    for m in range(NDOCS):
        ids = [k for k in range(N) if b["expected"][m * N + k]][: T + 1]
        idx.append(ids)
        pts.append([b["sigs"][m * N + k] for k in ids])
    out, st, v = engine.combine_verify_g2(T, idx, pts, b["mpk"], b["hashes"])
    assert st == [0] * NDOCS and v == b"\x01" * NDOCS
    for m in (0, 1, 511, 1023):
        assert out[m] == cbls.g2_mul(b["hashes"][m], b["coeffs"][0])


def test_config2_65536_dec_shares_and_combines(engine):
    rng = random.Random(2)
    coeffs, sks, pks, mpk = keyset(engine, rng, N, T)
    rs = [rng.randrange(1, R) for _ in range(NDOCS)]
    hs = [rng.randrange(1, R) for _ in range(NDOCS)]
    us = engine.g1_mul([G1] * NDOCS, rs)
    huv = engine.g2_mul([G2] * NDOCS, hs)
    ws = engine.g2_mul([G2] * NDOCS, [h * r % R for h, r in zip(hs, rs)])
    n = NDOCS * N
    bad = {c * N + (c * 29) % N for c in range(NDOCS)}
    shares = engine.g1_mul([us[i // N] for i in range(n)],
                           [rng.randrange(1, R) if i in bad else sks[i % N] for i in range(n)])
    v = engine.verify_dec_shares(shares, [pks[i % N] for i in range(n)], huv, ws, [i // N for i in range(n)])
    assert v == bytes(0 if i in bad else 1 for i in range(n))
    for i in sorted(random.Random(3).sample(range(n), 64)) + sorted(bad)[:4]:
        c = i // N
        assert cbls.pairing_eq(shares[i], huv[c], pks[i % N], ws[c]) == bool(v[i]), i
    idx, pts = [], []
    for c in range(NDOCS):
        ids = [k for k in range(N) if v[c * N + k]][: T + 1]
        idx.append(ids)
        pts.append([shares[c * N + k] for k in ids])
    out, st = engine.interpolate_g1(T, idx, pts)
    assert st == [0] * NDOCS
    assert out == engine.g1_mul(us, [coeffs[0]] * NDOCS)
    for c in (0, 17, 1023):
        assert out[c] == cbls.g1_mul(us[c], coeffs[0])


def test_config3_10000_acks(engine):
    rng = random.Random(33)
    n_nodes, t = 100, 33
    npos = (t + 1) * (t + 2) // 2
    coefs = [[rng.randrange(1, R) for _ in range(npos)] for _ in range(n_nodes)]
    flat = engine.g1_mul([G1] * (n_nodes * npos), [x for c in coefs for x in c])
    parts = [flat[p * npos:(p + 1) * npos] for p in range(n_nodes)]

    def cp(i, j):
        return j * (j + 1) // 2 + i if i <= j else i * (i + 1) // 2 + j

    x = 5
    pidx, xs, ys, vals = [], [], [], []
    for p in range(n_nodes):
        xp = [pow(x, i, R) for i in range(t + 1)]
        row = [sum(coefs[p][cp(i, j)] * xp[i] for i in range(t + 1)) % R for j in range(t + 1)]
        for y in range(1, n_nodes + 1):
            val = 0
            for j in reversed(range(t + 1)):
                val = (val * y + row[j]) % R
            pidx.append(p)
            xs.append(x)
            ys.append(y)
            vals.append(val)
    bad = set(range(3, len(vals), 97))
    for a in bad:
        vals[a] = (vals[a] + 1) % R
    v = engine.bivar_ack_check(t, parts, pidx, xs, ys, vals)
    assert v == bytes(0 if a in bad else 1 for a in range(len(vals)))
    for a in (0, 3, 4999, 9999):
        assert (cbls.bivar_evaluate(t, parts[pidx[a]], xs[a], ys[a]) == cbls.g1_mul(G1, vals[a])) == bool(v[a])


@pytest.mark.parametrize("n", [1024, 2048])
def test_dec_shares_wave_tabled_sides(engine, n):
    """Round 6: a WAVE call of >= 1,024 checks whose two G2 sides are both shared (decryption shares:
    H_uv and W per ciphertext) tables both and runs the combined-line TT program (138 Miller stages);
    WAVE, WAVE2 (both sides walked) and PAIR give the construction's verdicts."""
    from hbbft_amd._lib import IMPL_PAIR
    rng = random.Random(100 + n)
    coeffs, sks, pks, mpk = keyset(engine, rng, N, T)
    ncts = n // N
    rs = [rng.randrange(1, R) for _ in range(ncts)]
    hs = [rng.randrange(1, R) for _ in range(ncts)]
    us = engine.g1_mul([G1] * ncts, rs)
    huv = engine.g2_mul([G2] * ncts, hs)
    ws = engine.g2_mul([G2] * ncts, [h * r % R for h, r in zip(hs, rs)])
    bad = {c * N + (c * 13) % N for c in range(ncts)} | {5, n - 2}
    shares = engine.g1_mul([us[i // N] for i in range(n)],
                           [rng.randrange(1, R) if i in bad else sks[i % N] for i in range(n)])
    want = bytes(0 if i in bad else 1 for i in range(n))
    for impl in (IMPL_WAVE, IMPL_WAVE2, IMPL_PAIR):
        engine.set_pairing_impl(impl)
        try:
            v = engine.verify_dec_shares(shares, [pks[i % N] for i in range(n)], huv, ws, [i // N for i in range(n)])
        finally:
            engine.set_pairing_impl(IMPL_AUTO)
        assert v == want, impl
