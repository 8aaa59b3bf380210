"""GPU parity of the pairing-equality path against the oracle and the golden fixtures.

Bar: bit-exact (verdict bytes; canonical Fp12 coefficients of e(P,Q)^3)."""
import json
import os

import pytest

from oracle import bls12_381 as C
from hbbft_amd.engine import g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(params=[4, 5, 6, 7, 8, 3], ids=["pair", "wave", "quad", "oct", "wave2", "auto"])
def eng(engine, request):
    """Every pairing implementation (HBH_IMPL_PAIR, HBH_IMPL_WAVE, HBH_IMPL_QUAD, HBH_IMPL_OCT,
    HBH_IMPL_WAVE2) and the default HBH_IMPL_AUTO must give identical results."""
    engine.set_pairing_impl(request.param)
    yield engine
    engine.set_pairing_impl(3)


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def f12_bytes(e):
    return b"".join(c.to_bytes(48, "little") for six in e for f2 in six for c in f2)


def test_pairing_value_matches_oracle(eng):
    P = [C.g1_mul(C.G1_GEN, k) for k in (1, 5, 12345)]
    Q = [C.g2_mul(C.G2_GEN, k) for k in (1, 7, 999)]
    out = eng.dbg_pairing([g1a(C.g1_uncompressed(p)) for p in P], [g2a(C.g2_uncompressed(q)) for q in Q])
    for k, (p, q) in enumerate(zip(P, Q)):
        assert out[k] == f12_bytes(C.f12_pow(C.pairing(p, q), 3)), k


def test_pairing_with_infinity_is_one(eng):
    one = f12_bytes(C.F12_ONE)
    out = eng.dbg_pairing([bytes(96), g1a(C.g1_uncompressed(C.G1_GEN))],
                             [g2a(C.g2_uncompressed(C.G2_GEN)), bytes(192)])
    assert out == [one, one]


def sign_batch(d):
    pks, sigs, hashes, didx, exp = [], [], [], [], []
    for di, doc in enumerate(d["docs"]):
        hashes.append(g2a(bytes.fromhex(doc["hash"])))
        for s in doc["shares"]:
            pks.append(g1a(bytes.fromhex(d["pk_shares"][s["idx"]])))
            sigs.append(g2a(bytes.fromhex(s["sig"])))
            didx.append(di)
            exp.append(int(s["valid"]))
    return pks, sigs, hashes, didx, exp


def test_sig_share_verdicts_golden(eng):
    pks, sigs, hashes, didx, exp = sign_batch(load("threshold_sign_n10_t3.json"))
    assert list(eng.verify_sig_shares(pks, sigs, hashes, didx)) == exp


def test_sig_share_verdicts_golden_tiled(eng):
    """Ragged batch (not a multiple of the workgroup) with shuffled document indices."""
    pks, sigs, hashes, didx, exp = sign_batch(load("threshold_sign_n10_t3.json"))
    reps = 13
    order = [(i * 7 + r) % len(pks) for r in range(reps) for i in range(len(pks))]
    v = eng.verify_sig_shares([pks[i] for i in order], [sigs[i] for i in order], hashes, [didx[i] for i in order])
    assert list(v) == [exp[i] for i in order]


def test_dec_share_and_ciphertext_verdicts_golden(eng):
    d = load("threshold_decrypt_n10_t3.json")
    shares, pks, huv, w, cidx, exp = [], [], [], [], [], []
    for ci, ct in enumerate(d["ciphertexts"]):
        huv.append(g2a(bytes.fromhex(ct["huv"])))
        w.append(g2a(bytes.fromhex(ct["w"])))
        for s in ct["shares"]:
            shares.append(g1a(bytes.fromhex(s["share"])))
            pks.append(g1a(bytes.fromhex(d["pk_shares"][s["idx"]])))
            cidx.append(ci)
            exp.append(int(s["valid"]))
    assert list(eng.verify_dec_shares(shares, pks, huv, w, cidx)) == exp
    u = [g1a(bytes.fromhex(ct["u"])) for ct in d["ciphertexts"]]
    bad_w = [g2a(bytes.fromhex(ct["bad_w"])) for ct in d["ciphertexts"]]
    assert list(eng.verify_ciphertexts(u + u, w + bad_w, huv + huv)) == [1, 1, 0, 0]


def test_empty_batch(eng):
    assert eng.verify_sig_shares(b"", b"", bytes(192), None) == b""


def test_implementations_agree_random_batch(engine):
    """A 1,003-check random batch (valid, swapped, infinity, ragged vs the 128-checks-per-workgroup
    lane-pair layout): both implementations and the C oracle agree on every verdict."""
    import random
    from oracle import cbls
    rng = random.Random(7)
    g1, g2 = g1a(C.g1_uncompressed(C.G1_GEN)), g2a(C.g2_uncompressed(C.G2_GEN))
    hs = [cbls.g2_mul(g2, rng.randrange(1, C.R)) for _ in range(3)]
    sk = [rng.randrange(1, C.R) for _ in range(7)]
    pks = [cbls.g1_mul(g1, k) for k in sk]
    n = 1003
    P, S, D, want = [], [], [], []
    for i in range(n):
        d, j = i % 3, i % 7
        kind = i % 11
        pk, sig = pks[j], cbls.g2_mul(hs[d], sk[j])
        if kind == 3:
            sig = cbls.g2_mul(hs[(d + 1) % 3], sk[j])
        elif kind == 5:
            pk = pks[(j + 1) % 7]
        elif kind == 7:
            pk, sig = bytes(96), bytes(192)
        P.append(pk), S.append(sig), D.append(d)
    for i in range(0, n, 97):
        want.append((i, cbls.verify_g2(P[i], S[i], hs[D[i]])))
    try:
        engine.set_pairing_impl(4)
        v0 = engine.verify_sig_shares(P, S, hs, D)
        engine.set_pairing_impl(5)
        v5 = engine.verify_sig_shares(P, S, hs, D)
        engine.set_pairing_impl(6)
        v6 = engine.verify_sig_shares(P, S, hs, D)
        engine.set_pairing_impl(8)
        v8 = engine.verify_sig_shares(P, S, hs, D)
    finally:
        engine.set_pairing_impl(3)
    assert v5 == v0
    assert v6 == v0
    assert v8 == v0
    for i, w in want:
        assert v0[i] == int(w), i
    assert sum(v0) == sum(1 for i in range(n) if i % 11 not in (3, 5))


def test_verify_signatures_public_key_verify(eng):
    """PublicKey::verify for DHB signed votes / key-gen messages (votes.rs:153-158,
    dynamic_honey_badger.rs:514-526): valid, wrong message, wrong key, pk = sig = O (verifies:
    pairing with O is 1) -- verdicts equal the C oracle's."""
    import random
    from oracle import cbls
    rng = random.Random(157)
    G1 = g1a(C.g1_uncompressed(C.G1_GEN))
    G2 = g2a(C.g2_uncompressed(C.G2_GEN))
    sks = [rng.randrange(1, C.R) for _ in range(4)]
    pks = [cbls.g1_mul(G1, k) for k in sks]
    hs = [cbls.g2_mul(G2, rng.randrange(1, C.R)) for _ in range(4)]
    sigs = [cbls.g2_mul(h, k) for h, k in zip(hs, sks)]
    items = [(pks[0], sigs[0], hs[0]), (pks[1], sigs[1], hs[1]),
             (pks[2], sigs[2], hs[3]),          # signature of another message
             (pks[3], sigs[2], hs[2]),          # another voter's key
             (bytes(96), bytes(192), hs[0])]    # pk = O, sig = O
    got = eng.verify_signatures([a for a, _, _ in items], [b for _, b, _ in items], [c for _, _, c in items])
    want = [int(cbls.verify_g2(a, b, c)) for a, b, c in items]
    assert list(got) == want == [1, 1, 0, 0, 1]


@pytest.mark.parametrize("impl", [0, 1, 2], ids=["thread", "lane_coop", "thread_signed"])
def test_retired_impls_rejected(engine, impl):
    """HBH_IMPL_THREAD (0), HBH_IMPL_LANE_COOP (1) and HBH_IMPL_THREAD_SIGNED (2) are retired from
    the product build: selecting one is an argument error."""
    from hbbft_amd._lib import HbhError
    with pytest.raises(HbhError):
        engine.set_pairing_impl(impl)
