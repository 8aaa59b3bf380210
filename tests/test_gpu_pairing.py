"""GPU parity of the pairing-equality path against the oracle and the golden fixtures.

Bar: bit-exact (verdict bytes; canonical Fp12 coefficients of e(P,Q)^3)."""
import json
import os

import pytest

from oracle import bls12_381 as C
from hbbft_amd.engine import g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def f12_bytes(e):
    return b"".join(c.to_bytes(48, "little") for six in e for f2 in six for c in f2)


def test_pairing_value_matches_oracle(engine):
    P = [C.g1_mul(C.G1_GEN, k) for k in (1, 5, 12345)]
    Q = [C.g2_mul(C.G2_GEN, k) for k in (1, 7, 999)]
    out = engine.dbg_pairing([g1a(C.g1_uncompressed(p)) for p in P], [g2a(C.g2_uncompressed(q)) for q in Q])
    for k, (p, q) in enumerate(zip(P, Q)):
        assert out[k] == f12_bytes(C.f12_pow(C.pairing(p, q), 3)), k


def test_pairing_with_infinity_is_one(engine):
    one = f12_bytes(C.F12_ONE)
    out = engine.dbg_pairing([bytes(96), g1a(C.g1_uncompressed(C.G1_GEN))],
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


def test_sig_share_verdicts_golden(engine):
    pks, sigs, hashes, didx, exp = sign_batch(load("threshold_sign_n10_t3.json"))
    assert list(engine.verify_sig_shares(pks, sigs, hashes, didx)) == exp


def test_sig_share_verdicts_golden_tiled(engine):
    """Ragged batch (not a multiple of the workgroup) with shuffled document indices."""
    pks, sigs, hashes, didx, exp = sign_batch(load("threshold_sign_n10_t3.json"))
    reps = 13
    order = [(i * 7 + r) % len(pks) for r in range(reps) for i in range(len(pks))]
    v = engine.verify_sig_shares([pks[i] for i in order], [sigs[i] for i in order], hashes, [didx[i] for i in order])
    assert list(v) == [exp[i] for i in order]


def test_dec_share_and_ciphertext_verdicts_golden(engine):
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
    assert list(engine.verify_dec_shares(shares, pks, huv, w, cidx)) == exp
    u = [g1a(bytes.fromhex(ct["u"])) for ct in d["ciphertexts"]]
    bad_w = [g2a(bytes.fromhex(ct["bad_w"])) for ct in d["ciphertexts"]]
    assert list(engine.verify_ciphertexts(u + u, w + bad_w, huv + huv)) == [1, 1, 0, 0]


def test_empty_batch(engine):
    assert engine.verify_sig_shares(b"", b"", bytes(192), None) == b""
