"""CPU tests of the oracle (oracle/): known-answer vectors, algebraic identities, and the
committed golden fixtures (tests/golden/*.json) re-checked against the restatement.

Pins: SHA3-256 (FIPS-202 KAT), ChaCha20 (RFC 7539 §2.3.2 and A.1 block
vectors), the zcash/pairing-0.14 compressed encodings of the G1/G2 generators, curve/subgroup
membership, bilinearity.  threshold_crypto's own byte conventions (hash_g2, xor_with_hash,
parity) have no known-answer vectors anywhere in the reference: parity unpinned.
"""
import json
import os

import pytest

from oracle import bls12_381 as C
from oracle import tc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


# ------------------------------------------------------------------ known-answer vectors
def test_sha3_256_kat():
    assert tc.sha3_256(b"").hex() == "a7ffc6f8bf1ed76651c14756a061d662f580ff4de43b49fa82d80a4b80f8434a"
    assert tc.sha3_256(b"abc").hex() == "3a985da74fe225b2045c172d6bd390bd855f086e3e9d525b46bfe24511431532"


def test_chacha20_rfc7539_block():
    # RFC 7539 §2.3.2: key 00..1f, counter 1, nonce 00000009 0000004a 00000000
    key = [int.from_bytes(bytes(range(4 * i, 4 * i + 4)), "little") for i in range(8)]
    nonce = bytes.fromhex("000000090000004a00000000")
    w13 = int.from_bytes(nonce[0:4], "little")
    counter = 1 | (w13 << 32)
    nw = (int.from_bytes(nonce[4:8], "little"), int.from_bytes(nonce[8:12], "little"))
    out = tc.chacha20_block(key, counter, nw)
    assert out[:4] == [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3]
    assert out[12:] == [0xD19C12B5, 0xB94E16DE, 0xE883D0CB, 0x4E3C50A2]


def test_chacha20_zero_key_stream():
    # RFC 7539 A.1 test vector #1 (all-zero key/nonce, block 0)
    rng = tc.ChaChaRng(bytes(32))
    stream = b"".join(rng.next_u32().to_bytes(4, "little") for _ in range(16))
    assert stream.hex().startswith("76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7")


def test_generator_encodings():
    assert C.g1_compress(C.G1_GEN).hex() == (
        "97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
    assert C.g2_compress(C.G2_GEN).hex() == (
        "93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
        "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8")
    assert C.g1_decompress(C.g1_compress(C.G1_GEN)) == C.G1_GEN
    assert C.g2_decompress(C.g2_compress(C.G2_GEN)) == C.G2_GEN


def test_curve_constants():
    x = -C.X_ABS
    assert C.R == x ** 4 - x ** 2 + 1
    assert C.P == (x - 1) ** 2 * C.R // 3 + x
    assert C.g1_on_curve(C.G1_GEN) and C.g2_on_curve(C.G2_GEN)
    assert C.g1_mul(C.G1_GEN, C.R) is None


@pytest.mark.slow
def test_bilinearity():
    a, b = 1234567, 7654321
    e = C.pairing(C.G1_GEN, C.G2_GEN)
    assert e != C.F12_ONE
    assert C.pairing(C.g1_mul(C.G1_GEN, a), C.g2_mul(C.G2_GEN, b)) == C.f12_pow(e, a * b)
    assert C.f12_pow(e, C.R) == C.F12_ONE


def test_lagrange_and_poly():
    coeffs = [5, 7, 11, 13]
    ys = [(i, tc.poly_eval(coeffs, i + 1)) for i in (0, 3, 5, 9)]
    acc = 0
    for lam, (_, y) in zip(tc.lagrange_coeffs_at_zero([i + 1 for i, _ in ys]), ys):
        acc = (acc + lam * y) % C.R
    assert acc == 5
    assert tc.coeff_pos(1, 2) == tc.coeff_pos(2, 1) == 4


# ------------------------------------------------------------------ golden fixtures
def test_golden_sign_fixture_consistent():
    d = load("threshold_sign_n10_t3.json")
    t = d["t"]
    pks = [C.g1_decompress(bytes.fromhex(h)) for h in d["pk_shares_compressed"]]
    for i, h in enumerate(d["pk_shares"]):
        assert C.g1_uncompressed(pks[i]).hex() == h
    # pk shares lie on the degree-t polynomial of the master key: interpolate t+1 of them at 0
    master = tc.interpolate(t, [(i, pks[i]) for i in range(d["n"])], C.g1_add, C.g1_mul)
    assert C.g1_compress(master).hex() == d["master_pk"]
    for doc in d["docs"]:
        hm = C.g2_decompress(bytes.fromhex(doc["hash_compressed"]))
        assert C.g2_uncompressed(hm).hex() == doc["hash"]
        kinds = {s["kind"] for s in doc["shares"]}
        assert "valid" in kinds and len(kinds) > 1
        for s in doc["shares"]:
            assert s["valid"] == (s["kind"] == "valid")
        combined = C.g2_decompress(bytes.fromhex(doc["combined"]))
        assert tc.signature_parity(combined) == doc["parity"]


@pytest.mark.slow
def test_golden_sign_verdicts_recomputed():
    d = load("threshold_sign_n10_t3.json")
    doc = d["docs"][0]
    hm = C.g2_decompress(bytes.fromhex(doc["hash_compressed"]))
    for s in doc["shares"][:4]:
        sig = bytes.fromhex(s["sig"])
        sig_pt = None  # 0x40 flag: point at infinity
        if not sig[0] & 0x40:
            x = (int.from_bytes(sig[48:96], "big"), int.from_bytes(sig[0:48], "big"))
            y = (int.from_bytes(sig[144:192], "big"), int.from_bytes(sig[96:144], "big"))
            sig_pt = (x, y)
        pk = C.g1_decompress(bytes.fromhex(d["pk_shares_compressed"][s["idx"]]))
        assert tc.verify_g2(pk, sig_pt, hm) == s["valid"]


def test_golden_decrypt_fixture_consistent():
    d = load("threshold_decrypt_n10_t3.json")
    for ct in d["ciphertexts"]:
        assert ct["ct_valid"] is True and ct["bad_w_valid"] is False
        assert bytes.fromhex(ct["plaintext"]) == bytes.fromhex(ct["msg"])
        assert len(ct["combine_indices"]) == d["t"] + 1


def test_golden_dkg_rows():
    d = load("sync_key_gen_n4_t2.json")
    t = d["t"]
    assert len(d["commit"]) == (t + 1) * (t + 2) // 2
    for row in d["rows"][:2]:
        polyc = [int(c, 16) for c in row["row_poly"]]
        want = [C.g1_uncompressed(p).hex() for p in tc.poly_commitment(polyc)]
        assert want == row["row_commit"]
    bad = [a for a in d["acks"] if not a["valid"]]
    assert len(bad) == 1 and (bad[0]["x"], bad[0]["y"]) == (2, 3)
