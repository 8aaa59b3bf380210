"""Product host stage (csrc/host_hash.cpp through hbbft_amd.hoststage) against the oracle and the
golden fixtures: hash_g2, hash_g1_g2, xor_with_hash, Signature::parity, compression, secret-scalar
multiplication and encrypt_with_rng.  CPU only (no GPU is involved in the host stage).  Bar:
byte-identical outputs."""
import json
import os
import random

import pytest

from oracle import bls12_381 as C
from oracle import tc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def hs():
    from hbbft_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libhbbft_hip.so not built")
    from hbbft_amd import hoststage
    return hoststage


def abi_g1(pt):
    if pt is None:
        return bytes(96)
    return pt[0].to_bytes(48, "little") + pt[1].to_bytes(48, "little")


def abi_g2(pt):
    if pt is None:
        return bytes(192)
    (x0, x1), (y0, y1) = pt
    return b"".join(v.to_bytes(48, "little") for v in (x0, x1, y0, y1))


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_hash_g2_matches_oracle_and_golden(hs):
    d = load("threshold_sign_n10_t3.json")
    docs = [bytes.fromhex(doc["doc"]) for doc in d["docs"]]
    got = hs.hash_g2(docs, threads=2)
    for doc, g, rec in zip(docs, got, d["docs"]):
        assert g == abi_g2(tc.hash_g2(doc))
        assert hs.g2_compress([g])[0] == bytes.fromhex(rec["hash_compressed"])
    # empty, short, one-block-boundary and multi-block messages (SHA3 rate is 136 bytes)
    msgs = [b"", b"a", bytes(range(135)), bytes(range(136)), bytes(range(137)) * 3]
    assert hs.hash_g2(msgs) == [abi_g2(tc.hash_g2(m)) for m in msgs]


def test_hash_g1_g2_both_branches(hs):
    rng = random.Random(11)
    us = [C.g1_mul(C.G1_GEN, rng.randrange(1, C.R)) for _ in range(3)]
    vs = [bytes(32), bytes(range(64)), bytes(range(65))]  # <= 64 used as is, > 64 hashed first
    got = hs.hash_g1_g2([abi_g1(u) for u in us], vs)
    assert got == [abi_g2(tc.hash_g1_g2(u, v)) for u, v in zip(us, vs)]


def test_xor_with_hash_and_decrypt_golden(hs):
    d = load("threshold_decrypt_n10_t3.json")
    rng = random.Random(5)
    g = [C.g1_mul(C.G1_GEN, rng.randrange(1, C.R)) for _ in range(4)]
    datas = [b"", b"x", bytes(range(200)), bytes(70)]
    got = hs.xor_with_hash([abi_g1(p) for p in g], datas)
    assert got == [tc.xor_with_hash(p, v) for p, v in zip(g, datas)]
    assert "ciphertexts" in d


def test_signature_parity_and_compress(hs):
    rng = random.Random(9)
    pts = [C.g2_mul(C.G2_GEN, rng.randrange(1, C.R)) for _ in range(6)] + [None]
    assert hs.signature_parity([abi_g2(p) for p in pts]) == [tc.signature_parity(p) for p in pts]
    assert hs.g2_compress([abi_g2(p) for p in pts]) == [C.g2_compress(p) for p in pts]
    g1s = [C.g1_mul(C.G1_GEN, rng.randrange(1, C.R)) for _ in range(6)] + [None]
    assert hs.g1_compress([abi_g1(p) for p in g1s]) == [C.g1_compress(p) for p in g1s]
    # golden combined signatures: parity bit and compressed bytes
    from hbbft_amd.engine import g2_abi_from_uncompressed
    d = load("threshold_sign_n10_t3.json")
    sigs = [g2_abi_from_uncompressed(bytes.fromhex(doc["combined_uncompressed"])) for doc in d["docs"]]
    assert hs.signature_parity(sigs) == [bool(doc["parity"]) for doc in d["docs"]]
    assert [c.hex() for c in hs.g2_compress(sigs)] == [doc["combined"] for doc in d["docs"]]


def test_secret_scalar_mul(hs):
    rng = random.Random(3)
    ks = [rng.randrange(0, 1 << 256) for _ in range(4)] + [0, C.R]
    p1 = [C.g1_mul(C.G1_GEN, rng.randrange(1, C.R)) for _ in ks]
    p2 = [C.g2_mul(C.G2_GEN, rng.randrange(1, C.R)) for _ in ks]
    assert hs.g1_mul([abi_g1(p) for p in p1], ks) == [abi_g1(C.g1_mul(p, k % C.R)) for p, k in zip(p1, ks)]
    assert hs.g2_mul([abi_g2(p) for p in p2], ks) == [abi_g2(C.g2_mul(p, k % C.R)) for p, k in zip(p2, ks)]


def test_encrypt_matches_oracle(hs):
    rng = random.Random(21)
    sk = rng.randrange(1, C.R)
    pk = C.g1_mul(C.G1_GEN, sk)
    msgs = [b"", b"hello", bytes(range(100))]
    rs = [rng.randrange(1, C.R) for _ in msgs]
    got = hs.encrypt([abi_g1(pk)], msgs, rs)
    for (u, v, w), m, r in zip(got, msgs, rs):
        eu, ev, ew = tc.encrypt(pk, m, r)
        assert (u, v, w) == (abi_g1(eu), ev, abi_g2(ew))
        assert tc.ciphertext_verify((eu, ev, ew))
        # decrypting with the secret key recovers the message (SecretKey::decrypt)
        g = hs.g1_mul([u], [sk])[0]
        assert hs.xor_with_hash([g], [v])[0] == m


def test_bad_arguments(hs):
    from hbbft_amd._lib import HbhError
    with pytest.raises(HbhError):
        hs.g1_compress([b"\xff" * 96])  # coordinates >= p


def test_prefetch_coins_equals_hash_and_sign(hs):
    """honey_badger.prefetch_coins: the next epoch's BA coin documents (bincode((hb_id, epoch,
    proposer), BA epoch)) hashed and signed on the host-stage thread equal hash_g2 and sk * H."""
    from types import SimpleNamespace
    from hbbft_amd.binary_agreement import coin_document
    from hbbft_amd.honey_badger import prefetch_coins
    keys = SimpleNamespace(sks=[1234567, 89], pks=None)
    got = prefetch_coins(keys, 5, [0, 3], our=1, threads=2).result()
    docs = [coin_document(0, 5, p, 2) for p in (0, 3)]
    assert sorted(got) == sorted(docs)
    hashes = hs.hash_g2(docs)
    sigs = hs.g2_mul(hashes, [89, 89])
    for d, h, s in zip(docs, hashes, sigs):
        assert got[d] == (h, s)
