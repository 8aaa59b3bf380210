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


def test_hash_g2_many_messages(hs):
    """Round 5's hash path (norm-method square root, Budroni-Pintore image + GLS multiplication by
    h2 s^-1 mod r) against the oracle's textbook G2::rand (Fq2 exponentiation square root, double-and-add
    by the 636-bit h2) on 160 seeded messages of lengths 0..300: each hash samples ~2 curve x's, so
    the non-square / retry branch and both `greatest` choices are exercised many times over."""
    rng = random.Random(2024)
    msgs = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 301))) for _ in range(160)]
    assert hs.hash_g2(msgs, threads=2) == [abi_g2(tc.hash_g2(m)) for m in msgs]


def test_scalar_mul_edge_scalars(hs):
    """GLV (G1: k = k2 lambda + k1, lambda = z^2 - 1) and GLS (G2: base-|z| digits) split boundaries:
    scalars around lambda, |z|^i, r and 2^256 against the oracle's double-and-add of k mod r."""
    z, lam = C.X_ABS, C.X_ABS ** 2 - 1
    ks = [0, 1, 2, 15, 16, 17, lam - 1, lam, lam + 1, lam * lam - 1, lam * lam, lam * (lam + 1),
          z - 1, z, z + 1, z ** 2, z ** 3 - 1, z ** 3, z ** 3 + 1, C.R - 1, C.R, C.R + 1, 2 * C.R - 1, 2 * C.R,
          (1 << 255) - 1, 1 << 255, (1 << 256) - 1, int("5" * 76) % (1 << 256)]
    rng = random.Random(8)
    ks += [rng.randrange(0, 1 << 256) for _ in range(12)]
    p1 = C.g1_mul(C.G1_GEN, rng.randrange(1, C.R))
    p2 = C.g2_mul(C.G2_GEN, rng.randrange(1, C.R))
    assert hs.g1_mul([abi_g1(p1)] * len(ks), ks, threads=2) == [abi_g1(C.g1_mul(p1, k % C.R)) for k in ks]
    assert hs.g2_mul([abi_g2(p2)] * len(ks), ks, threads=2) == [abi_g2(C.g2_mul(p2, k % C.R)) for k in ks]
    # the point at infinity stays all-zero
    assert hs.g1_mul([bytes(96)], [5]) == [bytes(96)] and hs.g2_mul([bytes(192)], [5]) == [bytes(192)]


def test_fr_poly_eval(hs):
    """Poly::evaluate over Fr (hbh_fr_poly_eval, SyncKeyGen's rows and Ack values) against Horner in
    Python: random degree-33 polynomials, the all-(r-1) polynomial, x = 0, 1, 100 and 2^64 - 1."""
    rng = random.Random(9)
    polys = [[rng.randrange(C.R) for _ in range(34)] for _ in range(9)] + [[C.R - 1] * 34, [0] * 34]
    xs = [0, 1, 2, 100, (1 << 64) - 1]

    def ev(c, x):
        r = 0
        for a in reversed(c):
            r = (r * x + a) % C.R
        return r
    assert hs.fr_poly_eval(polys, xs, threads=2) == [[ev(c, x) for x in xs] for c in polys]
    assert hs.fr_poly_eval([[7]], [3]) == [[7]]
    from hbbft_amd._lib import HbhError
    with pytest.raises(HbhError):
        hs.fr_poly_eval([[C.R]], [1])


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


def test_encrypt_key_combs_equal_glv(hs):
    """hbh_encrypt builds a 4-bit comb for a key that encrypts >= 16 items of one call (SyncKeyGen's
    Acks: N values per key) and uses GLV otherwise: 2 x 20 items to two keys in one call equal the
    same items encrypted one call each, and the oracle on a sample."""
    rng = random.Random(41)
    sks = [rng.randrange(1, C.R) for _ in range(2)]
    pks = [C.g1_mul(C.G1_GEN, k) for k in sks]
    msgs = [bytes(rng.randrange(256) for _ in range(rng.choice([32, 100]))) for _ in range(40)]
    rs = [rng.randrange(1, C.R) for _ in msgs] + [0, C.R - 1]
    msgs += [b"x", b"y"]
    keys = [abi_g1(pks[i % 2]) for i in range(len(msgs))]
    got = hs.encrypt(keys, msgs, rs, threads=2)
    assert got == [hs.encrypt([k], [m], [r])[0] for k, m, r in zip(keys, msgs, rs)]
    for i in (0, 7, 40):
        eu, ev, ew = tc.encrypt(pks[i % 2], msgs[i], rs[i])
        assert got[i] == (abi_g1(eu), ev, abi_g2(ew))


def test_hash_bp_form(hs):
    """Q-form Ciphertext::verify inputs: [KCOF] hash_g1_g2_bp(U, V) == hash_g1_g2(U, V) and
    hash_bp_g1() == [KCOF^-1] g1, with KCOF = h2 s^-1 mod r from its definition."""
    z, lam = -C.X_ABS, C.P % C.R
    s_ = ((z * z - z - 1) + (z - 1) * lam + 2 * lam * lam) % C.R
    kcof = C.H2 * pow(s_, -1, C.R) % C.R
    rng = random.Random(12)
    us = [abi_g1(C.g1_mul(C.G1_GEN, rng.randrange(1, C.R))) for _ in range(6)]
    vs = [bytes(rng.randrange(256) for _ in range(ln)) for ln in (0, 32, 64, 65, 200, 1096)]
    q = hs.hash_g1_g2_bp(us, vs, threads=2)
    assert hs.g2_mul(q, [kcof] * len(q)) == hs.hash_g1_g2(us, vs)
    assert hs.hash_bp_g1() == abi_g1(C.g1_mul(C.G1_GEN, pow(kcof, -1, C.R)))


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
