"""GPU parity of the curve kernels (scalar multiplication, interpolate() for combine_signatures /
threshold decryption, SyncKeyGen bivariate commitments) against the C oracle and the golden
fixtures.  Bar: byte-identical canonical affine points, identical verdicts and statuses."""
import json
import os
import random

import pytest

from hbbft_amd._lib import HbhError

from oracle import bls12_381 as C
from oracle import cbls, tc
from hbbft_amd.engine import g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
G1 = g1a(C.g1_uncompressed(C.G1_GEN))
G2 = g2a(C.g2_uncompressed(C.G2_GEN))
EDGE_SCALARS = [0, 1, 2, 3, C.R - 1, C.R, C.R + 1, (1 << 256) - 1, 1 << 255]


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_g1_g2_mul(engine):
    rng = random.Random(1)
    ks = EDGE_SCALARS + [rng.randrange(1 << 256) for _ in range(40)]
    p1 = [cbls.g1_mul(G1, rng.randrange(1, C.R)) for _ in range(len(ks) - 1)] + [bytes(96)]
    assert engine.g1_mul(p1, ks) == [cbls.g1_mul(p, k) for p, k in zip(p1, ks)]
    p2 = [cbls.g2_mul(G2, rng.randrange(1, C.R)) for _ in range(len(ks) - 1)] + [bytes(192)]
    assert engine.g2_mul(p2, ks) == [cbls.g2_mul(p, k) for p, k in zip(p2, ks)]


def test_combine_signatures_golden(engine):
    d = load("threshold_sign_n10_t3.json")
    t = d["t"]
    for doc in d["docs"]:
        hm = C.g2_decompress(bytes.fromhex(doc["hash_compressed"]))
        idx = doc["combine_indices"]
        # the valid shares of these nodes: sk_i * H, recovered from the fixture's share list
        by_idx = {s["idx"]: s for s in doc["shares"]}
        pts = [g2a(bytes.fromhex(by_idx[i]["sig"])) for i in idx]
        out, st = engine.interpolate_g2(t, [idx], [pts])
        assert st == [0]
        assert g2a(bytes.fromhex(doc["combined_uncompressed"])) == out[0]
        # combined signature bytes (compressed, as the reference serialises it) and coin parity
        pt = (tuple(int.from_bytes(out[0][o:o + 48], "little") for o in (0, 48)),
              tuple(int.from_bytes(out[0][o:o + 48], "little") for o in (96, 144)))
        assert C.g2_compress(pt).hex() == doc["combined"]
        assert tc.signature_parity(pt) == doc["parity"]
        assert hm is not None



def test_interpolate_g2_n64_t21_matches_oracle(engine):
    """The BASELINE config's combine: 22 G2 shares of a degree-21 key, several index subsets."""
    rng = random.Random(21)
    t = 21
    coeffs = [rng.randrange(1, C.R) for _ in range(t + 1)]
    h = cbls.g2_mul(G2, rng.randrange(1, C.R))
    subsets = [list(range(t + 1)), sorted(rng.sample(range(64), t + 1)), list(range(63, 63 - t - 1, -1))]
    idx, pts = [], []
    for sub in subsets:
        idx.append(sub)
        pts.append([cbls.g2_mul(h, tc.poly_eval(coeffs, i + 1)) for i in sub])
    out, st = engine.interpolate_g2(t, idx, pts)
    want = cbls.g2_mul(h, coeffs[0])
    assert st == [0, 0, 0]
    assert out == [want, want, want]
    # same result as the reference-equivalent CPU interpolate on one subset
    assert cbls.combine_g2(t, idx[1], pts[1]) == (0, want)


def test_interpolate_batched_unsplit_mode(engine):
    """>= 128 combines per call take the throughput configuration of k_interp_endo (unsplit digit
    chains); < 128 the latency configuration (chunked chains + Horner tail).  Both must give the
    same group element: every (t+1)-subset of a degree-t key's shares interpolates to msk * H."""
    rng = random.Random(130)
    t = 21
    coeffs = [rng.randrange(1, C.R) for _ in range(t + 1)]
    h2 = cbls.g2_mul(G2, rng.randrange(1, C.R))
    h1 = cbls.g1_mul(G1, rng.randrange(1, C.R))
    s2 = [cbls.g2_mul(h2, tc.poly_eval(coeffs, i + 1)) for i in range(64)]
    s1 = [cbls.g1_mul(h1, tc.poly_eval(coeffs, i + 1)) for i in range(64)]
    subsets = [sorted(rng.sample(range(64), t + 1)) for _ in range(130)]
    subsets[77] = [subsets[77][1]] + subsets[77][1:]  # duplicate entry in one combine
    want2, want1 = cbls.g2_mul(h2, coeffs[0]), cbls.g1_mul(h1, coeffs[0])
    for n in (130, 3):
        out, st = engine.interpolate_g2(t, subsets[:n], [[s2[i] for i in sub] for sub in subsets[:n]])
        assert [s for c, s in enumerate(st) if c != 77] == [0] * (n - (n > 77))
        assert all(o == want2 for c, o in enumerate(out) if c != 77)
        out, st = engine.interpolate_g1(t, subsets[:n], [[s1[i] for i in sub] for sub in subsets[:n]])
        assert all(o == want1 for c, o in enumerate(out) if c != 77)
    assert st == [0, 0, 0]
    _, st = engine.interpolate_g2(t, subsets[:130], [[s2[i] for i in sub] for sub in subsets[:130]])
    assert st[77] == 5


def test_combine_verify_g2_matches_two_step(engine):
    """hbh_combine_verify_g2 (combine_and_verify_sig, src/threshold_sign.rs:249-270): same signature
    as interpolate_g2, master-key verdict as the C oracle's verify_g2; a wrong document hash gives
    VerificationFailed (verdict 0), a duplicate index DuplicateEntry."""
    rng = random.Random(22)
    t = 21
    msk = rng.randrange(1, C.R)
    coeffs = [msk] + [rng.randrange(1, C.R) for _ in range(t)]
    mpk = cbls.g1_mul(G1, msk)
    hs = [cbls.g2_mul(G2, rng.randrange(1, C.R)) for _ in range(3)]
    idx, pts = [], []
    for h in hs:
        sub = sorted(rng.sample(range(64), t + 1))
        idx.append(sub)
        pts.append([cbls.g2_mul(h, tc.poly_eval(coeffs, i + 1)) for i in sub])
    hashes = [hs[0], hs[1], hs[0]]  # third combine checked against the wrong document
    idx.append([idx[0][0]] + idx[0][:t])  # duplicate index
    pts.append(pts[0])
    hashes.append(hs[0])
    out, st, v = engine.combine_verify_g2(t, idx, pts, mpk, hashes)
    assert st == [0, 0, 0, 5]
    want = [cbls.g2_mul(h, msk) for h in hs]
    assert out[:3] == want
    assert list(v[:3]) == [1, 1, 0]
    assert [cbls.verify_g2(mpk, s, h) for s, h in zip(out[:3], hashes[:3])] == [True, True, False]
    golden = load("threshold_sign_n10_t3.json")
    doc = golden["docs"][0]
    by_idx = {s["idx"]: s for s in doc["shares"]}
    gi = doc["combine_indices"]
    out, st, v = engine.combine_verify_g2(golden["t"], [gi], [[g2a(bytes.fromhex(by_idx[i]["sig"])) for i in gi]],
                                          g1a(C.g1_uncompressed(C.g1_decompress(bytes.fromhex(golden["master_pk"])))),
                                          [g2a(bytes.fromhex(doc["hash"]))])
    assert st == [0] and v == b"\x01"
    assert out[0] == g2a(bytes.fromhex(doc["combined_uncompressed"]))


@pytest.fixture(scope="module")
def unsplit_engine():
    """An engine created with HBH_SPLIT_CHECK=0: every combine_and_verify_sig call interpolates, then
    verifies (the engine reads the switch at creation)."""
    from hbbft_amd.engine import Engine
    old = os.environ.get("HBH_SPLIT_CHECK")
    os.environ["HBH_SPLIT_CHECK"] = "0"
    try:
        e = Engine(0)
    finally:
        if old is None:
            del os.environ["HBH_SPLIT_CHECK"]
        else:
            os.environ["HBH_SPLIT_CHECK"] = old
    yield e
    e.close()


@pytest.fixture(scope="module")
def notree_engine():
    """An engine created with HBH_SPLIT_TREE=0: the split check multiplies the m + 1 Miller values in
    order in a second launch (wave_prod_fe) instead of up a tree inside the Miller launch."""
    from hbbft_amd.engine import Engine
    old = os.environ.get("HBH_SPLIT_TREE")
    os.environ["HBH_SPLIT_TREE"] = "0"
    try:
        e = Engine(0)
    finally:
        if old is None:
            del os.environ["HBH_SPLIT_TREE"]
        else:
            os.environ["HBH_SPLIT_TREE"] = old
    yield e
    e.close()


@pytest.mark.parametrize("t", [0, 1, 21, 70])
def test_combine_verify_split_matches_unsplit(engine, unsplit_engine, notree_engine, t):
    """Calls of at most 540 + 24 t one-pair Miller waves (ncomb x (t + 2)) take the split master check
    (partial Miller loops of (lambda_k g1, sigma_k) and (-mpk, H) beside the interpolation, one final
    exponentiation per combine); larger calls, and an engine created with HBH_SPLIT_CHECK=0, the
    interpolate-then-verify form.  Same signatures, statuses and verdicts on the same inputs:
    valid, wrong document, a tampered share (random G2 point), a share at infinity, a duplicate index."""
    rng = random.Random(700 + t)
    coeffs = [rng.randrange(1, C.R) for _ in range(t + 1)]
    mpk = cbls.g1_mul(G1, coeffs[0])
    hs = [cbls.g2_mul(G2, rng.randrange(1, C.R)) for _ in range(2)]
    n = max(t + 1, 8)
    shares = [[cbls.g2_mul(h, tc.poly_eval(coeffs, i + 1)) for i in range(n)] for h in hs]
    idx, pts, hashes = [], [], []
    for c in range(9):
        d = c % 2
        sub = sorted(rng.sample(range(n), t + 1))
        row = [shares[d][i] for i in sub]
        h = hs[d]
        if c == 2:
            h = hs[1 - d]                      # wrong document
        elif c == 3:
            row[-1] = cbls.g2_mul(G2, rng.randrange(1, C.R))  # tampered share
        elif c == 4:
            row[0] = bytes(192)                # share at infinity
        elif c == 5 and t > 0:
            sub = [sub[0]] + sub[:t]           # duplicate index
        idx.append(sub)
        pts.append(row)
        hashes.append(h)
    out9, st9, v9 = unsplit_engine.combine_verify_g2(t, idx, pts, mpk, hashes)
    assert engine.combine_verify_g2(t, idx, pts, mpk, hashes) == (out9, st9, v9)
    assert notree_engine.combine_verify_g2(t, idx, pts, mpk, hashes) == (out9, st9, v9)
    out8, st8, v8 = engine.combine_verify_g2(t, idx[:8], pts[:8], mpk, hashes[:8])
    out1, st1, v1 = engine.combine_verify_g2(t, idx[:1], pts[:1], mpk, hashes[:1])
    assert (out8, st8, v8) == (out9[:8], st9[:8], v9[:8])
    assert (out1, st1, v1) == (out9[:1], st9[:1], v9[:1])
    assert v9[0] == 1 and v9[1] == 1 and v9[2] == 0 and v9[3] == 0 and v9[4] == 0
    assert [cbls.verify_g2(mpk, s, h) for s, h in zip(out9[:5], hashes[:5])] == [bool(x) for x in v9[:5]]
    if t > 0:
        assert st9[5] == 5 and v9[5] == 0
    # master key at infinity (the split form's Z = 0 inactive pair): identical on both forms; the
    # signature then verifies only if it is the point at infinity too
    inf = bytes(96)
    assert engine.combine_verify_g2(t, idx, pts, inf, hashes) == unsplit_engine.combine_verify_g2(t, idx, pts, inf,
                                                                                                  hashes)
    # a master key coordinate >= p is an argument error on both forms
    bad = bytearray(mpk)
    bad[0:48] = (C.P + 1).to_bytes(48, "little")
    for eng in (engine, unsplit_engine):
        with pytest.raises(HbhError):
            eng.combine_verify_g2(t, idx[:1], pts[:1], bytes(bad), hashes[:1])


def test_interpolate_edge_cases(engine):
    rng = random.Random(3)
    # t = 0 returns the sample itself
    p = cbls.g2_mul(G2, 5)
    out, st = engine.interpolate_g2(0, [[7]], [[p]])
    assert st == [0] and out == [p]
    # duplicate index -> DuplicateEntry (status 5), other combines in the batch unaffected
    q = [cbls.g1_mul(G1, rng.randrange(1, C.R)) for _ in range(3)]
    out, st = engine.interpolate_g1(2, [[1, 1, 2], [0, 1, 2]], [q, q])
    assert st[0] == 5 and st[1] == 0
    rc, want = cbls.combine_g1(2, [0, 1, 2], q)
    assert out[1] == want
    # shares that are the point at infinity
    out, st = engine.interpolate_g1(1, [[0, 1]], [[bytes(96), bytes(96)]])
    assert st == [0] and out == [bytes(96)]


@pytest.mark.parametrize("t", [1, 5, 21, 70])
def test_interpolate_random_samples_match_oracle(engine, t):
    """Arbitrary subgroup points (not shares of one polynomial), ragged index sets, an infinity
    sample, and t = 70 (284 G2 / 142 G1 endomorphism terms: more terms than threads per combine)
    -- byte-identical to the C restatement of threshold_crypto interpolate()."""
    rng = random.Random(100 + t)
    m = t + 1
    idx = [sorted(rng.sample(range(200), m)) for _ in range(3)]
    p2 = [[cbls.g2_mul(G2, rng.randrange(1, C.R)) for _ in range(m)] for _ in range(3)]
    p1 = [[cbls.g1_mul(G1, rng.randrange(1, C.R)) for _ in range(m)] for _ in range(3)]
    p2[1][0], p1[2][m - 1] = bytes(192), bytes(96)
    out, st = engine.interpolate_g2(t, idx, p2)
    assert st == [0, 0, 0]
    assert out == [cbls.combine_g2(t, i, p)[1] for i, p in zip(idx, p2)]
    out, st = engine.interpolate_g1(t, idx, p1)
    assert st == [0, 0, 0]
    assert out == [cbls.combine_g1(t, i, p)[1] for i, p in zip(idx, p1)]


def test_threshold_decrypt_golden(engine):
    d = load("threshold_decrypt_n10_t3.json")
    t = d["t"]
    for ct in d["ciphertexts"]:
        by_idx = {s["idx"]: s for s in ct["shares"]}
        idx = ct["combine_indices"]
        out, st = engine.interpolate_g1(t, [idx], [[g1a(bytes.fromhex(by_idx[i]["share"])) for i in idx]])
        assert st == [0]
        g = (int.from_bytes(out[0][:48], "little"), int.from_bytes(out[0][48:], "little"))
        assert tc.xor_with_hash(g, bytes.fromhex(ct["v"])) == bytes.fromhex(ct["plaintext"])


def test_bivar_golden(engine):
    d = load("sync_key_gen_n4_t2.json")
    t = d["t"]
    commit = [g1a(bytes.fromhex(h)) for h in d["commit"]]
    rows = engine.bivar_row(t, [commit], [0] * len(d["rows"]), [r["x"] for r in d["rows"]])
    for r, got in zip(d["rows"], rows):
        assert got == [g1a(bytes.fromhex(h)) for h in r["row_commit"]]
    acks = d["acks"]
    v = engine.bivar_ack_check(t, [commit], [0] * len(acks), [a["x"] for a in acks], [a["y"] for a in acks],
                               [int(a["val"], 16) for a in acks])
    assert list(v) == [int(a["valid"]) for a in acks]


def test_bivar_t33_matches_oracle(engine):
    """SyncKeyGen N=100 t=33 shapes: 595-point commitments, rows at x = our index + 1."""
    rng = random.Random(33)
    t = 33
    npos = (t + 1) * (t + 2) // 2
    parts = []
    polys = []
    for _ in range(2):
        bp = tc.BivarPoly(t, [rng.randrange(1, C.R) for _ in range(npos)])
        polys.append(bp)
        parts.append([cbls.g1_mul(G1, c) for c in bp.coeffs])
    x = 17
    rows = engine.bivar_row(t, parts, [0, 1], [x, x])
    for bp, row in zip(polys, rows):
        assert row == [cbls.g1_mul(G1, c) for c in bp.row(x)]
    assert rows[0][:3] == cbls.bivar_row(t, parts[0], x)[:3]
    ys = [1, 2, 50, 100, 7, 9]
    pidx = [0, 1, 0, 1, 0, 1]
    vals = [polys[p].evaluate(x, y) for p, y in zip(pidx, ys)]
    vals[3] = (vals[3] + 1) % C.R  # a tampered Ack value
    v = engine.bivar_ack_check(t, parts, pidx, [x] * len(ys), ys, vals)
    assert list(v) == [1, 1, 1, 0, 1, 1]


def test_commitment_eval_public_key_shares(engine):
    """Commitment::evaluate(i + 1) = PublicKeySet::public_key_share(i) (src/network_info.rs:59-62):
    the golden fixture's key set (re-derived from its recorded seed, as gen_golden.py draws it) must
    give the fixture's public key shares; random commitments with an infinity coefficient and
    x = 0 (= C_0) match the C oracle."""
    d = load("threshold_sign_n10_t3.json")
    rng = random.Random(d["seed"])
    coeffs = [rng.randrange(1, C.R) for _ in range(d["t"] + 1)]
    commit = [cbls.g1_mul(G1, c) for c in coeffs]
    got = engine.commitment_eval(d["t"], [commit], [0] * d["n"], [i + 1 for i in range(d["n"])])
    assert got == [g1a(bytes.fromhex(p)) for p in d["pk_shares"]]
    master = engine.commitment_eval(d["t"], [commit], [0], [0])[0]
    assert master == g1a(C.g1_uncompressed(C.g1_decompress(bytes.fromhex(d["master_pk"]))))
    r2 = random.Random(33)
    t = 33
    polys = [[r2.randrange(1, C.R) for _ in range(t + 1)] for _ in range(3)]
    polys[1][5] = 0  # infinity coefficient
    commits = [[cbls.g1_mul(G1, c) for c in p] for p in polys]
    reqs = [(c, x) for c in range(3) for x in (0, 1, 2, 64, 100, 0xFFFFFFFF)]
    got = engine.commitment_eval(t, commits, [c for c, _ in reqs], [x for _, x in reqs])
    assert got == [cbls.g1_mul(G1, tc.poly_eval(polys[c], x)) for c, x in reqs]


def test_g1_decompress_matches_oracle(engine):
    """hbh_g1_decompress = pairing 0.14 G1Compressed::into_affine: valid points
    (both y signs), infinity, malformed flags, x >= p, x off the curve, and on-curve points outside
    the prime-order subgroup -- accept/reject and decoded bytes equal the oracle's."""
    rng = random.Random(48)
    encs = []
    for _ in range(24):
        encs.append(C.g1_compress(C.g1_mul(C.G1_GEN, rng.randrange(1, C.R))))
    encs.append(C.g1_compress(None))                       # infinity
    encs.append(bytes([0xC0]) + bytes(46) + b"\x01")       # bad infinity
    encs.append(bytes([0x00]) + encs[0][1:])                # not compressed
    encs.append(bytes([encs[1][0] ^ 0x20]) + encs[1][1:])   # other root: valid, negated point
    pb = (C.P + 5).to_bytes(48, "big")
    encs.append(bytes([pb[0] | 0x80]) + pb[1:])             # x >= p
    off, cof = 0, 0
    while off < 3 or cof < 3:                               # off-curve x / on-curve non-subgroup x
        x = rng.randrange(C.P)
        b = x.to_bytes(48, "big")
        e = bytes([b[0] | 0x80 | (0x20 if rng.random() < 0.5 else 0)]) + b[1:]
        try:
            C.g1_decompress(e)
            continue
        except C.DecodeError as err:
            kind = str(err)
        if "curve" in kind and off < 3:
            off += 1
            encs.append(e)
        elif "subgroup" in kind and cof < 3:
            cof += 1
            encs.append(e)
    want_pts, want_ok = [], []
    for e in encs:
        try:
            pt = C.g1_decompress(e)
            want_pts.append(bytes(96) if pt is None else g1a(C.g1_uncompressed(pt)))
            want_ok.append(1)
        except C.DecodeError:
            want_pts.append(bytes(96))
            want_ok.append(0)
    got, ok = engine.g1_decompress(encs)
    assert list(ok) == want_ok
    assert got == want_pts
    assert sum(want_ok) == 26 and len(encs) == 35


def test_g2_decompress_matches_oracle(engine):
    """hbh_g2_decompress = pairing 0.14 G2Compressed::into_affine: Fp2 square
    root, the c1-then-c0 root order, and the subgroup check, against the oracle."""
    rng = random.Random(96)
    encs = [C.g2_compress(C.g2_mul(C.G2_GEN, rng.randrange(1, C.R))) for _ in range(8)]
    encs.append(C.g2_compress(None))                                   # infinity
    encs.append(bytes([0xC0]) + bytes(94) + b"\x02")                   # bad infinity
    encs.append(bytes([encs[0][0] & 0x7F]) + encs[0][1:])               # not compressed
    encs.append(bytes([encs[1][0] ^ 0x20]) + encs[1][1:])               # other root
    pb = (C.P + 1).to_bytes(48, "big")
    encs.append(encs[2][:48] + pb)                                      # x.c0 >= p
    encs.append(bytes([pb[0] | 0x80]) + pb[1:] + encs[2][48:])           # x.c1 >= p
    off, cof = 0, 0
    while off < 2 or cof < 2:
        b = rng.randrange(C.P).to_bytes(48, "big") + rng.randrange(C.P).to_bytes(48, "big")
        e = bytes([b[0] | 0x80 | (0x20 if rng.random() < 0.5 else 0)]) + b[1:]
        try:
            C.g2_decompress(e)
            continue
        except C.DecodeError as err:
            kind = str(err)
        if "curve" in kind and off < 2:
            off += 1
            encs.append(e)
        elif "subgroup" in kind and cof < 2:
            cof += 1
            encs.append(e)
    want_pts, want_ok = [], []
    for e in encs:
        try:
            pt = C.g2_decompress(e)
            want_pts.append(bytes(192) if pt is None else g2a(C.g2_uncompressed(pt)))
            want_ok.append(1)
        except C.DecodeError:
            want_pts.append(bytes(192))
            want_ok.append(0)
    got, ok = engine.g2_decompress(encs)
    assert list(ok) == want_ok
    assert got == want_pts
    assert sum(want_ok) == 10 and len(encs) == 18


def test_subgroup_contract_wire_path(engine):
    """The ABI's subgroup contract (include/hbbft_hip.h, Conventions): points reach the engine only
    through subgroup-checked decoding, as threshold_crypto's deserialisation guarantees.  On-curve
    points outside the prime-order subgroup (G1 and G2) are rejected by hbh_g*_decompress, so they
    can never feed the GLS/GLV-split combines or the pairing checks; subgroup points decode and
    combine to the C oracle's bytes."""
    rng = random.Random(1234)
    for g2, dec, comp in ((False, engine.g1_decompress, C.g1_compress), (True, engine.g2_decompress, C.g2_compress)):
        nfe = 2 if g2 else 1
        outside = []
        while len(outside) < 3:
            b = b"".join(rng.randrange(C.P).to_bytes(48, "big") for _ in range(nfe))
            e = bytes([b[0] | 0x80]) + b[1:]
            try:
                (C.g2_decompress if g2 else C.g1_decompress)(e)
            except C.DecodeError as err:
                if "subgroup" in str(err):
                    outside.append(e)
        base = C.G2_GEN if g2 else C.G1_GEN
        inside = [comp((C.g2_mul if g2 else C.g1_mul)(base, rng.randrange(1, C.R))) for _ in range(3)]
        pts, ok = dec(outside + inside)
        assert list(ok) == [0, 0, 0, 1, 1, 1]
        assert pts[:3] == [bytes(192 if g2 else 96)] * 3
        idx = [[0, 1, 2]]
        out, st = (engine.interpolate_g2 if g2 else engine.interpolate_g1)(2, idx, [pts[3:]])
        assert st == [0]
        assert out[0] == (cbls.combine_g2 if g2 else cbls.combine_g1)(2, idx[0], pts[3:])[1]
