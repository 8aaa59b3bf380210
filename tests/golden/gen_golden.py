"""Generate the committed golden fixtures from the CPU restatement in ``oracle/``.

Run from the repo root:  python -m tests.golden.gen_golden
The fixtures are DATA (inputs + expected outputs).  Seeds are recorded in each file.
The reference's own threshold_crypto cannot run here, so these vectors pin
GPU <-> oracle parity; oracle <-> threshold_crypto parity is pinned only where noted in
DESIGN.md (encodings of the generators, SHA3, ChaCha20).
"""
import json
import os
import random

from oracle import bls12_381 as C
from oracle import tc

HERE = os.path.dirname(os.path.abspath(__file__))


def h(b):
    return bytes(b).hex()


def rand_fr(rng):
    return rng.randrange(1, C.R)


def gen_sign(seed=20261015, n=10, t=3, ndocs=2):
    rng = random.Random(seed)
    ks = tc.KeySet([rand_fr(rng) for _ in range(t + 1)])
    pks = [ks.pk_share(i) for i in range(n)]
    docs = []
    for d in range(ndocs):
        # coin-id layout of SURVEY §8a row a4: bincode((BaSessionId, epoch)) = 28 bytes
        doc = bytes(rng.randrange(256) for _ in range(28))
        hm = tc.hash_g2(doc)
        shares = []
        for i in range(n):
            sig = C.g2_mul(hm, ks.sk_share(i))
            kind = "valid"
            if i == 2 + d:       # a random G2 point (wrong share)
                sig = C.g2_mul(C.G2_GEN, rand_fr(rng))
                kind = "random_g2"
            elif i == 5 + d:     # the share of another document
                sig = C.g2_mul(tc.hash_g2(doc + b"x"), ks.sk_share(i))
                kind = "other_doc"
            elif i == 7 and d == 1:  # the point at infinity
                sig = None
                kind = "infinity"
            ok = tc.verify_g2(pks[i], sig, hm)
            shares.append({"idx": i, "sig": h(C.g2_uncompressed(sig)), "kind": kind, "valid": ok})
        valid = [(s["idx"], C.g2_mul(hm, ks.sk_share(s["idx"]))) for s in shares if s["valid"]]
        combined = tc.combine_signatures(t, valid)
        assert combined == C.g2_mul(hm, ks.coeffs[0])
        assert tc.verify_g2(ks.master_pk(), combined, hm)
        docs.append({
            "doc": h(doc),
            "hash": h(C.g2_uncompressed(hm)),
            "hash_compressed": h(C.g2_compress(hm)),
            "shares": shares,
            "combine_indices": [i for (i, _) in valid[: t + 1]],
            "combined": h(C.g2_compress(combined)),
            "combined_uncompressed": h(C.g2_uncompressed(combined)),
            "parity": tc.signature_parity(combined),
        })
    # edge case: pk = O and sig = O verifies (pairing with O is 1)
    edge = {
        "pk_inf_sig_inf": tc.verify_g2(None, None, docs[0] and tc.hash_g2(b"edge")),
    }
    return {
        "seed": seed, "n": n, "t": t,
        "master_pk": h(C.g1_compress(ks.master_pk())),
        "pk_shares": [h(C.g1_uncompressed(p)) for p in pks],
        "pk_shares_compressed": [h(C.g1_compress(p)) for p in pks],
        "docs": docs,
        "edge": edge,
    }


def gen_decrypt(seed=77, n=10, t=3):
    rng = random.Random(seed)
    ks = tc.KeySet([rand_fr(rng) for _ in range(t + 1)])
    pks = [ks.pk_share(i) for i in range(n)]
    cts = []
    for c, mlen in enumerate([32, 100]):
        msg = bytes(rng.randrange(256) for _ in range(mlen))
        ct = tc.encrypt(ks.master_pk(), msg, rand_fr(rng))
        u, v, w = ct
        huv = tc.hash_g1_g2(u, v)
        assert tc.ciphertext_verify(ct)
        shares = []
        for i in range(n):
            d = tc.decrypt_share(ks.sk_share(i), ct)
            kind = "valid"
            if i == 1 + c:
                d = C.g1_mul(C.G1_GEN, rand_fr(rng))
                kind = "random_g1"
            elif i == 4:
                d = C.g1_mul(u, ks.sk_share(i) + 1)
                kind = "off_by_one"
            ok = tc.verify_decryption_share(pks[i], d, ct, huv)
            shares.append({"idx": i, "share": h(C.g1_uncompressed(d)), "kind": kind, "valid": ok})
        valid = [(s["idx"], tc.decrypt_share(ks.sk_share(s["idx"]), ct)) for s in shares if s["valid"]]
        pt = tc.combine_decryption(t, valid, ct)
        assert pt == msg
        # tampered ciphertext: W replaced by another point -> Ciphertext::verify false
        bad_w = C.g2_mul(C.G2_GEN, rand_fr(rng))
        cts.append({
            "msg": h(msg),
            "u": h(C.g1_uncompressed(u)), "v": h(v), "w": h(C.g2_uncompressed(w)),
            "huv": h(C.g2_uncompressed(huv)),
            "ct_valid": True,
            "bad_w": h(C.g2_uncompressed(bad_w)),
            "bad_w_valid": tc.ciphertext_verify((u, v, bad_w)),
            "shares": shares,
            "combine_indices": [i for (i, _) in valid[: t + 1]],
            "plaintext": h(pt),
        })
    return {"seed": seed, "n": n, "t": t,
            "pk_shares": [h(C.g1_uncompressed(p)) for p in pks], "ciphertexts": cts}


def gen_dkg(seed=4242, n=4, t=2):
    rng = random.Random(seed)
    npos = (t + 1) * (t + 2) // 2
    bp = tc.BivarPoly(t, [rand_fr(rng) for _ in range(npos)])
    commit = bp.commitment()
    acks = []
    for x in range(1, n + 1):
        for y in range(1, n + 1):
            val = bp.evaluate(x, y)
            tampered = (x == 2 and y == 3)
            if tampered:
                val = (val + 1) % C.R
            ok = tc.bivar_commit_evaluate(t, commit, x, y) == C.g1_mul(C.G1_GEN, val)
            acks.append({"x": x, "y": y, "val": "%064x" % val, "valid": ok})
    rows = []
    for x in range(0, n + 1):
        crow = tc.bivar_commit_row(t, commit, x)
        prow = bp.row(x)
        assert crow == tc.poly_commitment(prow)
        rows.append({"x": x, "row_poly": ["%064x" % c for c in prow],
                     "row_commit": [h(C.g1_uncompressed(p)) for p in crow]})
    return {"seed": seed, "n": n, "t": t,
            "commit": [h(C.g1_uncompressed(p)) for p in commit], "acks": acks, "rows": rows}


def main():
    out = {
        "threshold_sign_n10_t3.json": gen_sign(),
        "threshold_decrypt_n10_t3.json": gen_decrypt(),
        "sync_key_gen_n4_t2.json": gen_dkg(),
    }
    for name, data in out.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
        print("wrote", name)


if __name__ == "__main__":
    main()
