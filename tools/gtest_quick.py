import sys, time, json
sys.path.insert(0, '/root/repo')
from oracle import bls12_381 as C, tc
from hbbft_amd.engine import Engine, g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a
eng = Engine(0)
g1, g2 = C.G1_GEN, C.G2_GEN
P = [C.g1_mul(g1, k) for k in (1, 5, 12345)]
Q = [C.g2_mul(g2, k) for k in (1, 7, 999)]
t = time.time()
out = eng.dbg_pairing([g1a(C.g1_uncompressed(p)) for p in P], [g2a(C.g2_uncompressed(q)) for q in Q])
print("dbg_pairing", time.time() - t)
for k, (p, q) in enumerate(zip(P, Q)):
    e = C.f12_pow(C.pairing(p, q), 3)
    want = b"".join(c.to_bytes(48, 'little') for six in e for f2 in six for c in f2)
    print("pairing", k, "MATCH" if out[k] == want else "MISMATCH")
    if out[k] != want:
        print(out[k][:48].hex(), want[:48].hex())
d = json.load(open('/root/repo/tests/golden/threshold_sign_n10_t3.json'))
pks, sigs, hashes, didx, exp = [], [], [], [], []
for di, doc in enumerate(d['docs']):
    hashes.append(g2a(bytes.fromhex(doc['hash'])))
    for s in doc['shares']:
        pks.append(g1a(bytes.fromhex(d['pk_shares'][s['idx']]))); sigs.append(g2a(bytes.fromhex(s['sig']))); didx.append(di); exp.append(int(s['valid']))
t = time.time()
v = eng.verify_sig_shares(pks, sigs, hashes, didx)
print("sig shares", time.time() - t, list(v) == exp, list(v), exp)
