"""Host-stage per-item costs on this machine's CPU (one thread and the process's CPU share): hash_g2,
hash_g1_g2, encrypt_with_rng, G1 / G2 secret-scalar multiplication, Fr Horner.  Prints one JSON line."""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hbbft_amd import hoststage  # noqa: E402
from hbbft_amd.sync_key_gen import G1_GEN, R_ORDER  # noqa: E402


def per_item(fn, n):
    t0 = time.perf_counter()
    fn()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    rng = random.Random(1)
    n = 256
    pks = hoststage.g1_mul([G1_GEN] * 8, [rng.randrange(1, R_ORDER) for _ in range(8)])
    msgs = [bytes(32)] * n
    nonces = [rng.randrange(1, R_ORDER) for _ in range(n)]
    full = hoststage.host_threads()
    out = {"host_threads": full, "items": n}
    for th in (1, full):
        cts = []
        r = {"encrypt_ms": per_item(lambda: cts.extend(hoststage.encrypt([pks[0]], msgs, nonces, th)), n)}
        us, vs = [c[0] for c in cts], [c[1] for c in cts]
        hs = []
        r["hash_g1_g2_ms"] = per_item(lambda: hs.extend(hoststage.hash_g1_g2(us, vs, th)), n)
        r["hash_g2_ms"] = per_item(lambda: hoststage.hash_g2([b"doc%d" % i for i in range(n)], th), n)
        r["g1_mul_ms"] = per_item(lambda: hoststage.g1_mul(us, nonces, th), n)
        r["g2_mul_ms"] = per_item(lambda: hoststage.g2_mul(hs, nonces, th), n)
        polys = [[rng.randrange(R_ORDER) for _ in range(34)] for _ in range(n)]
        r["fr_poly_eval_100pts_ms"] = per_item(lambda: hoststage.fr_poly_eval(polys, list(range(1, 101)), th), n)
        out["threads_%d" % th] = {k: round(v, 4) for k, v in r.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
