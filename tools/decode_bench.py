"""Device point decoding (k_g1_decompress / k_g2_decompress) on n compressed subgroup points:
kernel time from the engine's HIP events (median of reps) and the host-to-host call; decoded
points must equal the generated ones.  python3 tools/decode_bench.py [n] [reps]"""
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from hbbft_amd._lib import STAGE_CURVE  # noqa: E402
from hbbft_amd.engine import Engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    eng = Engine(0)
    rng = random.Random(5)
    from hbbft_amd.engine import g1_abi_from_uncompressed as g1a, g2_abi_from_uncompressed as g2a
    g1, g2 = g1a(bench.G1_UNC), g2a(bench.G2_UNC)
    m = min(n, 4096)
    p1 = eng.g1_mul([g1] * m, [rng.randrange(1, bench.R_ORDER) for _ in range(m)])
    p2 = eng.g2_mul([g2] * m, [rng.randrange(1, bench.R_ORDER) for _ in range(m)])
    e1 = [bench.g1_compress_abi(p) for p in p1]
    e2 = [bench.g2_compress_abi(p) for p in p2]
    out = {"n": n}
    for name, encs, pts, dec in (("g1", e1, p1, eng.g1_decompress), ("g2", e2, p2, eng.g2_decompress)):
        blob = b"".join(encs[i % m] for i in range(n))
        want = b"".join(pts[i % m] for i in range(n))
        dec(blob[:len(encs[0]) * 64])
        devs, hosts = [], []
        for _ in range(reps):
            eng.set_profiling(True)
            t0 = time.perf_counter()
            got, ok = dec(blob)
            hosts.append((time.perf_counter() - t0) * 1e3)
            devs.append(eng.stage_time(STAGE_CURVE)[0])
            eng.set_profiling(False)
            assert all(ok) and b"".join(got) == want, name + " decode mismatch"
        out[name + "_kernel_ms"] = statistics.median(devs)
        out[name + "_host_ms"] = statistics.median(hosts)
        out[name + "_per_s_device"] = n / (statistics.median(devs) / 1e3)
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
