"""k_pair_verify launch size A/B (second half): the sign workload's 65,536 checks
as one launch (2,048 waves: two lane-pair waves per SIMD, the last waves' tail idles SIMDs) against
131,072 / 196,608 checks in ONE launch (4,096 / 6,144 waves: the resident waves' exits backfill from
the queue without a second stream).  HBH_IMPL_PAIR forced; kernel time from the engine's HIP events
per launch; verdicts checked.  usage: pair_launch_sizes.py [reps]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from hbbft_amd._lib import IMPL_PAIR, STAGE_PAIRING, STAGE_PREPARE  # noqa: E402
from hbbft_amd.engine import Engine  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    eng.set_pairing_impl(IMPL_PAIR)
    n0 = 65536
    w = bench.Workload(eng, n0, seed=20261016)
    out = {"checks_per_round": n0, "runs": []}
    for k in (1, 2, 3):
        n = n0 * k

        def to_dev(b):
            return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).to(dev)
        d_pk, d_sg = to_dev(w.pk_batch * k), to_dev(w.sig_batch * k)
        d_hs = to_dev(w.hash_table)
        d_di = torch.from_numpy(np.tile(w.doc_idx, k)).to(dev)
        d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
        nh = len(w.hashes)

        def step():
            eng.verify_pairing_eq_dev(None, n, d_pk.data_ptr(), d_hs.data_ptr(), nh, d_di.data_ptr(), None,
                                      d_sg.data_ptr(), n, None, d_v.data_ptr())
        step()
        torch.cuda.synchronize(dev)
        ok = bool((d_v.cpu().numpy() == np.tile(w.expected, k)).all())
        eng.set_profiling(True)
        for _ in range(reps):
            step()
        torch.cuda.synchronize(dev)
        pm, pn = eng.stage_time(STAGE_PAIRING)
        qm, qn = eng.stage_time(STAGE_PREPARE)
        eng.set_profiling(False)
        ms = pm / max(pn, 1)
        out["runs"].append({"checks": n, "waves": n * 2 // 64, "verify_ms": ms, "ms_per_65536": ms / k,
                            "prep_ms": qm / max(qn, 1), "verdicts_ok": ok})
        print(json.dumps(out["runs"][-1]), flush=True)
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
