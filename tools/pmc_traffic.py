"""HBM traffic of one pairing stage (HBH_IMPL_THREAD_SIGNED, one 65,536-check step) from rocprofv3
--pmc FETCH_SIZE / WRITE_SIZE passes (separate runs), with the gfx950 correction of
MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of wide coalesced reads: doubled).
usage: python tools/pmc_traffic.py gpurun_out/<tag>/pmc profiles/r01/pmc_traffic.json"""
import collections
import csv
import glob
import json
import sys

STAGE = {"hbs::k_ts_miller": 1, "hbs::k_ts_easy": 1, "hbs::k_ts_exp": 5, "hbs::k_ts_glue": 2, "hbs::k_ts_verdict": 1}
CHECKS = 65536
# algorithmic bytes per check: P1 (96) + P2 (96) + verdict (1) + the per-check G2 line table read (68 lines x 84 words
# x 4 B = 22,848 B; the shared per-document H table is read once per 64 checks: 357 B/check)
ALGO_PER_CHECK = 96 + 96 + 1 + 22848 + 22848 // 64


def per_dispatch(root, counter):
    tot, n = collections.defaultdict(float), collections.defaultdict(set)
    for f in glob.glob(f"{root}/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            tot[k] += float(r["Counter_Value"])
            n[k].add((f, r["Dispatch_Id"]))
    return {k: tot[k] / len(n[k]) for k in tot}


def main():
    root, out = sys.argv[1], sys.argv[2]
    fetch = per_dispatch(root, "FETCH_SIZE")   # KB
    write = per_dispatch(root, "WRITE_SIZE")   # KB
    f_raw = sum(fetch.get(k, 0.0) * c for k, c in STAGE.items()) * 1024
    w = sum(write.get(k, 0.0) * c for k, c in STAGE.items()) * 1024
    res = {
        "kernel": "hbs::k_ts_* (one pairing stage: miller + easy + 5 exp + 2 glue + verdict)",
        "checks_per_launch": CHECKS,
        "FETCH_SIZE_bytes_raw": f_raw,
        "FETCH_SIZE_bytes_gfx950_x2": 2 * f_raw,
        "WRITE_SIZE_bytes": w,
        "hbm_bytes_per_launch": 2 * f_raw + w,
        "algorithmic_bytes_per_launch": ALGO_PER_CHECK * CHECKS,
        "prepare": {"kernel": "hb::k_g2_prepare", "FETCH_SIZE_bytes_gfx950_x2": 2 * fetch.get("hb::k_g2_prepare", 0) * 1024,
                    "WRITE_SIZE_bytes": write.get("hb::k_g2_prepare", 0) * 1024},
        "per_kernel_KB": {k: {"FETCH_SIZE": fetch.get(k), "WRITE_SIZE": write.get(k)} for k in STAGE},
        "source": root,
        "note": "Fp12 state crosses HBM between the stage kernels (6 x 14 x 4 x 2 B per check per hand-over) and the "
                "256V+256A-register kernels spill to scratch; traffic / algorithmic shows both",
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
