"""Per-kernel HBM traffic from rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) plus the kernel-trace
average duration, as profiles/<round>/pmc_traffic.json (read by bench.py's roofline "traffic").
FETCH_SIZE is doubled (gfx950: it tallies 128-B requests at 64 B, MI355X_MICROARCH.md HBM
section); both counters are in KiB per dispatch.
usage: pmc_traffic.py OUT.json DIR [DIR ...]   (each DIR holds fetch/ write/ trace/ of one bench)
The library the passes ran (HBBFT_HIP_LIB or the in-tree libhbbft_hip.so) is recorded by sha256
with the git commit of the tree, so bench.py can tell whether the traffic it reports was measured on
the kernels it is running (roofline.traffic.matches_loaded_lib)."""
import collections
import csv
import glob
import json
import os
import hashlib
import subprocess
import sys


def norm(name):
    n = name.split("(")[0]
    return n[5:] if n.startswith("void ") else n


def counters(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = norm(r["Kernel_Name"])
            disp[k].add(r["Dispatch_Id"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in acc.items()}


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("HBBFT_HIP_LIB") or os.path.join(ROOT, "hbbft_amd", "libhbbft_hip.so")
try:
    commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                            text=True).stdout.strip() or None
except OSError:
    commit = None
out = {"kernels": {}, "note": "bytes per launch; FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE; KiB counters x1024",
       "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest() if os.path.exists(LIB) else None,
       "git_commit": commit}
for d in sys.argv[2:]:
    fetch, write = counters(os.path.join(d, "fetch")), counters(os.path.join(d, "write"))
    sq = counters(os.path.join(d, "sq"))
    dur = {}
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[norm(r["Name"])] = float(r["AverageNs"])
    for k in fetch:
        fb = fetch[k].get("FETCH_SIZE", 0.0) * 1024 * 2
        wb = write.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        e = {"fetch_bytes_x2": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb,
             "avg_ns": dur.get(k), "source": os.path.basename(os.path.normpath(d)).replace("pmc_", "", 1)}
        if k in sq:
            e["sq"] = sq[k]
            w = sq[k].get("SQ_WAVE_CYCLES")
            if w:
                e["sq_wait_any_frac"] = sq[k].get("SQ_WAIT_ANY", 0.0) / w
        out["kernels"][k] = e
        out.setdefault("by_source", {}).setdefault(e["source"], {})[k] = e
json.dump(out, open(sys.argv[1], "w"), indent=1)
print(json.dumps({k: {"hbm_MB": round(v["hbm_bytes_per_launch"] / 1e6, 2), "avg_ms": (v["avg_ns"] or 0) / 1e6,
                      "wait": round(v.get("sq_wait_any_frac", -1), 3)} for k, v in out["kernels"].items()}, indent=1))
