"""Latency anatomy of combine_and_verify_sig (bench.py's combine_latency_ms): repeated single-combine
hbh_combine_verify_g2 calls on a small seeded workload, for a rocprofv3 --kernel-trace of the split
check (k_g1_gen_quad, k_wave Miller-only and product / final-exponentiation waves on the side stream,
k_interp_pair + k_interp_join on the engine stream).  With --trace DIR after the run it prints, per
call, each kernel's start / end relative to the call's first kernel, and the host-to-host times."""
import argparse
import csv
import glob
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(reps):
    import bench
    from hbbft_amd.engine import Engine
    eng = Engine(0)
    w = bench.Workload(eng, 64 * 16, seed=7)
    idx = [k for k in range(bench.N_NODES) if w.expected[k]][: bench.T + 1]
    pts = [w.sigs[k] for k in idx]
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out, st, v = eng.combine_verify_g2(bench.T, [idx], [pts], w.master_pk, [w.hashes[0]])
        times.append((time.perf_counter() - t0) * 1e3)
        assert st == [0] and v == b"\x01"
    print("host-to-host ms:", [round(t, 3) for t in times], "median", round(statistics.median(times), 3))


def anatomy(d, last=3):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    # calls = groups separated by > 200 us of idle
    calls, cur, end = [], [], 0
    for s, e, n in rows:
        if cur and s - end > 200_000:
            calls.append(cur)
            cur = []
        cur.append((s, e, n))
        end = max(end, e)
    if cur:
        calls.append(cur)
    for c in calls[-last:]:
        t0 = c[0][0]
        span = (max(e for _, e, _ in c) - t0) / 1e3
        print("call span %.1f us" % span)
        for s, e, n in c:
            print("  %8.1f %8.1f  %7.1f us  %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, n[-60:]))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--trace", default=None)
    a = ap.parse_args()
    if a.trace:
        anatomy(a.trace)
    else:
        run(a.reps)
