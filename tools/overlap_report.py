"""From a rocprofv3 --kernel-trace CSV of the two-stream sign bench: for every k_pair_prep launch,
how much of it ran while another stream's pairing kernel was still running (overlap), and the
serial time it added.  usage: overlap_report.py <kernel_trace.csv dir or file>"""
import csv
import glob
import os
import sys

p = sys.argv[1]
files = [p] if os.path.isfile(p) else glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True)
rows = []
for f in files:
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0], r.get("Queue_Id")))
rows.sort()
pair = [(s, e, q) for s, e, n, q in rows if "k_pair_verify" in n]
prep = [(s, e, q) for s, e, n, q in rows if ("k_pair_prep" in n or "k_oct_prep" in n)]
tot = hidden = 0
for s, e, q in prep:
    d = e - s
    cover = 0
    for ps, pe, pq in pair:
        if pq == q:
            continue
        lo, hi = max(s, ps), min(e, pe)
        if hi > lo:
            cover += hi - lo
    cover = min(cover, d)
    tot += d
    hidden += cover
    print("prep %.3f ms, %.3f ms under another stream's pairing kernel" % (d / 1e6, cover / 1e6))
if prep:
    print("total prep %.3f ms, hidden %.3f ms (%.0f %%)" % (tot / 1e6, hidden / 1e6, 100 * hidden / max(tot, 1)))
