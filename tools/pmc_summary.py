"""Summarise rocprofv3 --pmc counter CSVs per kernel: each counter's sum divided by the dispatches
of the pass(es) that collected it.  A profile directory holds one sub-directory per --pmc pass
(rocprofv3 collects a counter group per run), so a kernel's dispatch count differs per counter;
dividing every counter by the dispatches of all passes (rounds 2-5) understated each counter by
the number of passes (What's weak 7).  usage: pmc_summary.py DIR"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)   # (kernel, counter) -> {(file, dispatch)}
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        disp[(k, r["Counter_Name"])].add((f, r["Dispatch_Id"]))
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(acc.items()):
    ns = sorted({len(disp[(k, name)]) for name in c})
    print(k, "dispatches per pass", "/".join(str(n) for n in ns))
    for name, v in sorted(c.items()):
        print("   %-22s %.4g per dispatch" % (name, v / len(disp[(k, name)])))
