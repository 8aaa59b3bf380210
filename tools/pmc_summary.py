"""Summarise rocprofv3 --pmc counter CSVs per kernel (sum over dispatches / dispatch count)."""
import collections, csv, glob, sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        disp[k].add((f, r["Dispatch_Id"]))
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(acc.items()):
    n = len(disp[k])
    print(k, "dispatches", n)
    for name, v in sorted(c.items()):
        print("   %-22s %.4g per dispatch" % (name, v / n))
