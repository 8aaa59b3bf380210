"""Per-kernel average of every rocprofv3 counter and the kernel-trace average duration under one
profile directory (as written by tools/gpu_r4_ab.sh PROF=1).  usage: pmc_summary4.py DIR [filter]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = {}
for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Name"].split("(")[0]] = (int(r["Calls"]), float(r["AverageNs"]) / 1e6)
for k in sorted(set(agg) | set(dur)):
    if filt not in k:
        continue
    c = {n: sum(v) / len(v) for n, v in agg.get(k, {}).items()}
    line = "%-50s" % k[-50:]
    if k in dur:
        line += " calls %d avg %.3f ms" % dur[k]
    if c.get("SQ_WAVE_CYCLES"):
        line += " | VALU/wave %.3fM wait_inst %.1f%% wait_any %.1f%%" % (
            c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_WAVES", 1), 1) / 1e6,
            100 * c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"], 100 * c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"])
    if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
        line += " | HBM %.2f GB" % ((2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024 / 1e9)
    if c.get("SQC_ICACHE_REQ"):
        line += " | icache hit %.1f%% (%.2fG req)" % (100 * c.get("SQC_ICACHE_HITS", 0) / c["SQC_ICACHE_REQ"],
                                                    c["SQC_ICACHE_REQ"] / 1e9)
    if "SQ_INSTS_VMEM_RD" in c:
        line += " | vmem rd %.0f wr %.0f /wave" % (c["SQ_INSTS_VMEM_RD"] / max(c.get("SQ_WAVES", 1), 1),
                                                  c.get("SQ_INSTS_VMEM_WR", 0) / max(c.get("SQ_WAVES", 1), 1))
    print(line)
