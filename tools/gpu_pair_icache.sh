#!/bin/bash
# instruction-cache behaviour of the sign kernel: one SQC pass (hits / misses)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof/icache
mkdir -p $O
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-combine --streams 1"
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $O/sqc -o run -- python3 $B > $O/sqc.log 2>&1 || { echo "sqc failed"; tail -5 $O/sqc.log; exit 1; }
python3 - <<'PY'
import csv, collections, glob, os
f = glob.glob(os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out/prof/icache/sqc/*counter_collection.csv"))[0]
agg = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    agg[(r["Kernel_Name"][:40], r["Counter_Name"])] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print(k, v)
PY
