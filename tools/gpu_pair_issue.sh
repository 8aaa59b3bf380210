#!/bin/bash
# issue-stall breakdown of the sign kernel: one SQ pass (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof/issue
mkdir -p $O
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-combine --streams 1"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH --output-format csv -d $O/sq -o run -- python3 $B > $O/sq.log 2>&1 || { echo "sq failed"; tail -5 $O/sq.log; exit 1; }
python3 - <<'PY'
import csv, collections, glob, os
f = glob.glob(os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out/prof/issue/sq/*counter_collection.csv"))[0]
agg = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    if "k_pair_verify" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print(k, v, v / max(agg.get("SQ_WAVE_CYCLES", 1), 1))
PY
