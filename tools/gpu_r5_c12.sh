#!/bin/bash
# round 5 call 12: engine-call probe A/B (round-4 tree vs this tree, and this tree with HBH_SPLIT_TREE=0),
# then the epoch line with HBH_SPLIT_TREE=0
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c12}
mkdir -p $O
( cd $R && timeout -k 10 300 python3 -u tools/probe_calls.py ) 2>&1 | tail -2
( cd $R/ab_r4wt && timeout -k 10 300 python3 -u $R/tools/probe_calls.py ) 2>&1 | tail -2
( cd $R && HBH_SPLIT_TREE=0 timeout -k 10 300 python3 -u tools/probe_calls.py ) 2>&1 | tail -2
( cd $R && timeout -k 10 300 python3 -u tools/probe_calls.py ) 2>&1 | tail -2
( cd $R/ab_r4wt && timeout -k 10 300 python3 -u $R/tools/probe_calls.py ) 2>&1 | tail -2
cd $R
HBH_SPLIT_TREE=0 timeout -k 10 400 python3 -u bench.py --workload epoch --no-cpu-baseline > $O/epoch_notree.json 2> $O/epoch_notree.err || { tail -5 $O/epoch_notree.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/epoch_notree.json')); p=d['phase_ms']; print('notree', round(d['value'],2), {k: round(v,2) for k,v in p.items()})"
