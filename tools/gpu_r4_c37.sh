#!/bin/bash
# round 4, call 37: spread of the epoch and decrypt lines on the final library (one box)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c37
mkdir -p $O
cd $R
for r in 1 2 3; do
  for W in epoch decrypt; do
    timeout -k 10 300 python3 -u bench.py --workload $W --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b.json')); print('$W %.3f %s ms %.2f' % (d['value'], d['unit'], d['ms_per_step']))" | tee -a $O/spread.txt
  done
done
echo done
