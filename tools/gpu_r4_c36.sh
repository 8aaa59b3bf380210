#!/bin/bash
# round 4, call 36: sign line vs number of alternating streams, with the lane-octo line tables
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c36
mkdir -p $O
cd $R
for r in 1 2; do
  for S in 1 2 3 4; do
    timeout -k 10 300 python3 -u bench.py --workload sign --streams $S --no-cpu-baseline > $O/s.json 2> $O/s.err || { tail -5 $O/s.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s.json')); print('streams $S sign %.3f M/s ms %.3f' % (d['value']/1e6, d['ms_per_step']), d['verdicts_ok'])" | tee -a $O/streams.txt
  done
done
echo done
