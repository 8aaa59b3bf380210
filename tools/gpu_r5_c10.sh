#!/bin/bash
# round 5 call 10: epoch line spread (after the fast paths moved into the classes) with a host profile
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c10}
mkdir -p $O
cd $R
for k in 1 2 3; do
  timeout -k 10 400 python3 -u bench.py --workload epoch --no-cpu-baseline > $O/epoch_$k.json 2> $O/epoch_$k.err || { tail -5 $O/epoch_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/epoch_$k.json')); print('epoch', round(d['value'],2), 'ms/step', round(d['ms_per_step'],2), json.dumps(d.get('host_vs_gpu')))"
done
timeout -k 10 400 python3 -u bench.py --workload epoch --no-cpu-baseline --profile-epoch $O/epoch_prof.txt > $O/epoch_p.json 2> $O/epoch_p.err || { tail -5 $O/epoch_p.err; exit 1; }
head -40 $O/epoch_prof.txt
