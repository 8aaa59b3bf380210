#!/bin/bash
# round 5 call 1: GPU suite + smoke on the round-5 host stage, the dkg line with the one-node
# SyncKeyGen round (node_round), the sign line, and the host-stage per-item costs on the box's CPU.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c1}
mkdir -p $O
cd $R
nproc > $O/nproc.txt; grep -m1 "model name" /proc/cpuinfo >> $O/nproc.txt
timeout -k 10 120 python3 -u tools/host_costs.py > $O/host_costs.txt 2>&1 || { tail -5 $O/host_costs.txt; exit 1; }
cat $O/host_costs.txt
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu_all.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
fi
for W in ${WORKLOADS:-dkg sign}; do
  timeout -k 10 600 python3 -u bench.py --workload $W > $O/bench_$W.json 2> $O/bench_$W.err || { tail -5 $O/bench_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$W.json')); r=d.get('roofline',{}); print('$W', d['value'], d['unit'], 'ms/step', round(d['ms_per_step'],3), 'frac', round(r.get('frac',0),4)); print(json.dumps(d.get('node_round')))"
done
