#!/bin/bash
# round 5 call 6: FD seed levels (difference table straight from the row) -- FD parity tests, dkg line and kernel stats
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c6}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_commit_set.py -x -v --timeout 300 --timeout-method thread -k "ack or fd" > $O/pytest.log 2>&1
rc=$?; tail -8 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for A in auto auto; do
  timeout -k 10 300 python3 -u bench.py --workload dkg --ack-impl $A --no-cpu-baseline --no-node-round > $O/dkg_$A.json 2> $O/dkg_$A.err || { tail -5 $O/dkg_$A.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/dkg_$A.json')); r=d['roofline']; print('$A', round(d['value']/1e6,3), 'M acks/s', round(d['ms_per_step'],3), 'ms', 'frac', round(r['frac'],4), d['verdicts_ok'])"
done
cd /tmp
mkdir -p $O/trace
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --workload dkg --steps 4 --no-cpu-baseline --no-node-round > $O/trace/run.log 2>&1 || { echo "trace failed"; tail -5 $O/trace/run.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec head -8 {} \;
