#!/bin/bash
# round 4 closing bench refresh after host-side (Python) changes: the library is unchanged since the
# last tools/gpu_r4_final.sh call (same sha256 as profiles/r04/pmc_traffic.json), so this reruns the
# GPU suite, smoke and the four bench lines only.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-final_bench}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1
rc=$?; tail -3 $O/pytest_gpu_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for W in sign decrypt dkg epoch; do
  timeout -k 10 600 python3 -u bench.py --workload $W > $O/bench_$W.json 2> $O/bench_$W.err || { tail -5 $O/bench_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$W.json')); r=d.get('roofline',{}); print('$W', d['value'], d['unit'], 'ms/step', round(d['ms_per_step'],3), 'frac', round(r.get('frac',0),4), r.get('traffic_source'))"
done
echo done
