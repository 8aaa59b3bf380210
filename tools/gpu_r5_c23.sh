#!/bin/bash
# round 5 call 23: speculative coin combines on a third engine -- HB / BA GPU tests, epoch A/B
# (HBH_EPOCH_SPEC=0 turns them off), interleaved
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c23}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_honey_badger.py tests/test_gpu_binary_agreement.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for k in a b c; do
  for S in 1 0; do
    HBH_EPOCH_SPEC=$S timeout -k 10 400 python3 -u bench.py --workload epoch --no-cpu-baseline > $O/e$S$k.json 2> $O/e$S$k.err || { tail -5 $O/e$S$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e$S$k.json')); p=d['phase_ms']; h=d['host_vs_gpu']; print('spec=$S', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'host', round(h['host_ms'],1), 'blocked', round(h['blocked_on_engine_ms'],1), 'resolve', round(p['coin_resolve'],2), 'local', round(p['coin_local'],2), 'coin', round(p['coin_verify'],1), 'ok', d['outputs_ok'])"
  done
done
