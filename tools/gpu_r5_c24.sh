#!/bin/bash
# round 5 call 24: speculative decryption combines A/B on one box (HBH_EPOCH_SPEC_G1), interleaved
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c24}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_honey_badger.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for k in a b c; do
  for S in 1 0; do
    HBH_EPOCH_SPEC_G1=$S timeout -k 10 400 python3 -u bench.py --workload epoch --no-cpu-baseline > $O/e$S$k.json 2> $O/e$S$k.err || { tail -5 $O/e$S$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e$S$k.json')); p=d['phase_ms']; h=d['host_vs_gpu']; print('specg1=$S', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'host', round(h['host_ms'],1), 'blocked', round(h['blocked_on_engine_ms'],1), 'coin', round(p['coin_verify'],1), 'combine', round(p['combine'],2), 'dverify', round(p['decrypt_verify'],1), 'ok', d['outputs_ok'])"
  done
done
