#!/bin/bash
# round 5 call 22: speculative decryption combines beside the coin phase -- HB GPU tests, epoch line
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c22}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_honey_badger.py tests/test_gpu_protocol.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  timeout -k 10 400 python3 -u bench.py --workload epoch --no-cpu-baseline > $O/e$k.json 2> $O/e$k.err || { tail -5 $O/e$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e$k.json')); p=d['phase_ms']; h=d['host_vs_gpu']; print('epoch', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'host', round(h['host_ms'],1), 'blocked', round(h['blocked_on_engine_ms'],1), 'combine', round(p['combine'],2), 'dverify', round(p['decrypt_verify'],1), 'pre_eng', round(p['decrypt_pre_engine'],1), 'pre_wait', round(p['decrypt_pre_wait'],2), 'ok', d.get('plaintexts_ok', d.get('verdicts_ok')))"
done
