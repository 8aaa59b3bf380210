#!/bin/bash
# round 5 call 13: epoch loop skip filter -- honey badger GPU tests, epoch line vs the round-4 tree on one box
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c13}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_honey_badger.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag dir
  local tag=$1 dir=$2
  ( cd $dir && timeout -k 10 400 python3 -u bench.py --workload epoch --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err ) || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); p=d.get('phase_ms',{}); h=d.get('host_vs_gpu',{}); print('$tag', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'host', round(h.get('host_ms',0),1), 'blocked', round(h.get('blocked_on_engine_ms',0),1), 'resolve', round(p.get('coin_resolve',0),1), 'local', round(p.get('coin_local',0),1), 'msgs', round(p.get('coin_messages',0),1), 'dverify', round(p.get('decrypt_verify',0),1))"
}
run now1 $R
run r4_1 $R/ab_r4wt
run now2 $R
run r4_2 $R/ab_r4wt
run now3 $R
