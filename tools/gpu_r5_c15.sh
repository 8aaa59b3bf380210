#!/bin/bash
# round 5 call 15: epoch schedule variants (pre-verification start, prefetch start)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c15}
mkdir -p $O
cd $R
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 400 python3 -u bench.py --workload epoch --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); p=d.get('phase_ms',{}); h=d.get('host_vs_gpu',{}); print('%-14s' % '$tag', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'host', round(h.get('host_ms',0),1), 'blocked', round(h.get('blocked_on_engine_ms',0),1), 'resolve', round(p.get('coin_resolve',0),1), 'local', round(p.get('coin_local',0),1), 'msgs', round(p.get('coin_messages',0),1), 'dverify', round(p.get('decrypt_verify',0),1), 'pre_eng', round(p.get('decrypt_pre_engine',0),1), 'pre_wait', round(p.get('decrypt_pre_wait',0),1))"
}
run default
run pre_start --preverify-at start
run pf_early --prefetch-early
run nopre --no-preverify
run default_b
run pre_start_b --preverify-at start
run nopre_b --no-preverify
