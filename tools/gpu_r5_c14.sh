#!/bin/bash
# round 5 call 14: where the epoch's coin resolve / local time goes -- this tree and the round-4 tree
# with and without the decryption pre-verification and the coin prefetch
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c14}
mkdir -p $O
run() {  # tag dir args...
  local tag=$1 dir=$2; shift 2
  ( cd $dir && timeout -k 10 400 python3 -u bench.py --workload epoch --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err ) || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); p=d.get('phase_ms',{}); h=d.get('host_vs_gpu',{}); print('%-14s' % '$tag', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'host', round(h.get('host_ms',0),1), 'blocked', round(h.get('blocked_on_engine_ms',0),1), 'resolve', round(p.get('coin_resolve',0),1), 'local', round(p.get('coin_local',0),1), 'msgs', round(p.get('coin_messages',0),1), 'dsetup', round(p.get('decrypt_setup',0),1), 'dverify', round(p.get('decrypt_verify',0),1), 'pre_eng', round(p.get('decrypt_pre_engine',0),1))"
}
run now $R
run r4 $R/ab_r4wt
run now_nopre $R --no-preverify
run r4_nopre $R/ab_r4wt --no-preverify
run now_nopf $R --no-prefetch
run r4_nopf $R/ab_r4wt --no-prefetch
run now_b $R
run r4_b $R/ab_r4wt
