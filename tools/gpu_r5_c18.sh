#!/bin/bash
# round 5 call 18: epoch window sweep, interleaved repeats
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c18}
mkdir -p $O
cd $R
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 400 python3 -u bench.py --workload epoch --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); p=d.get('phase_ms',{}); h=d.get('host_vs_gpu',{}); print('%-10s' % '$tag', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'host', round(h.get('host_ms',0),1), 'blocked', round(h.get('blocked_on_engine_ms',0),1), 'coin', round(p.get('coin_verify',0),1), 'dverify', round(p.get('decrypt_verify',0),1))"
}
for r in a b c; do
  run w6144$r
  run w12288$r --window 12288
  run w16384$r --window 16384
  run w12288p$r --window 12288 --pipeline
done
