#!/bin/bash
# round 5 call 17: epoch window sizes and pipelined drains under the round-5 schedule
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c17}
mkdir -p $O
cd $R
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 400 python3 -u bench.py --workload epoch --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); p=d.get('phase_ms',{}); h=d.get('host_vs_gpu',{}); print('%-10s' % '$tag', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'host', round(h.get('host_ms',0),1), 'blocked', round(h.get('blocked_on_engine_ms',0),1), 'coin', round(p.get('coin_verify',0),1), 'dverify', round(p.get('decrypt_verify',0),1))"
}
run w6144
run w4096 --window 4096
run w8192 --window 8192
run w12288 --window 12288
run pipe --pipeline
run w6144b
run w8192b --window 8192
run w4096b --window 4096
