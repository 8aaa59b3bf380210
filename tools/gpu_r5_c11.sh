#!/bin/bash
# round 5 call 11: epoch A/B on one box -- round-4 final tree (Python + library, ab_r4wt/) vs this
# tree, and the round-4 Python on this library (which side the epoch slowdown comes from)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c11}
mkdir -p $O
run() {  # tag dir [lib]
  local tag=$1 dir=$2 lib=$3
  ( cd $dir && if [ -n "$lib" ]; then export HBBFT_HIP_LIB=$lib; fi; timeout -k 10 400 python3 -u bench.py --workload epoch --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err ) || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); p=d.get('phase_ms',{}); h=d.get('host_vs_gpu',{}); print('$tag', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'host', round(h.get('host_ms',0),1), 'blocked', round(h.get('blocked_on_engine_ms',0),1), 'gpu', json.dumps({k: round(v,1) for k,v in h.get('gpu_kernel_by_stage_ms',{}).items()}), 'resolve', round(p.get('coin_resolve',0),1), 'local', round(p.get('coin_local',0),1), 'msgs', round(p.get('coin_messages',0),1))"
}
run now1 $R
run r4_1 $R/ab_r4wt
run r4py_nowlib $R/ab_r4wt $R/hbbft_amd/libhbbft_hip.so
run now2 $R
run r4_2 $R/ab_r4wt
