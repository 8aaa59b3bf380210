#!/bin/bash
# round 5 closing epoch line on the final code (library unchanged since final_a/b), three samples
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-final_e}
mkdir -p $O
cd $R
sha256sum hbbft_amd/libhbbft_hip.so > $O/lib_sha256.txt
for k in 1 2 3; do
  timeout -k 10 600 python3 -u bench.py --workload epoch > $O/bench_epoch_$k.json 2> $O/bench_epoch_$k.err || { tail -5 $O/bench_epoch_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_epoch_$k.json')); h=d['host_vs_gpu']; print('epoch', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'host', round(h['host_ms'],1), 'blocked', round(h['blocked_on_engine_ms'],1), 'ok', d['outputs_ok'], 'cpu', d['cpu_baseline']['value'])"
done
