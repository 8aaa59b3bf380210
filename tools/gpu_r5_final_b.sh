#!/bin/bash
# round 5 closing evidence, part B: the four bench lines (default sign line = the driver's BENCH)
# citing profiles/r05/pmc_traffic.json of part A (same library), the default bench under rocprofv3
# --kernel-trace --stats, the check-latency sweep and the combine latency.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-final_b}
mkdir -p $O
cd $R
sha256sum hbbft_amd/libhbbft_hip.so > $O/lib_sha256.txt
for W in ${WORKLOADS:-sign decrypt dkg epoch}; do
  timeout -k 10 600 python3 -u bench.py --workload $W > $O/bench_$W.json 2> $O/bench_$W.err || { tail -5 $O/bench_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$W.json')); r=d.get('roofline',{}); print('$W', d['value'], d['unit'], 'ms/step', round(d['ms_per_step'],3), 'frac', round(r.get('frac',0),4), 'traffic', r.get('traffic'), 'match', (r.get('traffic_source') or {}).get('matches_loaded_lib'))"
done
timeout -k 10 300 python3 -u tools/latency_probe.py 1 1024 2048 4096 8192 > $O/latency.txt 2>&1 || { tail -5 $O/latency.txt; exit 1; }
cat $O/latency.txt
cd /tmp
mkdir -p $O/default_bench
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/default_bench -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $O/default_bench/run.log 2>&1 || { echo "default trace failed"; tail -5 $O/default_bench/run.log; exit 1; }
head -6 $O/default_bench/run_kernel_stats.csv
echo done
