#!/bin/bash
# round 4, call 27: epoch line vs messages per drain (window) after the flow fast paths
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c27
mkdir -p $O
cd $R
for r in 1 2; do
  for W in 5120 6144 7168 8192 10240; do
    timeout -k 10 300 python3 -u bench.py --workload epoch --window $W --no-cpu-baseline > $O/e.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e.json')); h=d['host_vs_gpu']; r=d['roofline']; print('window $W epoch %.2f/s' % d['value'], 'ms %.1f host %.1f gpu %.1f' % (d['ms_per_step'], h['host_ms'], h['gpu_kernel_ms']), 'drains/epoch %.1f avg %d checks %.2f ms' % (d['engine_calls_per_epoch'], r['units_per_launch'], r['avg_launch_ms']), 'blocked', {k: round(v, 1) for k, v in h['blocked_by_phase_ms'].items()})" | tee -a $O/windows.txt
  done
done
echo done
