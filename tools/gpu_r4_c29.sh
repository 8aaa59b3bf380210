#!/bin/bash
# round 4, call 29: window 6,144 default; decrypt-phase sub-timings
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c29
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_honey_badger.py tests/test_gpu_binary_agreement.py tests/test_gpu_wire_msgs.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --workload epoch > $O/epoch_$r.json 2> $O/epoch_$r.err || { tail -5 $O/epoch_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/epoch_$r.json')); h=d['host_vs_gpu']; print('epoch %.2f/s' % d['value'], 'ms %.1f host %.1f gpu %.1f' % (d['ms_per_step'], h['host_ms'], h['gpu_kernel_ms']), {k: round(v, 1) for k, v in d['phase_ms'].items()}, d['outputs_ok'])" | tee -a $O/epoch.txt
done
echo done
