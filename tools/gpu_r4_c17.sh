#!/bin/bash
# round 4, call 17: lane-quad kernel under the max-ilp / iterative-ilp schedulers (ab/qmaxilp.so,
# ab/qitilp.so) vs the default at 8,192 / 16,384 checks; the epoch after the flow changes (tests + line)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c17
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_honey_badger.py tests/test_gpu_binary_agreement.py tests/test_gpu_protocol.py tests/test_gpu_threshold_sign_sizes.py tests/test_gpu_dhb_era.py tests/test_gpu_wire_msgs.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for N in 8192 16384; do
    for L in "" hbbft_amd/ab/qmaxilp.so hbbft_amd/ab/qitilp.so; do
      HBBFT_HIP_LIB=${L:+$R/$L} timeout -k 10 200 python3 -u bench.py --workload sign --impl quad --batch $N --steps 3 --warmup 1 --no-cpu-baseline --no-combine > $O/q.json 2> $O/q.err || { tail -5 $O/q.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/q.json')); r=d['roofline']; print('quad $N', '${L:-intree}', 'kernel %.3f ms' % r['avg_launch_ms'], 'frac %.3f' % r['frac'], d.get('verdicts_ok'))" | tee -a $O/ab.txt
    done
  done
done
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --workload epoch --steps 8 --warmup 2 --no-cpu-baseline > $O/e.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e.json')); h=d.get('host_vs_gpu'); print('epoch', round(d['value'],2), round(d['ms_per_step'],1), 'blocked', {k: round(v,1) for k,v in h['blocked_by_phase_ms'].items()}, 'gpu', round(h['gpu_kernel_ms'],1), 'host', round(h['host_ms'],1), d.get('outputs_ok'))" | tee -a $O/epoch.txt
done
echo done
