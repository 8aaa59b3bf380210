#!/bin/bash
# round 4, call 12: epoch (configs[4]) window sweep -- messages per drain (bench --window)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c12
mkdir -p $O
cd $R
# the lane-quad line-table prep: pairing tests (TABLE sides everywhere), then the sign line's prep time
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pairing.py tests/test_gpu_dev_variants.py tests/test_gpu_full_size.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for L in "" hbbft_amd/ab/tower.so; do
  HBBFT_HIP_LIB=${L:+$R/$L} timeout -k 10 300 python3 -u bench.py --workload sign --steps 5 --warmup 2 --no-cpu-baseline --no-combine > $O/s.json 2> $O/s.err || { tail -5 $O/s.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/s.json')); k=d['roofline']['kernels']; print('sign ${L:-intree}', round(d['value']), round(d['ms_per_step'],3), [(x['kernel'], round(x['avg_launch_ms'],3)) for x in k], d.get('verdicts_ok'))" | tee -a $O/prep.txt
done
for r in 1 2; do
  for W in 4096 8192 16384 32768; do
    timeout -k 10 300 python3 -u bench.py --workload epoch --steps 8 --warmup 2 --no-cpu-baseline --window $W > $O/e_$W.json 2> $O/e_$W.err || { tail -5 $O/e_$W.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e_$W.json')); h=d['host_vs_gpu']; print('window $W', round(d['value'],2), round(d['ms_per_step'],1), 'calls', d['engine_calls_per_epoch'], 'drained', d['checks_drained_per_epoch'], 'gpu', round(h['gpu_kernel_ms'],1), {k: round(v,1) for k,v in h['gpu_kernel_by_stage_ms'].items()}, 'host', round(h['host_ms'],1), 'blocked', round(h['blocked_on_engine_ms'],1), 'wave frac', round(d['roofline']['frac'],3), d.get('outputs_ok'))" | tee -a $O/windows.txt
  done
done
echo done
