#!/bin/bash
# round 4, call 22: the lane-octo pairing kernel (HBH_IMPL_OCT) -- parity tests, then kernel time vs
# WAVE / QUAD from 2,048 to 16,384 checks (sign workload)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c22
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pairing.py tests/test_gpu_dev_variants.py -k "oct" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for N in 2048 4096 6144 8192 12288 16384; do
  for I in oct wave quad; do
    timeout -k 10 200 python3 -u bench.py --workload sign --impl $I --batch $N --steps 3 --warmup 1 --no-cpu-baseline --no-combine > $O/s.json 2> $O/s.err || { tail -5 $O/s.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s.json')); r=d['roofline']; print('batch $N $I pairing-stage %.3f ms' % r['avg_launch_ms'], '%.0f checks/s' % ($N / r['avg_launch_ms'] * 1e3), d.get('verdicts_ok'))" | tee -a $O/sweep.txt
  done
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_full_size.py -k "oct" > $O/pytest_full.log 2>&1 || { tail -30 $O/pytest_full.log; exit 1; }
tail -1 $O/pytest_full.log
echo done
