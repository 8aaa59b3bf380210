#!/bin/bash
# round 4, call 8: the lane-quad kernel (HBH_IMPL_QUAD) -- pairing parity tests, then the batch-size
# sweep of WAVE / QUAD / PAIR on the sign workload (kernel ms per call, HIP events)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c8
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pairing.py tests/test_gpu_dev_variants.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for N in ${SIZES:-2048 4096 8192 12288 16384 24576 32768 49152 65536}; do
  for I in ${IMPLS:-wave quad pair}; do
    if [ $I = wave ] && [ $N -gt 16384 ]; then continue; fi
    timeout -k 10 200 python3 -u bench.py --workload sign --impl $I --batch $N --steps 3 --warmup 1 --no-cpu-baseline --no-combine > $O/s_${I}_$N.json 2> $O/s_${I}_$N.err || { tail -5 $O/s_${I}_$N.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s_${I}_$N.json')); r=d['roofline']; print('batch $N $I kernel %.3f ms' % r['avg_launch_ms'], '%.0f checks/s' % ($N / r['avg_launch_ms'] * 1e3), 'frac %.3f' % r['frac'], d.get('verdicts_ok', d.get('outputs_ok')))" | tee -a $O/sweep.txt
  done
done
echo done
