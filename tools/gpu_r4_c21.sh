#!/bin/bash
# round 4, call 21: AUTO's PAIR + QUAD split for (32,768, 49,152] checks -- the boundary tests, then
# AUTO vs PAIR alone across the band
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c21
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_full_size.py tests/test_gpu_pairing.py tests/test_gpu_dev_variants.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for N in 36864 40960 49152 70656 81920 106496; do
    for I in auto pair; do
      timeout -k 10 200 python3 -u bench.py --workload sign --impl $I --batch $N --steps 3 --warmup 1 --no-cpu-baseline --no-combine > $O/s.json 2> $O/s.err || { tail -5 $O/s.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/s.json')); r=d['roofline']; print('batch $N $I pairing-stage %.3f ms' % r['avg_launch_ms'], '%.0f checks/s' % ($N / r['avg_launch_ms'] * 1e3), d.get('verdicts_ok'))" | tee -a $O/split.txt
    done
  done
done
echo done
