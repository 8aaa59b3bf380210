#!/bin/bash
# round 4, call 35: line tables on lane octos (k_oct_prep) -- GPU suite, then the sign line A/B against the
# lane-quad prep library (hbbft_amd/ab/prep_quad.so), interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c35
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for L in hbbft_amd/ab/prep_quad.so hbbft_amd/libhbbft_hip.so; do
    HBBFT_HIP_LIB=$R/$L timeout -k 10 300 python3 -u bench.py --workload sign --no-cpu-baseline > $O/s.json 2> $O/s.err || { tail -5 $O/s.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s.json')); ks=d['roofline'].get('kernels', []); print('$L', 'sign %.3f M/s' % (d['value']/1e6), 'ms %.3f' % d['ms_per_step'], [(k['kernel'], round(k['avg_launch_ms'], 3)) for k in ks])" | tee -a $O/ab.txt
  done
done
echo done
