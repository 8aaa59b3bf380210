#!/bin/bash
# round 5 call 21: k_wave with one non-inlined stage interpreter (half the code) vs the closing library:
# pairing / combine tests, check latency by size, combine latency, each A/B/A on one box
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c21}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_curve.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for L in new old new old; do
  if [ $L = old ]; then export HBBFT_HIP_LIB=$R/ab_lib/libhbbft_hip_final.so; else unset HBBFT_HIP_LIB; fi
  timeout -k 10 300 python3 -u tools/latency_probe.py 1 1024 4096 > $O/lat_$L.txt 2>&1 || { tail -5 $O/lat_$L.txt; exit 1; }
  timeout -k 10 300 python3 -u tools/combine_trace.py --reps 30 > $O/comb_$L.txt 2>&1 || { tail -5 $O/comb_$L.txt; exit 1; }
  echo "$L $(tr '\n' ' ' < $O/lat_$L.txt) | $(tail -1 $O/comb_$L.txt | sed 's/.*median/median/')"
done
