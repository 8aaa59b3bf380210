#!/bin/bash
# round 5 call 8: multi-chain squares in k_wave -- pairing / combine parity, check latency by size,
# combine latency
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c8}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_curve.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/latency_probe.py 1 1024 2048 4096 8192 > $O/latency.txt 2>&1 || { tail -5 $O/latency.txt; exit 1; }
cat $O/latency.txt
timeout -k 10 300 python3 -u tools/combine_trace.py --reps 30 > $O/combine.txt 2>&1 || { tail -5 $O/combine.txt; exit 1; }
tail -1 $O/combine.txt
