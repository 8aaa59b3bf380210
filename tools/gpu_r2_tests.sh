#!/bin/bash
# round 2: GPU test files given as arguments (default: the whole -m gpu suite)
set -o pipefail
mkdir -p gpurun_out
T=${*:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r2_tests.log | tail -60
exit $rc
