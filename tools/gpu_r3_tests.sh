#!/bin/bash
# round 3: GPU test files given as arguments (default: the whole -m gpu suite), then smoke()
set -o pipefail
mkdir -p gpurun_out
T=${*:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r3_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1
rc=$?
tail -3 gpurun_out/r3_smoke.log
exit $rc
