#!/bin/bash
# round 5 call 19: FD parity test with the duplicate-heavy short run
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c19}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_commit_set.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -10 $O/pytest.log; exit $rc
