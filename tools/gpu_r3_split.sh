#!/bin/bash
# round 3: split master check -- its tests, then the combine latency A/B and a kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/split
timeout -k 10 400 python -u -m pytest tests/test_gpu_curve.py tests/test_gpu_protocol.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/split/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/split/tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
for k in 1 0 1 0; do
  HBH_SPLIT_CHECK=$k timeout -k 10 120 python3 tools/probe_split.py >> gpurun_out/split/ab.jsonl 2>> gpurun_out/split/ab.err || { tail gpurun_out/split/ab.err; exit 1; }
done
cat gpurun_out/split/ab.jsonl
R=$GRAFT_REPO_ROOT
cd /tmp && PROBE_REPS=5 timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/split/trace -o run -- python3 $R/tools/probe_split.py > $R/gpurun_out/split/trace.log 2>&1 || { echo trace failed; exit 1; }
cat $R/gpurun_out/split/trace/run_kernel_stats.csv | cut -c1-200
