#!/bin/bash
# round 3: register-resident cyclotomic-squaring runs in k_wave -- the whole GPU suite, then the
# combine latency (split and unsplit) and a kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cyc6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cyc6/tests.log 2>&1
rc=$?
tail -5 gpurun_out/cyc6/tests.log
[ $rc -eq 0 ] || exit $rc
for k in 1 0 1; do
  HBH_SPLIT_CHECK=$k timeout -k 10 120 python3 tools/probe_split.py >> gpurun_out/cyc6/ab.jsonl 2>> gpurun_out/cyc6/ab.err || { tail gpurun_out/cyc6/ab.err; exit 1; }
done
cat gpurun_out/cyc6/ab.jsonl
R=$GRAFT_REPO_ROOT
cd /tmp && PROBE_REPS=5 timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/cyc6/trace -o run -- python3 $R/tools/probe_split.py > $R/gpurun_out/cyc6/trace.log 2>&1 || { echo trace failed; exit 1; }
cut -c1-160 $R/gpurun_out/cyc6/trace/run_kernel_stats.csv
