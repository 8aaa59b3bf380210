#!/bin/bash
# kernel trace of the epoch bench line -> gpurun_out/prof_epoch/
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_epoch
mkdir -p $O
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --workload epoch --steps 3 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || { echo trace failed; tail -5 $O/trace.log; exit 1; }
head -20 $O/trace/run_kernel_stats.csv | cut -c1-160
tail -1 $O/trace.log | cut -c1-300
