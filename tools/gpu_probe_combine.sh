#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/comb
timeout -k 10 200 python3 tools/probe_combine.py > gpurun_out/comb/probe.json 2> gpurun_out/comb/probe.err || { tail gpurun_out/comb/probe.err; exit 1; }
cat gpurun_out/comb/probe.json
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/comb/trace -o run -- python3 $R/tools/probe_combine.py > $R/gpurun_out/comb/trace.log 2>&1 || { echo trace failed; exit 1; }
cat $R/gpurun_out/comb/trace/run_kernel_stats.csv
