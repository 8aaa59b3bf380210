#!/bin/bash
# round 3 profile of one bench configuration: kernel trace + separate PMC passes (FETCH_SIZE,
# WRITE_SIZE, SQ counters), each its own rocprofv3 run
# usage: tools/gpu_r3_prof.sh <tag> [bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof3/$TAG
mkdir -p $O
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-combine --streams 1 $*"
cd /tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $B > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $B > $O/fetch.log 2>&1 || { echo "fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $B > $O/write.log 2>&1 || { echo "write failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU --output-format csv -d $O/sq -o run -- python3 $B > $O/sq.log 2>&1 || { echo "sq failed"; exit 1; }
echo "== $TAG"; find $O/trace -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -c1-160
