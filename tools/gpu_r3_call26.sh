#!/bin/bash
# round 3: rocprofv3 kernel trace + stats of the exact default bench command (python3 bench.py)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/c26
mkdir -p $O
cd /tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py > $O/bench.json 2> $O/bench.err || { echo "trace failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json | cut -c1-400
find $O/trace -name "*kernel_stats.csv" | head -1 | xargs head -8 | cut -c1-160
