# bench + rocprofv3 kernel-trace/stats summary (run via gpurun from the repo root)
set -e
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline 2>&1 | tee gpurun_out/${TAG}_bench.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_bench.log 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -name "*stats*" | head
