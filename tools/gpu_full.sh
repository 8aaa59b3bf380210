# Full GPU session: all gpu tests, smoke, bench (all workloads), rocprof kernel trace + PMC passes.
set -e
export TMPDIR=/tmp
TAG=${1:-r01}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
timeout -k 10 300 python -u bench.py --workload decrypt --steps 5 --warmup 1 > $O/bench_decrypt.json 2> $O/bench_decrypt.err || tail -5 $O/bench_decrypt.err
cat $O/bench_decrypt.json
timeout -k 10 400 python -u bench.py --workload dkg --steps 10 > $O/bench_dkg.json 2> $O/bench_dkg.err || tail -5 $O/bench_dkg.err
cat $O/bench_dkg.json
timeout -k 10 300 python -u bench.py --impl lane_coop --steps 5 --warmup 1 --no-cpu-baseline --no-combine > $O/bench_lane_coop.json 2> $O/bench_lane_coop.err
cat $O/bench_lane_coop.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_bench.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-combine > $GRAFT_REPO_ROOT/$O/pmc_fetch.log 2>&1 || echo "pmc pass failed"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-combine > $GRAFT_REPO_ROOT/$O/pmc_write.log 2>&1 || echo "pmc pass failed"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_sq -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-combine > $GRAFT_REPO_ROOT/$O/pmc_sq.log 2>&1 || echo "pmc pass failed"
echo done
