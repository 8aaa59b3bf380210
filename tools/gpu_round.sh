# One GPU session: parity tests, smoke, bench, rocprof kernel trace + one PMC pass, microbenchmarks.
# Usage (via gpurun, from the repo root): bash tools/gpu_round.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-r01}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_bench.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-combine > $GRAFT_REPO_ROOT/$O/pmc_fetch.log 2>&1 || echo "pmc pass failed"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-combine > $GRAFT_REPO_ROOT/$O/pmc_write.log 2>&1 || echo "pmc pass failed"
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/ubench_fpmul > $O/ubench_fpmul.txt 2>&1 || true
timeout -k 10 120 ./tools/ubench_imad > $O/ubench_imad.txt 2>&1 || true
echo done
