# quick GPU check: pairing parity tests + bench of both pairing implementations
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-quick}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pairing.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-combine --impl lane_coop > $O/bench_lc.json 2> $O/bench_lc.err || { tail -20 $O/bench_lc.err; exit 1; }
cat $O/bench_lc.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-combine --impl thread > $O/bench_thread.json 2> $O/bench_thread.err
cat $O/bench_thread.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-combine > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
cut -d, -f1-4 $GRAFT_REPO_ROOT/$O/prof/run_kernel_stats.csv | sed 's/(.*)"/"/'
