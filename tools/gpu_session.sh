# Full GPU session: all gpu tests, smoke, latency probe, bench (sign default + decrypt + dkg),
# rocprofv3 kernel-trace stats of the default bench, PMC passes (HBM traffic, SQ issue counters).
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-session}
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python -u tools/lat_probe.py > $O/lat.json 2> $O/lat.err || { tail -20 $O/lat.err; exit 1; }
cat $O/lat.json
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u bench.py --workload decrypt --steps 5 --warmup 1 > $O/bench_decrypt.json 2> $O/bench_decrypt.err || { tail -5 $O/bench_decrypt.err; exit 1; }
cat $O/bench_decrypt.json
timeout -k 10 300 python -u bench.py --workload dkg --steps 10 > $O/bench_dkg.json 2> $O/bench_dkg.err || { tail -5 $O/bench_dkg.err; exit 1; }
cat $O/bench_dkg.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/$O/prof_bench.log 2>&1
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-combine"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc/fetch -o run -- python3 $B > $R/$O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc/write -o run -- python3 $B > $R/$O/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU --output-format csv -d $R/$O/pmc/sq -o run -- python3 $B > $R/$O/pmc_sq.log 2>&1
echo session done
