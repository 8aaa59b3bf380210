# combine-path GPU check: curve parity tests, latency probe, bench with combine (no CPU baseline)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-combine}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python -u tools/lat_probe.py > $O/lat.json 2> $O/lat.err || { tail -20 $O/lat.err; exit 1; }
cat $O/lat.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
