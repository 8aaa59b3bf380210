#!/bin/bash
# round 2: lane-pair kernel parity + first throughput numbers
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pairing.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_pair_pytest.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -40 gpurun_out/r2_pair_pytest.log; exit 1; }
tail -5 gpurun_out/r2_pair_pytest.log
timeout -k 10 200 python -u bench.py --impl pair --steps 5 --warmup 1 --no-cpu-baseline --no-combine > gpurun_out/r2_bench_pair.json 2> gpurun_out/r2_bench_pair.err || { echo "BENCH PAIR FAILED"; tail -20 gpurun_out/r2_bench_pair.err; exit 1; }
cat gpurun_out/r2_bench_pair.json
timeout -k 10 200 python -u bench.py --impl thread_signed --steps 5 --warmup 1 --no-cpu-baseline --no-combine > gpurun_out/r2_bench_ts.json 2> gpurun_out/r2_bench_ts.err || { echo "BENCH TS FAILED"; tail -20 gpurun_out/r2_bench_ts.err; exit 1; }
cat gpurun_out/r2_bench_ts.json
