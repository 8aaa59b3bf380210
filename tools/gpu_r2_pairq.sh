#!/bin/bash
# quick pairing check: parity tests of the pairing + ciphertext paths, then the PAIR bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_protocol.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_pair_pytest.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -40 gpurun_out/r2_pair_pytest.log; exit 1; }
tail -3 gpurun_out/r2_pair_pytest.log
timeout -k 10 200 python -u bench.py --impl pair --steps 5 --warmup 1 --no-cpu-baseline --no-combine > gpurun_out/r2_bench_pair.json 2> gpurun_out/r2_bench_pair.err || { echo "BENCH PAIR FAILED"; tail -20 gpurun_out/r2_bench_pair.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r2_bench_pair.json')); r=d['roofline']; print('value', d['value'], 'kernel_ms', r['avg_launch_ms'], 'frac', r['frac'])"
