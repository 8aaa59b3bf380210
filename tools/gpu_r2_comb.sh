#!/bin/bash
# combine path: curve/protocol/dev-variant parity tests, then the latency probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_curve.py tests/test_gpu_protocol.py tests/test_gpu_dev_variants.py tests/test_gpu_full_size.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_comb_pytest.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -40 gpurun_out/r2_comb_pytest.log; exit 1; }
tail -3 gpurun_out/r2_comb_pytest.log
./tools/gpu_probe_combine.sh
timeout -k 10 200 python -u bench.py --impl lane_coop --batch 8192 --steps 5 --warmup 1 --no-cpu-baseline --no-combine > gpurun_out/r2_bench_lc8k.json 2> gpurun_out/r2_bench_lc8k.err || { echo "BENCH LC FAILED"; tail -20 gpurun_out/r2_bench_lc8k.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r2_bench_lc8k.json')); r=d['roofline']; print('lane_coop 8192: value', d['value'], 'kernel_ms', r['avg_launch_ms'])"
