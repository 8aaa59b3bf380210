#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dev_variants.py tests/test_gpu_pairing.py tests/test_gpu_protocol.py tests/test_gpu_pool.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_streams_pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 gpurun_out/r2_streams_pytest.log; exit 1; }
tail -2 gpurun_out/r2_streams_pytest.log
for st in 1 2 3; do
  timeout -k 10 300 python3 bench.py --streams $st --steps 10 --warmup 2 --no-cpu-baseline --no-combine > gpurun_out/r2_sign_s$st.json 2> gpurun_out/r2_sign_s$st.err || { echo "bench failed"; tail gpurun_out/r2_sign_s$st.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r2_sign_s$st.json')); print('streams $st', round(d['value']), round(d['ms_per_step'],2), d['verdicts_ok'], 'kernel', round(d['roofline']['avg_launch_ms'],2))"
done
