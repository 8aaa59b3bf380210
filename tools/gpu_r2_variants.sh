#!/bin/bash
# parity + bench of the in-tree library, then of variant libraries in tools/variants/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_protocol.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_var_pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 gpurun_out/r2_var_pytest.log; exit 1; }
tail -1 gpurun_out/r2_var_pytest.log
timeout -k 10 300 python3 bench.py --streams 1 --steps 10 --warmup 2 --no-cpu-baseline --no-combine > gpurun_out/r2_var_main.json 2> gpurun_out/r2_var_main.err || { echo "bench failed"; tail gpurun_out/r2_var_main.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r2_var_main.json')); print('in-tree', round(d['value']), d['verdicts_ok'], 'kernel', round(d['roofline']['avg_launch_ms'],3))"
for v in tools/variants/*.so; do
  HBBFT_HIP_LIB=$PWD/$v timeout -k 10 300 python3 bench.py --streams 1 --steps 10 --warmup 2 --no-cpu-baseline --no-combine > gpurun_out/r2_var.json 2> gpurun_out/r2_var.err || { echo "bench $v failed"; tail gpurun_out/r2_var.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r2_var.json')); print('$v', round(d['value']), d['verdicts_ok'], 'kernel', round(d['roofline']['avg_launch_ms'],3))"
done
