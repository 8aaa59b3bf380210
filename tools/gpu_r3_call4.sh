#!/bin/bash
# round 3: vartime FE inversion variant (hbbft_amd/ab/inv.so): pairing + full-size parity on it, the
# new threshold_sign.rs size-sweep port on the in-tree library, then the sign/decrypt A/B
set -o pipefail
mkdir -p gpurun_out
HBBFT_HIP_LIB=$PWD/hbbft_amd/ab/inv.so timeout -k 10 600 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_inv_tests.log 2>&1 || { tail -20 gpurun_out/r3_inv_tests.log; exit 1; }
tail -2 gpurun_out/r3_inv_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_threshold_sign_sizes.py -m gpu -x -v --timeout 500 --timeout-method thread --durations=5 > gpurun_out/r3_tssizes.log 2>&1 || { tail -20 gpurun_out/r3_tssizes.log; exit 1; }
tail -8 gpurun_out/r3_tssizes.log
bash tools/gpu_r3_ab.sh && W=decrypt bash tools/gpu_r3_ab.sh
