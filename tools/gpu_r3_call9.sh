#!/bin/bash
# round 3: integer multiply issue rates, the MAD-digit variant (hbbft_amd/ab/mad.so) on the pairing
# tests and the sign / decrypt A/B, and the new DHB key-gen test on the in-tree library
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench_mullo | tee gpurun_out/ubench_mullo.txt || exit 1
HBBFT_HIP_LIB=$PWD/hbbft_amd/ab/mad.so timeout -k 10 600 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_curve.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_mad_tests.log 2>&1 || { tail -20 gpurun_out/r3_mad_tests.log; exit 1; }
tail -1 gpurun_out/r3_mad_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_dhb_key_gen.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_dhb.log 2>&1 || { tail -20 gpurun_out/r3_dhb.log; exit 1; }
tail -1 gpurun_out/r3_dhb.log
bash tools/gpu_r3_ab.sh && W=decrypt bash tools/gpu_r3_ab.sh
