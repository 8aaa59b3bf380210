#!/bin/bash
# round 3: lazy reduction in the lane-pair tower (HP_LAZY, csrc/pfp.hpp) -- pairing parity on the
# in-tree (lazy) library, then sign / decrypt A/B against hbbft_amd/ab/lazy0.so (HP_LAZY=0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_lazy_tests.log 2>&1 || { tail -30 gpurun_out/r3_lazy_tests.log; exit 1; }
tail -1 gpurun_out/r3_lazy_tests.log
bash tools/gpu_r3_ab.sh && W=decrypt bash tools/gpu_r3_ab.sh
