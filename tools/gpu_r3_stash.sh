#!/bin/bash
# round 3: f parked in the LDS stash while a walked side computes its line (KP_STASH_WALK, in-tree)
# vs not (hbbft_amd/ab/nostash.so): pairing parity on the in-tree library, then sign / decrypt A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_stash_tests.log 2>&1 || { tail -30 gpurun_out/r3_stash_tests.log; exit 1; }
tail -1 gpurun_out/r3_stash_tests.log
rm -f gpurun_out/ab_sign.txt gpurun_out/ab_decrypt.txt
bash tools/gpu_r3_ab.sh && W=decrypt bash tools/gpu_r3_ab.sh
