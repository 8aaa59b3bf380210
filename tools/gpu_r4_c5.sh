#!/bin/bash
# round 4 call 5: 64-bit shift microbenchmark, epoch Python A/B (in-tree flows vs hbbft_amd/ab/pyold),
# sign / decrypt A/B (in-tree vs hbbft_amd/ab/tower.so)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c5
mkdir -p $O
cd $R
timeout -k 10 120 tools/ubench_shift > $O/ubench_shift.txt 2>&1 || { cat $O/ubench_shift.txt; exit 1; }
cat $O/ubench_shift.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_honey_badger.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=r4c5 REPS=3 bash tools/gpu_r4_epoch_ab.sh || exit 1
TAG=r4c5 WORKLOADS="sign decrypt" REPS=2 bash tools/gpu_r4_ab.sh || exit 1
