#!/bin/bash
# round 3: whole -m gpu suite + smoke, then the epoch line with BA-driven coins
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r3_tests.sh || exit $?
bash tools/gpu_r3_bench_all.sh epoch
