#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r3_tests.sh || exit $?
rm -f gpurun_out/epoch_coins_ab.txt
bash tools/gpu_r3_epoch.sh
