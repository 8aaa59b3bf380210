#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/prof_epoch_ba.py > gpurun_out/prof_epoch_ba.txt 2>&1 || { tail -20 gpurun_out/prof_epoch_ba.txt; exit 1; }
grep -E "^(synthetic|ba) epoch" gpurun_out/prof_epoch_ba.txt
