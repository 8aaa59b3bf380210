#!/bin/bash
# round 3: sign bench line with the side stream created lazily (HW-queue mapping check), then decrypt
set -o pipefail
bash tools/gpu_r3_bench_all.sh sign decrypt
