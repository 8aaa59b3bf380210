#!/bin/bash
# round 3: whole -m gpu suite + smoke, then the network-wide dkg line and the sign line
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r3_tests.sh || exit $?
timeout -k 10 300 python3 -u bench.py --workload dkg --steps 6 > gpurun_out/r3_bench_dkg.json 2> gpurun_out/r3_bench_dkg.err || { tail -20 gpurun_out/r3_bench_dkg.err; exit 1; }
tail -c 1500 gpurun_out/r3_bench_dkg.json
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 > gpurun_out/r3_bench_sign.json 2> gpurun_out/r3_bench_sign.err || { tail -20 gpurun_out/r3_bench_sign.err; exit 1; }
tail -c 1500 gpurun_out/r3_bench_sign.json
