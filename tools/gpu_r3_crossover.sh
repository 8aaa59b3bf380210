#!/bin/bash
# AUTO crossover without LANE_COOP: ms per step of the sign workload for WAVE and PAIR by batch size
set -o pipefail
mkdir -p gpurun_out
for B in 2048 4096 6144 8192 12288 16384 24576; do
  for I in wave pair; do
    timeout -k 10 200 python3 -u bench.py --impl $I --batch $B --steps 3 --warmup 1 --streams 1 --no-cpu-baseline --no-combine > gpurun_out/xo.json 2> gpurun_out/xo.err || { tail -5 gpurun_out/xo.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/xo.json')); print('batch', $B, '$I', round(d['ms_per_step'],3), 'ms', round(d['value']), '/s', d['verdicts_ok'])" | tee -a gpurun_out/crossover_r3.txt
  done
done
