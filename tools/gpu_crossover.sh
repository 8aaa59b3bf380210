#!/bin/bash
# pairing kernel time vs batch size for the lane-pair and lane-coop implementations (AUTO crossover)
set -o pipefail
mkdir -p gpurun_out/xover
for b in 64 1024 4096 8192 16384; do
  for impl in pair lane_coop; do
    timeout -k 10 200 python3 bench.py --impl $impl --batch $b --steps 5 --warmup 1 --no-cpu-baseline --no-combine > gpurun_out/xover/${impl}_$b.json 2> gpurun_out/xover/${impl}_$b.err || { echo "failed $impl $b"; tail -5 gpurun_out/xover/${impl}_$b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/xover/${impl}_$b.json')); print('$impl', $b, 'ms/step', round(d['ms_per_step'],3), 'value', round(d['value']))"
  done
done
