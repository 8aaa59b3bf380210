#!/bin/bash
# A/B of the sign bench line over libraries: the in-tree one and every hbbft_amd/ab/*.so, interleaved
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for L in "" hbbft_amd/ab/*.so; do
    HBBFT_HIP_LIB=${L:+$PWD/$L} timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-combine > gpurun_out/ab_sign.json 2> gpurun_out/ab_sign.err || { tail -5 gpurun_out/ab_sign.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_sign.json')); r=d['roofline']; print('${L:-intree}', round(d['value']), r['avg_launch_ms'], r['frac'])"
  done
done
