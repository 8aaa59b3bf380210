#!/bin/bash
# A/B of the sign bench line: the in-tree library vs hbbft_amd/ab/lib_base.so
set -o pipefail
mkdir -p gpurun_out
for L in "" "$PWD/hbbft_amd/ab/lib_base.so"; do
  HBBFT_HIP_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-combine > gpurun_out/ab_sign.json 2> gpurun_out/ab_sign.err || { tail -5 gpurun_out/ab_sign.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_sign.json')); r=d['roofline']; print('${L:-new}', round(d['value']), r['avg_launch_ms'], r['frac'])"
done
