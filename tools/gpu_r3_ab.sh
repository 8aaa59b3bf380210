#!/bin/bash
# round 3: A/B of the sign (and decrypt) bench lines over the in-tree library and hbbft_amd/ab/*.so,
# interleaved, 3 reps; one line per run: lib, value, isolated launch ms, frac
set -o pipefail
mkdir -p gpurun_out
W=${W:-sign}
for r in 1 2 3; do
  for L in "" hbbft_amd/ab/*.so; do
    HBBFT_HIP_LIB=${L:+$PWD/$L} timeout -k 10 300 python3 -u bench.py --workload $W --steps 5 --warmup 2 --no-cpu-baseline --no-combine > gpurun_out/ab_$W.json 2> gpurun_out/ab_$W.err || { tail -5 gpurun_out/ab_$W.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_$W.json')); r=d['roofline']; print('$W', '${L:-intree}', round(d['value']), round(r['avg_launch_ms'],3), round(r['frac'],4), d.get('verdicts_ok'))" | tee -a gpurun_out/ab_$W.txt
  done
done
