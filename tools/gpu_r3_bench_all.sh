#!/bin/bash
# round 3: every bench line (sign = the headline, decrypt, dkg, epoch) -> gpurun_out/r3_bench_<w>.json
set -o pipefail
mkdir -p gpurun_out
W=${*:-sign decrypt dkg epoch}
for w in $W; do
  timeout -k 10 400 python3 -u bench.py --workload $w > gpurun_out/r3_bench_$w.json 2> gpurun_out/r3_bench_$w.err || { echo "bench $w failed"; tail -20 gpurun_out/r3_bench_$w.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r3_bench_$w.json')); r=d.get('roofline', {})
print('$w', d['metric'], round(d['value']), d['unit'], 'ms/step', round(d['ms_per_step'], 3), 'frac', round(r.get('frac', 0), 3), 'ok', d.get('verdicts_ok'), 'combine', d.get('combine_latency_ms'))"
done
