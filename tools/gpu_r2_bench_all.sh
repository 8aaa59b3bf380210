#!/bin/bash
# round 2: every bench line (sign = the headline, decrypt, dkg, epoch) -> gpurun_out/r2_bench_<w>.json
set -o pipefail
mkdir -p gpurun_out
W=${*:-sign decrypt dkg epoch}
for w in $W; do
  timeout -k 10 400 python3 -u bench.py --workload $w > gpurun_out/r2_bench_$w.json 2> gpurun_out/r2_bench_$w.err || { echo "bench $w failed"; tail -20 gpurun_out/r2_bench_$w.err; exit 1; }
  echo "== $w"; cat gpurun_out/r2_bench_$w.json
done
