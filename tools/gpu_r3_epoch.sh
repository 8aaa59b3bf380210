#!/bin/bash
# round 3: the epoch line with BA-driven coins and with the synthetic coin set, twice each
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for C in ba synthetic; do
    timeout -k 10 300 python3 -u bench.py --workload epoch --epoch-coins $C --no-cpu-baseline > gpurun_out/ep_$C.json 2> gpurun_out/ep_$C.err || { tail -20 gpurun_out/ep_$C.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ep_$C.json')); print('$C', round(d['value'],2), 'epochs/s', round(d['ms_per_step'],1), 'ms', d.get('engine_calls_per_epoch'), 'calls', d.get('checks_drained_per_epoch'), 'checks', d.get('outputs_ok'), d.get('phase_ms'))" | tee -a gpurun_out/epoch_coins_ab.txt
  done
done
cp gpurun_out/ep_ba.json gpurun_out/r3_bench_epoch.json
