#!/bin/bash
# round 3: commit-set tests, then the Ack-check kernel sweep (quad vs one lane) by acks per call
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_commit_set.py tests/test_gpu_sync_key_gen.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_cs_tests.log 2>&1 || { tail -30 gpurun_out/r3_cs_tests.log; exit 1; }
tail -2 gpurun_out/r3_cs_tests.log
for K in 1 4 16 50 100; do
  for I in quad lane; do
    timeout -k 10 200 python3 -u bench.py --workload dkg --dkg-nodes $K --ack-impl $I --steps 4 --no-cpu-baseline > gpurun_out/ack.json 2> gpurun_out/ack.err || { tail -5 gpurun_out/ack.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ack.json')); print('acks', d['config']['total_acks'], '$I', round(d['ms_per_step'],3), 'ms', round(d['value']), '/s host', round(d['host_to_host_ms'],2), 'frac', round(d['roofline']['frac'],3), d['verdicts_ok'])" | tee -a gpurun_out/ack_sweep.txt
  done
done
