#!/bin/bash
# round 3: GPU suite, then the sign (headline + combine latency) and epoch bench lines
set -o pipefail
mkdir -p gpurun_out/c20
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c20/tests.log 2>&1
rc=$?
tail -3 gpurun_out/c20/tests.log
[ $rc -eq 0 ] || exit $rc
for k in 1 0; do
  HBH_SPLIT_CHECK=$k timeout -k 10 120 python3 tools/probe_split.py >> gpurun_out/c20/probe.jsonl 2>> gpurun_out/c20/probe.err || { tail gpurun_out/c20/probe.err; exit 1; }
done
cat gpurun_out/c20/probe.jsonl
bash tools/gpu_r3_bench_all.sh sign epoch
