#!/bin/bash
# round 3 closing call: GPU suite + smoke, combine probe (split / unsplit), sign profile
# (trace + PMC passes), every bench line
set -o pipefail
mkdir -p gpurun_out/c25
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/c25/pytest_gpu_all.log 2>&1
rc=$?
tail -3 gpurun_out/c25/pytest_gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c25/smoke.log 2>&1 || { tail gpurun_out/c25/smoke.log; exit 1; }
tail -2 gpurun_out/c25/smoke.log
for k in 1 1 0; do
  HBH_SPLIT_CHECK=$k timeout -k 10 120 python3 tools/probe_split.py | tee -a gpurun_out/c25/probe.jsonl || exit 1
done
bash tools/gpu_r3_prof.sh sign_final || exit 1
bash tools/gpu_r3_bench_all.sh sign decrypt dkg epoch
