#!/bin/bash
# round 3 final: GPU suite + smoke, sign profile (trace + PMC passes), every bench line
set -o pipefail
mkdir -p gpurun_out/c24
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/c24/pytest_gpu_all.log 2>&1
rc=$?
tail -3 gpurun_out/c24/pytest_gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c24/smoke.log 2>&1 || { tail gpurun_out/c24/smoke.log; exit 1; }
tail -2 gpurun_out/c24/smoke.log
for k in 1 1 0; do
  HBH_SPLIT_CHECK=$k timeout -k 10 120 python3 tools/probe_split.py | tee -a gpurun_out/c24/probe.jsonl || exit 1
done
for r in 1 2; do
  for L in "" hbbft_amd/ab/*.so; do
    HBBFT_HIP_LIB=${L:+$PWD/$L} timeout -k 10 120 python3 tools/probe_split.py > gpurun_out/c24/one.json 2> gpurun_out/c24/err.txt || { tail -5 gpurun_out/c24/err.txt; exit 1; }
    echo "${L:-intree} $(cat gpurun_out/c24/one.json)" | tee -a gpurun_out/c24/ab.txt
  done
done
bash tools/gpu_r3_prof.sh sign_final || exit 1
bash tools/gpu_r3_bench_all.sh sign decrypt dkg epoch
