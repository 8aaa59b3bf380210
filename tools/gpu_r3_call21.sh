#!/bin/bash
# round 3: GPU suite; combine-latency A/B (in-tree = one pair per wave, homogeneous walk; ab/pairs2 = two
# pairs per wave); then the sign (headline + combine latency) and epoch bench lines
set -o pipefail
mkdir -p gpurun_out/c21
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c21/tests.log 2>&1
rc=$?
tail -3 gpurun_out/c21/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for L in "" hbbft_amd/ab/*.so; do
    HBBFT_HIP_LIB=${L:+$PWD/$L} timeout -k 10 120 python3 tools/probe_split.py > gpurun_out/c21/one.json 2> gpurun_out/c21/err.txt || { tail -5 gpurun_out/c21/err.txt; exit 1; }
    echo "${L:-intree} $(cat gpurun_out/c21/one.json)" | tee -a gpurun_out/c21/ab.txt
  done
done
HBH_SPLIT_CHECK=0 timeout -k 10 120 python3 tools/probe_split.py | tee -a gpurun_out/c21/ab.txt
bash tools/gpu_r3_bench_all.sh sign epoch
