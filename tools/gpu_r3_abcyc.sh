#!/bin/bash
# A/B of the combine latency (split master check) over libraries: in-tree and hbbft_amd/ab/*.so, interleaved
set -o pipefail
mkdir -p gpurun_out/abcyc
for r in 1 2 3; do
  for L in "" hbbft_amd/ab/*.so; do
    HBBFT_HIP_LIB=${L:+$PWD/$L} timeout -k 10 120 python3 tools/probe_split.py > gpurun_out/abcyc/one.json 2> gpurun_out/abcyc/err.txt || { tail -5 gpurun_out/abcyc/err.txt; exit 1; }
    echo "${L:-intree} $(cat gpurun_out/abcyc/one.json)" | tee -a gpurun_out/abcyc/ab.txt
  done
done
