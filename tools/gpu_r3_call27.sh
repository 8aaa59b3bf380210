#!/bin/bash
# round 3: split vs unsplit combine latency by batch size (t = 21, t = 33), then the default-bench profile
set -o pipefail
mkdir -p gpurun_out/c27
timeout -k 10 240 python3 -u tools/probe_split_sweep.py 21 1 8 16 32 64 > gpurun_out/c27/sweep21.jsonl 2> gpurun_out/c27/sweep21.err || { tail -5 gpurun_out/c27/sweep21.err; exit 1; }
cat gpurun_out/c27/sweep21.jsonl
timeout -k 10 300 python3 -u tools/probe_split_sweep.py 33 8 16 33 50 100 > gpurun_out/c27/sweep33.jsonl 2> gpurun_out/c27/sweep33.err || { tail -5 gpurun_out/c27/sweep33.err; exit 1; }
cat gpurun_out/c27/sweep33.jsonl
bash tools/gpu_r3_call26.sh
