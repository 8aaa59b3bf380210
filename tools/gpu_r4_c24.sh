#!/bin/bash
# round 4, call 24: cProfile of the epoch flows (configs[4]) on the octo library, sorted by own time
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c24
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py --workload epoch --steps 6 --warmup 2 --no-cpu-baseline --profile-epoch $O/epoch_prof.txt > $O/epoch.json 2> $O/epoch.err || { tail -5 $O/epoch.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/epoch.json')); print(d['value'], d['host_vs_gpu']['host_ms'], d['host_vs_gpu']['gpu_kernel_ms'], d['phase_ms'])"
echo done
