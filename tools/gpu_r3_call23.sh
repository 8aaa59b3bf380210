#!/bin/bash
# round 3 final profiles: WAVE/PAIR crossover with the CYC-run k_wave, rocprof kernel traces of the sign
# bench line and of the combine-latency probe
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c23
rm -f gpurun_out/crossover_r3.txt
bash tools/gpu_r3_crossover.sh || exit 1
cp gpurun_out/crossover_r3.txt gpurun_out/c23/crossover.txt
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c23/sign -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/c23/sign_bench.json 2> $R/gpurun_out/c23/sign_bench.err || { echo sign trace failed; tail $R/gpurun_out/c23/sign_bench.err; exit 1; }
cut -c1-200 $R/gpurun_out/c23/sign/run_kernel_stats.csv | head -12
cd /tmp && PROBE_REPS=9 timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c23/combine -o run -- python3 $R/tools/probe_split.py > $R/gpurun_out/c23/combine_probe.json 2> $R/gpurun_out/c23/combine_probe.err || { echo combine trace failed; exit 1; }
cut -c1-200 $R/gpurun_out/c23/combine/run_kernel_stats.csv | head -12
