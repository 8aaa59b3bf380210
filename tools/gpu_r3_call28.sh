#!/bin/bash
# round 3: split-check wave rule -- GPU suite, sweep (split / unsplit / AUTO rule), sign + epoch bench lines
set -o pipefail
mkdir -p gpurun_out/c28
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/c28/pytest_gpu_all.log 2>&1
rc=$?
tail -3 gpurun_out/c28/pytest_gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c28/smoke.log 2>&1 || { tail gpurun_out/c28/smoke.log; exit 1; }
timeout -k 10 240 python3 -u tools/probe_split_sweep.py 21 1 8 16 32 48 64 > gpurun_out/c28/sweep21.jsonl 2> gpurun_out/c28/sweep21.err || { tail -5 gpurun_out/c28/sweep21.err; exit 1; }
cat gpurun_out/c28/sweep21.jsonl
timeout -k 10 300 python3 -u tools/probe_split_sweep.py 33 16 33 40 50 > gpurun_out/c28/sweep33.jsonl 2> gpurun_out/c28/sweep33.err || { tail -5 gpurun_out/c28/sweep33.err; exit 1; }
cat gpurun_out/c28/sweep33.jsonl
bash tools/gpu_r3_bench_all.sh epoch sign epoch
