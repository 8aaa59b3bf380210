#!/bin/bash
# round 4, call 9: the whole GPU suite (the lane-quad kernel at full size and at the AUTO
# boundaries), then the epoch serial vs pipelined with the pipelining instrumentation
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c9
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1 || { tail -30 $O/pytest_gpu_all.log; exit 1; }
tail -2 $O/pytest_gpu_all.log
for V in serial pipelined serial pipelined; do
  case $V in serial) A="";; pipelined) A="--pipeline";; esac
  timeout -k 10 300 python3 -u bench.py --workload epoch --steps 8 --warmup 2 --no-cpu-baseline $A > $O/e_$V.json 2> $O/e_$V.err || { tail -5 $O/e_$V.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e_$V.json')); print('$V', round(d['value'],2), round(d['ms_per_step'],1), {k: round(v,1) for k,v in d.get('phase_ms',{}).items()}, json.dumps(d.get('host_vs_gpu')), d.get('checks_drained_per_epoch'), d.get('outputs_ok'))" | tee -a $O/epoch_ab.txt
done
echo done
