#!/bin/bash
# round 4, call 13: epoch at the 8,192-message window, serial vs pipelined (combines on a second engine)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c13
mkdir -p $O
cd $R
for V in serial pipelined serial pipelined; do
  case $V in serial) A="";; pipelined) A="--pipeline";; esac
  timeout -k 10 300 python3 -u bench.py --workload epoch --steps 8 --warmup 2 --no-cpu-baseline $A > $O/e_$V.json 2> $O/e_$V.err || { tail -5 $O/e_$V.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e_$V.json')); h=d.get('host_vs_gpu'); print('$V', round(d['value'],2), round(d['ms_per_step'],1), {k: round(v,1) for k,v in d.get('phase_ms',{}).items()}, 'blocked', {k: round(v,1) for k,v in h['blocked_by_phase_ms'].items()}, 'gpu', round(h['gpu_kernel_ms'],1), 'host', round(h['host_ms'],1), h.get('pipelined_ms'), d.get('outputs_ok'))" | tee -a $O/epoch_ab.txt
done
timeout -k 10 300 python3 -u bench.py --workload epoch --steps 8 --warmup 2 --no-cpu-baseline --profile-epoch $O/epoch_prof.txt > $O/e_prof.json 2> $O/e_prof.err || { tail -5 $O/e_prof.err; exit 1; }
echo done
