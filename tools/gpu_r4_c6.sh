#!/bin/bash
# round 4, call 6: epoch (configs[4]) host/GPU split -- pipelined vs serial drains vs the earlier
# flows (hbbft_amd/ab/pyold), with the host_vs_gpu block and a cProfile of the pipelined flows
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c6
mkdir -p $O
cd $R
L=$R/hbbft_amd/libhbbft_hip.so
timeout -k 10 300 python3 -u bench.py --workload epoch --steps 8 --warmup 2 --no-cpu-baseline --profile-epoch $O/epoch_prof.txt > $O/e_prof.json 2> $O/e_prof.err || { tail -5 $O/e_prof.err; exit 1; }
for r in 1 2; do
  for V in new serial old; do
    case $V in
      new) B="bench.py";; serial) B="bench.py --no-pipeline";; old) B="hbbft_amd/ab/pyold/bench.py";;
    esac
    HBBFT_HIP_LIB=$L timeout -k 10 300 python3 -u $B --workload epoch --steps 8 --warmup 2 --no-cpu-baseline > $O/e_$V.json 2> $O/e_$V.err || { tail -5 $O/e_$V.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e_$V.json')); print('$V', round(d['value'],2), round(d['ms_per_step'],1), {k: round(v,1) for k,v in d.get('phase_ms',{}).items()}, json.dumps(d.get('host_vs_gpu')), d.get('checks_drained_per_epoch'), d.get('outputs_ok'))" | tee -a $O/epoch_ab.txt
  done
done
echo done
