#!/bin/bash
# round 4: epoch (configs[4]) A/B of the Python flows: the in-tree package vs the copy under
# hbbft_amd/ab/pyold (an earlier commit's hbbft_amd/*.py and bench.py), both on the in-tree library,
# interleaved, REPS reps.  One line per run: variant, epochs/s, ms per epoch, phase_ms.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-epoch_ab}
mkdir -p $O
cd $R
for r in $(seq ${REPS:-3}); do
  for V in new old; do
    if [ $V = new ]; then B=bench.py; else B=hbbft_amd/ab/pyold/bench.py; fi
    HBBFT_HIP_LIB=$R/hbbft_amd/libhbbft_hip.so timeout -k 10 300 python3 -u $B --workload epoch --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline > $O/e_$V.json 2> $O/e_$V.err || { tail -5 $O/e_$V.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e_$V.json')); print('$V', round(d['value'],2), round(d['ms_per_step'],1), {k: round(v,1) for k,v in d.get('phase_ms',{}).items()}, d.get('outputs_ok'))" | tee -a $O/epoch_ab.txt
  done
done
echo done
