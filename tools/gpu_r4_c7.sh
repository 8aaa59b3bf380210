#!/bin/bash
# round 4, call 7: epoch (configs[4]) with serial drains + next-epoch coin prefetch (default) vs
# without the prefetch; the epoch / BA / wire GPU tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c7
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_honey_badger.py tests/test_gpu_binary_agreement.py tests/test_gpu_wire_msgs.py tests/test_gpu_protocol.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do
  for V in default noprefetch; do
    case $V in default) A="";; noprefetch) A="--no-prefetch";; esac
    timeout -k 10 300 python3 -u bench.py --workload epoch --steps 8 --warmup 2 --no-cpu-baseline $A > $O/e_$V.json 2> $O/e_$V.err || { tail -5 $O/e_$V.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e_$V.json')); print('$V', round(d['value'],2), round(d['ms_per_step'],1), {k: round(v,1) for k,v in d.get('phase_ms',{}).items()}, json.dumps(d.get('host_vs_gpu')), d.get('checks_drained_per_epoch'), d.get('outputs_ok'))" | tee -a $O/epoch_ab.txt
  done
done
timeout -k 10 300 python3 -u bench.py --workload epoch --steps 8 --warmup 2 --no-cpu-baseline --profile-epoch $O/epoch_prof.txt > $O/e_prof.json 2> $O/e_prof.err || { tail -5 $O/e_prof.err; exit 1; }
echo done
