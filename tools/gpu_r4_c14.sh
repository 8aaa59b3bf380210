#!/bin/bash
# round 4, call 14: decryption-share pre-verification beside the coin phase (default) vs none;
# the epoch / BA / wire GPU tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c14
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_honey_badger.py tests/test_gpu_binary_agreement.py tests/test_gpu_wire_msgs.py tests/test_gpu_protocol.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for V in preverify none; do
    case $V in preverify) A="";; none) A="--no-preverify";; esac
    timeout -k 10 300 python3 -u bench.py --workload epoch --steps 8 --warmup 2 --no-cpu-baseline $A > $O/e_$V.json 2> $O/e_$V.err || { tail -5 $O/e_$V.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e_$V.json')); h=d.get('host_vs_gpu'); print('$V', round(d['value'],2), round(d['ms_per_step'],1), {k: round(v,1) for k,v in d.get('phase_ms',{}).items()}, 'blocked', {k: round(v,1) for k,v in h['blocked_by_phase_ms'].items()}, 'gpu', round(h['gpu_kernel_ms'],1), 'host', round(h['host_ms'],1), 'drained', d['checks_drained_per_epoch'], d.get('outputs_ok'))" | tee -a $O/epoch_ab.txt
  done
done
echo done
