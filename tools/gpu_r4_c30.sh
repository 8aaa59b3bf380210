#!/bin/bash
# round 4, call 30: decryption-share pre-verification started with the epoch vs after the first coin drain
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c30
mkdir -p $O
cd $R
for r in 1 2 3; do
  for A in first_drain start; do
    timeout -k 10 300 python3 -u bench.py --workload epoch --preverify-at $A --no-cpu-baseline > $O/e.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e.json')); h=d['host_vs_gpu']; p=d['phase_ms']; print('$A epoch %.2f/s' % d['value'], 'ms %.1f host %.1f gpu %.1f' % (d['ms_per_step'], h['host_ms'], h['gpu_kernel_ms']), {k: round(v, 1) for k, v in p.items() if k.startswith('decrypt') or k in ('coin_verify', 'epoch')}, d['outputs_ok'])" | tee -a $O/pre_at.txt
  done
done
echo done
