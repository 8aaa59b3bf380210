#!/bin/bash
# round 4, call 34: preverify ciphertext checks merged into the share-check call --
# the GPU suite, then the epoch line x3
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c34
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --workload epoch --no-cpu-baseline > $O/e.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e.json')); h=d['host_vs_gpu']; p=d['phase_ms']; print('epoch %.2f/s' % d['value'], 'ms %.1f host %.1f gpu %.1f' % (d['ms_per_step'], h['host_ms'], h['gpu_kernel_ms']), {k: round(v, 1) for k, v in p.items() if k.startswith('decrypt') or k in ('coin_verify', 'epoch')}, d['outputs_ok'])" | tee -a $O/epoch.txt
done
echo done
