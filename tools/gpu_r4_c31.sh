#!/bin/bash
# round 4, call 31: next-epoch coin prefetch after the decryption prep (default) vs beside it (--prefetch-early)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c31
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_honey_badger.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for A in "" "--prefetch-early" "--preverify-at start"; do
    timeout -k 10 300 python3 -u bench.py --workload epoch $A --no-cpu-baseline > $O/e.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e.json')); h=d['host_vs_gpu']; p=d['phase_ms']; print('[$A] epoch %.2f/s' % d['value'], 'ms %.1f host %.1f gpu %.1f' % (d['ms_per_step'], h['host_ms'], h['gpu_kernel_ms']), {k: round(v, 1) for k, v in p.items() if k.startswith('decrypt_pre') or k in ('coin_verify', 'epoch')}, d['outputs_ok'])" | tee -a $O/prefetch_order.txt
  done
done
echo done
