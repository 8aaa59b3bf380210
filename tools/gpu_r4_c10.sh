#!/bin/bash
# round 4, call 10: (1) dkg ack check in (tile, y) order (in-tree) vs y order (ab/tower.so) + the
# in-tree dkg FETCH/WRITE passes; (2) the lane-quad kernel at one vs two waves per SIMD (ab/quad2.so)
# at 16,384-32,768 checks; (3) the epoch with pipelined drains and combines on a second engine
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c10
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sync_key_gen.py tests/test_gpu_commit_set.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for L in "" hbbft_amd/ab/tower.so; do
    HBBFT_HIP_LIB=${L:+$R/$L} timeout -k 10 300 python3 -u bench.py --workload dkg --steps 3 --warmup 1 --no-cpu-baseline > $O/dkg.json 2> $O/dkg.err || { tail -5 $O/dkg.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/dkg.json')); r=d['roofline']; print('dkg', '${L:-intree}', round(d['value']), round(d['ms_per_step'],3), round(r['avg_launch_ms'],3), round(r['frac'],4), d.get('verdicts_ok', d.get('outputs_ok')))" | tee -a $O/ab.txt
  done
done
cd /tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-combine --streams 1 --workload dkg"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $O/pmc_dkg/$C -o run -- python3 $B > $O/pmc_dkg_$C.log 2>&1 || { echo "$C failed"; exit 1; }
done
cd $R
for N in 16384 24576 32768; do
  for L in "" hbbft_amd/ab/quad2.so; do
    HBBFT_HIP_LIB=${L:+$R/$L} timeout -k 10 200 python3 -u bench.py --workload sign --impl quad --batch $N --steps 3 --warmup 1 --no-cpu-baseline --no-combine > $O/q.json 2> $O/q.err || { tail -5 $O/q.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/q.json')); r=d['roofline']; print('quad $N', '${L:-intree}', 'kernel %.3f ms' % r['avg_launch_ms'], 'frac %.3f' % r['frac'], d.get('verdicts_ok'))" | tee -a $O/ab.txt
  done
done
for V in serial pipelined serial pipelined; do
  case $V in serial) A="";; pipelined) A="--pipeline";; esac
  timeout -k 10 300 python3 -u bench.py --workload epoch --steps 8 --warmup 2 --no-cpu-baseline $A > $O/e_$V.json 2> $O/e_$V.err || { tail -5 $O/e_$V.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e_$V.json')); h=d.get('host_vs_gpu'); print('$V', round(d['value'],2), round(d['ms_per_step'],1), {k: round(v,1) for k,v in d.get('phase_ms',{}).items()}, 'blocked', {k: round(v,1) for k,v in h['blocked_by_phase_ms'].items()}, 'gpu', round(h['gpu_kernel_ms'],1), 'host', round(h['host_ms'],1), h.get('pipelined_ms'), d.get('outputs_ok'))" | tee -a $O/epoch_ab.txt
done
echo done
