#!/bin/bash
# round 4, call 18: scheduler variants -- k_wave under iterative-ilp / max-ilp (ab/witilp.so,
# ab/wmaxilp.so) at 2,048 / 4,096 checks, and k_pair_verify without the minreg scheduler
# (ab/pdef.so) or under iterative-ilp (ab/pitilp.so) on the sign line, vs the in-tree build
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c18
mkdir -p $O
cd $R
for r in 1 2; do
  for N in 2048 4096; do
    for L in "" hbbft_amd/ab/witilp.so hbbft_amd/ab/wmaxilp.so; do
      HBBFT_HIP_LIB=${L:+$R/$L} timeout -k 10 200 python3 -u bench.py --workload sign --impl wave --batch $N --steps 3 --warmup 1 --no-cpu-baseline --no-combine > $O/w.json 2> $O/w.err || { tail -5 $O/w.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/w.json')); r=d['roofline']; print('wave $N', '${L:-intree}', 'kernel %.3f ms' % r['avg_launch_ms'], d.get('verdicts_ok'))" | tee -a $O/ab.txt
    done
  done
  for L in "" hbbft_amd/ab/pdef.so hbbft_amd/ab/pitilp.so; do
    HBBFT_HIP_LIB=${L:+$R/$L} timeout -k 10 300 python3 -u bench.py --workload sign --steps 5 --warmup 2 --no-cpu-baseline --no-combine > $O/s.json 2> $O/s.err || { tail -5 $O/s.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s.json')); r=d['roofline']; print('sign', '${L:-intree}', round(d['value']), round(d['ms_per_step'],3), 'kernel %.3f' % r['avg_launch_ms'], 'frac %.4f' % r['frac'], d.get('verdicts_ok'))" | tee -a $O/ab.txt
  done
done
echo done
