#!/bin/bash
# round 4, call 16: k_bivar_check occupancy -- 1 (255 VGPRs, in-tree), 3 (168 VGPRs, ab/bv3.so) and
# 4 (128 VGPRs, ab/bv4.so) waves per SIMD on configs[3] (10^6 acks), interleaved, 3 reps
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c16
mkdir -p $O
cd $R
timeout -k 10 300 env HBBFT_HIP_LIB=$R/hbbft_amd/ab/bv4.so python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_commit_set.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for L in "" hbbft_amd/ab/bv3.so hbbft_amd/ab/bv4.so; do
    HBBFT_HIP_LIB=${L:+$R/$L} timeout -k 10 300 python3 -u bench.py --workload dkg --steps 3 --warmup 1 --no-cpu-baseline > $O/dkg.json 2> $O/dkg.err || { tail -5 $O/dkg.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/dkg.json')); r=d['roofline']; print('dkg', '${L:-intree}', round(d['value']), round(d['ms_per_step'],3), round(r['avg_launch_ms'],3), round(r['frac'],4), d.get('verdicts_ok', d.get('outputs_ok')))" | tee -a $O/ab.txt
  done
done
echo done
