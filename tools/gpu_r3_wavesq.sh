#!/bin/bash
# round 3: k_wave's square on WV_NACC accumulator chains (in-tree) vs one chain (hbbft_amd/ab/sq1.so):
# WAVE parity tests on the in-tree library, then single-check wave-kernel time, interleaved, and the
# combine latency of the sign bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pairing.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_wavesq_tests.log 2>&1 || { tail -30 gpurun_out/r3_wavesq_tests.log; exit 1; }
tail -1 gpurun_out/r3_wavesq_tests.log
for r in 1 2 3; do
  for L in "" hbbft_amd/ab/sq1.so; do
    HBBFT_HIP_LIB=${L:+$PWD/$L} timeout -k 10 120 python -u tools/wave_time.py || exit 1
  done
done
for L in "" hbbft_amd/ab/sq1.so; do
  HBBFT_HIP_LIB=${L:+$PWD/$L} timeout -k 10 300 python3 -u bench.py --workload sign --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wsq.json 2> gpurun_out/wsq.err || { tail -5 gpurun_out/wsq.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/wsq.json')); print('${L:-intree}', 'combine_latency_ms', d.get('combine_latency_ms'), {k: v for k, v in d.items() if 'combine' in k and k != 'combine_latency_ms'})"
done
