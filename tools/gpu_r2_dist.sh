#!/bin/bash
# rehearsal of the driver's multi-GPU launch (torchrun, one rank per GPU) with 2 ranks sharing the
# box's one GPU: gloo for the barrier / max-over-ranks (HBH_DIST_BACKEND), every line of bench.py
set -o pipefail
mkdir -p gpurun_out/dist
export HBH_DIST_BACKEND=gloo
P=29611
for w in sign decrypt dkg epoch; do
  P=$((P+1))
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $P bench.py --gpus 2 --steps 3 --warmup 1 --workload $w --no-cpu-baseline > gpurun_out/dist/$w.json 2> gpurun_out/dist/$w.err || { echo "dist $w failed"; tail -20 gpurun_out/dist/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/dist/$w.json')); print('$w', d['n_gpus'], d['value'], d['ms_per_step'], d.get('verdicts_ok', d.get('outputs_ok')))"
done
