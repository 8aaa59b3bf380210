#!/bin/bash
# round 4, call 11: ack order for the one-lane ack check (configs[3], 10^6 acks): y order (tile 0)
# vs (tile, y) order for tiles of 64-1,024 row slots (HBH_ACK_TILE_AB, A/B knob); FETCH/WRITE per tile
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c11
mkdir -p $O
cd $R
for r in 1 2; do
  for T in 0 64 256 512 1024 4096; do
    HBH_ACK_TILE_AB=$T timeout -k 10 300 python3 -u bench.py --workload dkg --steps 3 --warmup 1 --no-cpu-baseline > $O/dkg.json 2> $O/dkg.err || { tail -5 $O/dkg.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/dkg.json')); r=d['roofline']; print('dkg tile $T', round(d['value']), round(d['ms_per_step'],3), round(r['avg_launch_ms'],3), round(r['frac'],4), d.get('verdicts_ok', d.get('outputs_ok')))" | tee -a $O/ab.txt
  done
done
cd /tmp
for T in 0 256 1024; do
  B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-combine --streams 1 --workload dkg"
  for C in FETCH_SIZE WRITE_SIZE; do
    HBH_ACK_TILE_AB=$T timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $O/pmc_t$T/$C -o run -- python3 $B > $O/pmc_t${T}_$C.log 2>&1 || { echo "$C failed"; exit 1; }
  done
done
echo done
