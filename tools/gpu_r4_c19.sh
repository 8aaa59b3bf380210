#!/bin/bash
# round 4, call 19: the WAVE / QUAD / PAIR crossover on a finer grid (AUTO's thresholds), SQ counter
# passes of the lane-quad kernel (16,384 checks) and the wave kernel (2,048), and the epoch line's
# kernel mix under rocprofv3 --kernel-trace --stats
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c19
mkdir -p $O
cd $R
for N in 1024 3072 5120 6144 10240 16384 20480 28672 40960; do
  for I in wave quad pair auto; do
    if [ $I = wave ] && [ $N -gt 16384 ]; then continue; fi
    timeout -k 10 200 python3 -u bench.py --workload sign --impl $I --batch $N --steps 3 --warmup 1 --no-cpu-baseline --no-combine > $O/s.json 2> $O/s.err || { tail -5 $O/s.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s.json')); r=d['roofline']; print('batch $N $I kernel %.3f ms' % r['avg_launch_ms'], '%.0f checks/s' % ($N / r['avg_launch_ms'] * 1e3), 'frac %.3f' % r['frac'], d.get('verdicts_ok'))" | tee -a $O/sweep.txt
  done
done
cd /tmp
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
SQ2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD"
for W in "quad16k:--impl quad --batch 16384" "wave2k:--impl wave --batch 2048"; do
  T=${W%%:*}; A=${W#*:}
  B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-combine --streams 1 --workload sign $A"
  mkdir -p $O/$T
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$T/trace -o run -- python3 $B > $O/$T/trace.log 2>&1 || { echo "$T trace failed"; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc $SQ1 --output-format csv -d $O/$T/sq -o run -- python3 $B > $O/$T/sq.log 2>&1 || { echo "$T sq failed"; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc $SQ2 --output-format csv -d $O/$T/sq2 -o run -- python3 $B > $O/$T/sq2.log 2>&1 || { echo "$T sq2 failed"; exit 1; }
done
mkdir -p $O/epoch_trace
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/epoch_trace -o run -- python3 $R/bench.py --workload epoch --steps 8 --warmup 2 --no-cpu-baseline > $O/epoch_trace/run.log 2>&1 || { echo "epoch trace failed"; exit 1; }
echo done
