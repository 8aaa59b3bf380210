#!/bin/bash
# round 4, call 1: GPU suite at the start of the round + baseline SQ counters (instruction-fetch waits,
# issue) of k_pair_verify (sign, 65,536 checks) and k_wave (4,096-check wave batch)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c1
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1
rc=$?; tail -3 $O/pytest_gpu_all.log; [ $rc -eq 0 ] || exit $rc
fi
cd /tmp
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQ_ACTIVE_INST_VALU"
SQ2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD"
for W in "sign:--workload sign" "wave4k:--workload sign --impl wave --batch 4096"; do
  T=${W%%:*}; A=${W#*:}
  mkdir -p $O/$T
  B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-combine --streams 1 $A"
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$T/trace -o run -- python3 $B > $O/$T/trace.log 2>&1 || { echo "$T trace failed"; tail -5 $O/$T/trace.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $SQ1 --output-format csv -d $O/$T/sq -o run -- python3 $B > $O/$T/sq.log 2>&1 || { echo "$T sq failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $SQ2 --output-format csv -d $O/$T/sq2 -o run -- python3 $B > $O/$T/sq2.log 2>&1 || { echo "$T sq2 failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$T/fetch -o run -- python3 $B > $O/$T/fetch.log 2>&1 || { echo "$T fetch failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$T/write -o run -- python3 $B > $O/$T/write.log 2>&1 || { echo "$T write failed"; exit 1; }
done
echo done
