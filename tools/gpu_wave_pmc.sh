#!/bin/bash
# PMC passes of the wave kernel on single-check calls -> gpurun_out/wpmc/
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wpmc
mkdir -p $O
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/wave_one.py > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $O/sq -o run -- python3 $R/tools/wave_one.py > $O/sq.log 2>&1 || { echo sq failed; tail $O/sq.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT --output-format csv -d $O/sq2 -o run -- python3 $R/tools/wave_one.py > $O/sq2.log 2>&1 || { echo sq2 failed; tail $O/sq2.log; exit 1; }
grep -h k_wave $O/sq/*counter_collection.csv $O/sq2/*counter_collection.csv | tail -40
