# PMC passes (one counter group per run) over a short bench run: HBM traffic + SQ issue counters.
# usage: BENCH_ARGS="--impl thread_signed" bash tools/gpu_pmc.sh <outdir>
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc}
mkdir -p $O
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-combine $BENCH_ARGS"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/fetch -o run -- python3 $B > $R/$O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/write -o run -- python3 $B > $R/$O/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU --output-format csv -d $R/$O/sq -o run -- python3 $B > $R/$O/sq.log 2>&1
echo pmc done
