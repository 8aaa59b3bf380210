#!/bin/bash
# round 4: A/B of bench lines over the in-tree library and hbbft_amd/ab/*.so (interleaved, REPS reps),
# then (PROF=1) a kernel trace + SQ counter pass of the in-tree sign line.  One line per run:
# workload, lib, value, pairing-stage ms per launch, frac, verdicts_ok.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-ab}
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq ${REPS:-2}); do
  for W in ${WORKLOADS:-sign}; do
    for L in "" hbbft_amd/ab/*.so; do
      HBBFT_HIP_LIB=${L:+$PWD/$L} timeout -k 10 300 python3 -u bench.py --workload $W --steps 5 --warmup 2 --no-cpu-baseline --no-combine > $O/ab_$W.json 2> $O/ab_$W.err || { tail -5 $O/ab_$W.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/ab_$W.json')); r=d['roofline']; print('$W', '${L:-intree}', round(d['value']), round(d['ms_per_step'],3), round(r['avg_launch_ms'],3), round(r['frac'],4), d.get('verdicts_ok'))" | tee -a $O/ab.txt
    done
  done
done
for PL in $PROF; do
  [ "$PL" = "1" ] || [ "$PL" = "intree" ] && export -n HBBFT_HIP_LIB || export HBBFT_HIP_LIB=$R/hbbft_amd/ab/$PL.so
  cd /tmp
  B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-combine --streams 1 --workload ${PROF_W:-sign}"
  P=$O/prof_$PL
  mkdir -p $P
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 $B > $P/trace.log 2>&1 || { echo "trace failed"; tail -5 $P/trace.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $P/sq -o run -- python3 $B > $P/sq.log 2>&1 || { echo "sq failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $P/icache -o run -- python3 $B > $P/icache.log 2>&1 || { echo "icache failed"; tail -3 $P/icache.log; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- python3 $B > $P/fetch.log 2>&1 || { echo "fetch failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- python3 $B > $P/write.log 2>&1 || { echo "write failed"; exit 1; }
  cd $R
done
unset HBBFT_HIP_LIB
echo done
