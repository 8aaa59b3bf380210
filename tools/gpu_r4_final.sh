#!/bin/bash
# round 4 closing evidence (one fresh box): GPU suite, smoke, the four bench lines (default sign line
# = the driver's BENCH), the default bench under rocprofv3 --kernel-trace --stats, separate PMC passes
# (FETCH_SIZE / WRITE_SIZE / SQ counters) per workload for profiles/r04/pmc_traffic.json, and a
# two-stream kernel trace of the sign line (line-table prep overlap).  Every GPU step has its own limit.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-final}
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu_all.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
fi
for W in ${WORKLOADS:-sign decrypt dkg epoch}; do
  timeout -k 10 600 python3 -u bench.py --workload $W > $O/bench_$W.json 2> $O/bench_$W.err || { tail -5 $O/bench_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$W.json')); r=d.get('roofline',{}); print('$W', d['value'], d['unit'], 'ms/step', round(d['ms_per_step'],3), 'frac', round(r.get('frac',0),4))"
done
cd /tmp
B="$R/bench.py --steps 5 --warmup 2"
mkdir -p $O/default_bench
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/default_bench -o run -- python3 $B > $O/default_bench/run.log 2>&1 || { echo "default trace failed"; tail -5 $O/default_bench/run.log; exit 1; }
# PMC passes: name:bench arguments (quad16k / oct8k / wave4k: the mid-size and epoch-size pairing kernels)
for S in ${PMC_SETS:-"sign:--workload sign" "decrypt:--workload decrypt" "dkg:--workload dkg" "quad16k:--workload sign --impl quad --batch 16384" "oct8k:--workload sign --impl oct --batch 8192" "wave4k:--workload sign --impl wave --batch 4096"}; do
  W=${S%%:*}; A=${S#*:}
  P=$O/pmc_$W
  mkdir -p $P
  BW="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-combine --streams 1 $A"
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 $BW > $P/trace.log 2>&1 || { echo "$W trace failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- python3 $BW > $P/fetch.log 2>&1 || { echo "$W fetch failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- python3 $BW > $P/write.log 2>&1 || { echo "$W write failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $P/sq -o run -- python3 $BW > $P/sq.log 2>&1 || { echo "$W sq failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD --output-format csv -d $P/sq2 -o run -- python3 $BW > $P/sq2.log 2>&1 || { echo "$W sq2 failed"; exit 1; }
done
mkdir -p $O/two_stream
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $O/two_stream -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-combine --streams 2 > $O/two_stream/run.log 2>&1 || { echo "two-stream trace failed"; exit 1; }
cd $R
python3 tools/pmc_traffic.py $O/pmc_traffic.json $O/pmc_* > $O/pmc_traffic.txt 2>&1 || true
python3 tools/overlap_report.py $O/two_stream > $O/two_stream/overlap.txt 2>&1 || true
echo done
