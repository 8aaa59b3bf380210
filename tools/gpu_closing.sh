#!/bin/bash
# Round-6 closing evidence on one fresh box (the round-5 final_a / final_b pair in one script).
#   PART=a: GPU suite + smoke, then separate rocprofv3 passes per workload (kernel trace, FETCH_SIZE,
#           WRITE_SIZE, one SQ set) -> pmc_traffic.json (becomes profiles/r06/pmc_traffic.json, which
#           the bench lines cite with the same library).
#   PART=b: the bench lines (sign = the driver's BENCH, sign from wire bytes, decrypt, dkg, epoch,
#           epoch from raw bytes), the check-latency sweep, the decoders, the default bench's trace.
# Each GPU step has its own time limit and the first failure ends the call.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-closing}
mkdir -p $O
cd $R
sha256sum hbbft_amd/libhbbft_hip.so > $O/lib_sha256.txt
if [ "${PART:-a}" = "a" ]; then
  if [ -z "$SKIP_TESTS" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1
    rc=$?; tail -3 $O/pytest_gpu_all.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
    tail -2 $O/smoke.log
  fi
  cd /tmp
  for S in ${PMC_SETS:-"sign:--workload sign" "wire:--workload sign --from-wire" "decrypt:--workload decrypt" "dkg:--workload dkg --no-node-round" "oct8k:--workload sign --impl oct --batch 8192" "wave4k:--workload sign --impl wave --batch 4096" "wave2_512:--workload sign --impl wave2 --batch 512"}; do
    W=${S%%:*}; A=${S#*:}
    P=$O/pmc_$W
    mkdir -p $P
    BW="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-combine --no-wire --streams 1 $A"
    timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 $BW > $P/trace.log 2>&1 || { echo "$W trace failed"; exit 1; }
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- python3 $BW > $P/fetch.log 2>&1 || { echo "$W fetch failed"; exit 1; }
    timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- python3 $BW > $P/write.log 2>&1 || { echo "$W write failed"; exit 1; }
    timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $P/sq -o run -- python3 $BW > $P/sq.log 2>&1 || { echo "$W sq failed"; exit 1; }
    echo "pmc $W done"
  done
  cd $R
  python3 tools/pmc_traffic.py $O/pmc_traffic.json $O/pmc_* > $O/pmc_traffic.txt 2>&1 || { tail -5 $O/pmc_traffic.txt; exit 1; }
  for d in $O/pmc_*/; do python3 tools/pmc_summary.py $d > $d/summary.txt; done
  tail -12 $O/pmc_traffic.txt
else
  for S in ${LINES:-"sign:" "sign_wire:--from-wire" "decrypt:--workload decrypt" "dkg:--workload dkg" "epoch:--workload epoch" "epoch_raw:--workload epoch --raw"}; do
    W=${S%%:*}; A=${S#*:}
    timeout -k 10 600 python3 -u bench.py $A > $O/bench_$W.json 2> $O/bench_$W.err || { tail -5 $O/bench_$W.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_$W.json')); r=d.get('roofline',{}); print('$W', round(d['value'],1), d['unit'], 'ms/step', round(d['ms_per_step'],3), 'frac', round(r.get('frac',0),4), 'match', (r.get('traffic_source') or {}).get('matches_loaded_lib'))"
  done
  timeout -k 10 300 python3 -u tools/latency_probe.py 1 64 256 512 1024 2048 4096 > $O/latency.txt 2>&1 || { tail -5 $O/latency.txt; exit 1; }
  cat $O/latency.txt
  timeout -k 10 300 python3 -u tools/decode_bench.py 65536 5 > $O/decode_65536.txt 2>&1 || { tail -5 $O/decode_65536.txt; exit 1; }
  timeout -k 10 300 python3 -u tools/decode_bench.py 4096 5 > $O/decode_4096.txt 2>&1 || { tail -5 $O/decode_4096.txt; exit 1; }
  tail -1 $O/decode_65536.txt
  cd /tmp
  mkdir -p $O/default_bench
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/default_bench -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $O/default_bench/run.log 2>&1 || { echo "default trace failed"; tail -5 $O/default_bench/run.log; exit 1; }
  head -8 $O/default_bench/run_kernel_stats.csv | cut -c1-150
fi
echo done
