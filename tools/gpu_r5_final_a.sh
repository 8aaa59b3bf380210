#!/bin/bash
# round 5 closing evidence, part A (one fresh box): the GPU suite, smoke, and separate PMC passes
# (FETCH_SIZE / WRITE_SIZE / two SQ sets) per workload -> pmc_traffic.json (becomes
# profiles/r05/pmc_traffic.json, which part B's bench lines then cite with the same library).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-final_a}
mkdir -p $O
cd $R
sha256sum hbbft_amd/libhbbft_hip.so > $O/lib_sha256.txt
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu_all.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
fi
cd /tmp
for S in ${PMC_SETS:-"sign:--workload sign" "decrypt:--workload decrypt" "dkg:--workload dkg --no-node-round" "oct8k:--workload sign --impl oct --batch 8192" "wave4k:--workload sign --impl wave --batch 4096"}; do
  W=${S%%:*}; A=${S#*:}
  P=$O/pmc_$W
  mkdir -p $P
  BW="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-combine --streams 1 $A"
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 $BW > $P/trace.log 2>&1 || { echo "$W trace failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- python3 $BW > $P/fetch.log 2>&1 || { echo "$W fetch failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- python3 $BW > $P/write.log 2>&1 || { echo "$W write failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $P/sq -o run -- python3 $BW > $P/sq.log 2>&1 || { echo "$W sq failed"; exit 1; }
  echo "pmc $W done"
done
cd $R
python3 tools/pmc_traffic.py $O/pmc_traffic.json $O/pmc_* > $O/pmc_traffic.txt 2>&1 || { tail -5 $O/pmc_traffic.txt; exit 1; }
tail -12 $O/pmc_traffic.txt
