#!/bin/bash
# round 5 call 9: split check with the Miller-value product tree and the FE in the Miller launch --
# combine parity (tree / no tree / unsplit), combine latency A/B and its kernel anatomy
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-c9}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_curve.py tests/test_gpu_pairing.py tests/test_gpu_ba_network.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for T in 1 0 1; do
  HBH_SPLIT_TREE=$T timeout -k 10 300 python3 -u tools/combine_trace.py --reps 30 > $O/combine_tree$T.txt 2>&1 || { tail -5 $O/combine_tree$T.txt; exit 1; }
  echo "tree=$T $(tail -1 $O/combine_tree$T.txt | sed 's/.*median/median/')"
done
cd /tmp
mkdir -p $O/trace
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/combine_trace.py --reps 20 > $O/trace/run.log 2>&1 || { echo "combine trace failed"; tail -5 $O/trace/run.log; exit 1; }
python3 $R/tools/combine_trace.py --trace $O/trace > $O/anatomy.txt; sed -n 14,40p $O/anatomy.txt
