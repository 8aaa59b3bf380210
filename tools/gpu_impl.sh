# Parity of every pairing implementation + one bench line and a rocprof stats pass per implementation.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-impl}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairing.py -x -v --timeout 240 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
for impl in ${IMPLS:-thread_signed thread}; do
  timeout -k 10 300 python -u bench.py --impl $impl --steps 3 --warmup 1 --no-cpu-baseline --no-combine > $O/$impl.json 2> $O/$impl.err || { tail -5 $O/$impl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$impl.json')); print('$impl', round(d['value']), d['roofline']['kernel_ms'], d['verdicts_ok'])"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$impl -o run -- python3 $GRAFT_REPO_ROOT/bench.py --impl $impl --steps 2 --warmup 0 --no-cpu-baseline --no-combine > $GRAFT_REPO_ROOT/$O/prof_$impl.log 2>&1)
done
