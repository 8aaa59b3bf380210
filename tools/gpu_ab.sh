# A/B: bench the pairing kernels of several in-tree builds (HBBFT_HIP_LIB) + a rocprof stats pass of each
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}
mkdir -p $O
for lib in hbbft_amd/ab/*.so; do
  tag=$(basename $lib .so)
  HBBFT_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-combine $BENCH_ARGS > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/$tag.json')); print('$tag', round(d['value']), d['roofline']['kernel_ms'], d['verdicts_ok'])"
  (cd /tmp && HBBFT_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$tag -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-combine $BENCH_ARGS > $GRAFT_REPO_ROOT/$O/prof_$tag.log 2>&1)
done
