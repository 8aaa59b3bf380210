set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread 2>&1 | tee gpurun_out/r01_pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/r01_smoke.log
timeout -k 10 300 python -u bench.py --batch 8192 --steps 2 --warmup 1 --no-cpu-baseline 2>&1 | tee gpurun_out/r01_bench_small.log
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 2>&1 | tee gpurun_out/r01_bench.log
