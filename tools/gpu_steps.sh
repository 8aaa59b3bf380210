#!/bin/bash
# One parameterised GPU-box script (replaces the per-call gpu_r*_c*.sh of rounds 2-5).
#   tools/gpu_steps.sh OUT STEP [STEP ...]      (run via gpurun from the repo root)
# Each STEP is NAME=SPEC and runs under its own time limit; the first failing step ends the call
# (no GPU work after a fault, abort or time-limit kill).  Output goes to gpurun_out/OUT/NAME.*
#   test:NAME=<pytest args>            python -u -m pytest -x -v --timeout 120 ...
#   bench:NAME=<bench.py args>         stdout -> NAME.json, stderr -> NAME.err
#   trace:NAME=<script args>           rocprofv3 --kernel-trace --stats -> NAME/ (+ stats csv copy);
#                                      script relative to the repo root (bench.py, tools/x.py)
#   pmc:NAME=<counters>|<script args>  one rocprofv3 --pmc pass (counters space-separated)
#   py:NAME=<python args>              any python tool (tools/*.py), stdout -> NAME.txt
#   smoke:NAME=                        __graft_entry__.smoke()
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/$1"
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
step_limit=${STEP_LIMIT:-300}
for st in "$@"; do
  kind="${st%%:*}"
  rest="${st#*:}"
  name="${rest%%=*}"
  spec="${rest#*=}"
  echo "== $(date +%T) $kind $name: $spec" | tee -a "$OUT/steps.txt"
  case "$kind" in
    test)
      (cd "$ROOT" && timeout -k 10 "$step_limit" python -u -m pytest -x -v --timeout 120 --timeout-method thread \
        $spec > "$OUT/$name.log" 2>&1)
      rc=$?; tail -3 "$OUT/$name.log" | tee -a "$OUT/steps.txt" ;;
    bench)
      (cd "$ROOT" && timeout -k 10 "$step_limit" python -u bench.py $spec > "$OUT/$name.json" 2> "$OUT/$name.err")
      rc=$?; tail -c 600 "$OUT/$name.json" | tee -a "$OUT/steps.txt" ;;
    trace)
      (cd /tmp && timeout -k 10 "$step_limit" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- \
        python3 $ROOT/$spec > "$OUT/$name.json" 2> "$OUT/$name.err")
      rc=$?
      f=$(find "$OUT/$name" -name "*kernel_stats.csv" | head -1)
      [ -n "$f" ] && cp "$f" "$OUT/$name.kernel_stats.csv" && head -12 "$f" | cut -c1-160 | tee -a "$OUT/steps.txt" ;;
    pmc)
      ctr="${spec%%|*}"
      args="${spec#*|}"
      (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$OUT/$name" -o run -- \
        python3 $ROOT/$args > "$OUT/$name.json" 2> "$OUT/$name.err")
      rc=$?
      f=$(find "$OUT/$name" -name "*counter_collection.csv" | head -1)
      [ -n "$f" ] && cp "$f" "$OUT/$name.counters.csv" ;;
    py)
      (cd "$ROOT" && timeout -k 10 "$step_limit" python -u $spec > "$OUT/$name.txt" 2>&1)
      rc=$?; tail -5 "$OUT/$name.txt" | tee -a "$OUT/steps.txt" ;;
    smoke)
      (cd "$ROOT" && timeout -k 10 "$step_limit" python -u -c "import __graft_entry__ as g; g.smoke()" \
        > "$OUT/$name.log" 2>&1)
      rc=$?; tail -2 "$OUT/$name.log" | tee -a "$OUT/steps.txt" ;;
    *) echo "unknown step kind $kind"; exit 2 ;;
  esac
  echo "== rc=$rc" | tee -a "$OUT/steps.txt"
  if [ $rc -ne 0 ]; then
    exit $rc
  fi
done
