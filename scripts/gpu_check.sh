#!/bin/bash
# One GPU session: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel stats of the bench.
# Every GPU step has its own time limit; a fault / abort / timeout ends the script.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  return $rc
}
MODE=${1:-all}
step smoke 300 python __graft_entry__.py smoke || exit $?
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
  rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py --steps 3 --warmup 1 || exit $?
  cat gpurun_out/bench.log | tail -1 > gpurun_out/bench.json
  step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline || exit $?
fi
echo done
