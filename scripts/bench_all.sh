#!/bin/bash
# Bench lines for C2 (default), C5 and C4 on one box; each run has its own time limit.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
for w in ${WORKLOADS:-c2 c5 c4}; do
  echo "== $w ($(date +%T))"
  timeout -k 10 400 python bench.py --workload $w --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS} > gpurun_out/bench_${TAG}_$w.log 2>&1
  rc=$?
  echo "== $w rc=$rc"
  tail -1 gpurun_out/bench_${TAG}_$w.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
