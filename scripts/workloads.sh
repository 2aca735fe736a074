#!/bin/bash
# Bench lines for the BASELINE.json workloads other than the default C2 (c4 long clip, c5 DDIM-50).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
for w in ${WORKLOADS:-c5 c4}; do
  echo "== $w ($(date +%T))"
  timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 ${BENCH_ARGS} > gpurun_out/bench_${TAG}_$w.log 2>&1
  rc=$?
  echo "== $w rc=$rc"
  tail -3 gpurun_out/bench_${TAG}_$w.log
  [ $rc -eq 0 ] || exit $rc
done
