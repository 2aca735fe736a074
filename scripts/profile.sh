#!/bin/bash
# rocprofv3 kernel statistics of a short bench run (kernel-trace + stats only, no PMC).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
shift
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -3 gpurun_out/prof_$TAG.log
f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && head -30 "$f"
exit $rc
