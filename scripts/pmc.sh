#!/bin/bash
# PMC counter passes (each its own run; --pmc only beside --kernel-trace / --stats).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
shift
i=0
for CTRS in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTRS -d gpurun_out/${TAG}_$i -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-profile --steps 1 --warmup 1 --respacing 25 > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i ($CTRS) rc=$rc"
  [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_$i.log; exit $rc; }
done
