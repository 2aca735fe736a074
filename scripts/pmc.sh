#!/bin/bash
# PMC counter passes over a bench run (each pass its own rocprofv3 run: --pmc beside --kernel-trace only),
# summarised per dispatch of the dominant kernel by scripts/pmc_summary.py.
#   bash scripts/pmc.sh TAG "COUNTERS PASS 1" "COUNTERS PASS 2" ...      (BENCH_ARGS: extra bench.py args)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
shift
i=0
for CTRS in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d gpurun_out/${TAG}_$i -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-profile --steps 1 --warmup 1 ${BENCH_ARGS} > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i ($CTRS) rc=$rc"
  [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_$i.log; exit $rc; }
done
python3 scripts/pmc_summary.py gpurun_out ${TAG} ${WORKLOAD} > gpurun_out/${TAG}_summary.json && cat gpurun_out/${TAG}_summary.json
