#!/bin/bash
# C4 evidence for one tag: bench line, rocprofv3 kernel stats, HBM-traffic PMC passes (FETCH_SIZE and
# WRITE_SIZE each in its own run, beside --kernel-trace only).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02k}
timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/${TAG}_c4_bench.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_c4_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c4prof -o run --output-format csv -- \
  python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c4prof.log 2>&1 || exit 1
BENCH_ARGS="--workload c4" bash scripts/pmc.sh ${TAG}_pmc_c4 "FETCH_SIZE" "WRITE_SIZE" > gpurun_out/${TAG}_pmc.log 2>&1 || { tail -5 gpurun_out/${TAG}_pmc.log; exit 1; }
echo pmc done
