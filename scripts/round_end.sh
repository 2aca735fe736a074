#!/bin/bash
# Round-end evidence on one box: GPU suite, smoke, C4 evidence (bench, kernel stats, PMC), default bench.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02m}
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
echo smoke ok
TAG=$TAG bash scripts/c4_profile.sh || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_c2_bench.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_c2_bench.log | cut -c1-200
