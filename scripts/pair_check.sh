#!/bin/bash
# Clip-pair loop: its GPU tests, then the C5 bench line (each step under its own time limit).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "pair or per_clip or auto_route" > gpurun_out/pair_pytest.log 2>&1
rc=$?; tail -12 gpurun_out/pair_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pair_c5.log 2>&1
rc=$?; tail -1 gpurun_out/pair_c5.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.loads(open('gpurun_out/pair_c5.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_us'])"
