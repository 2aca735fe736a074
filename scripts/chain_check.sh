#!/bin/bash
# Row-block chain route: parity tests, a kernel-trace of C4-shape denoise calls, the C4 bench line.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-chain}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "chain or fp8 or long_clip or clip_attention or long_loop" > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_pytest.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
  python3 scripts/chain_probe.py ${PROBE_ARGS} > gpurun_out/${TAG}_probe.log 2>&1 || { tail -20 gpurun_out/${TAG}_probe.log; exit 1; }
python3 - "$TAG" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/{tag}_prof/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "chain_kernel" in r["Kernel_Name"] or "attn_q" in r["Kernel_Name"]]
d = [(r["Kernel_Name"][:40], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
print([round(x[1], 1) for x in d[-20:]])
PY
[ -n "$NO_BENCH" ] && exit 0
WORKLOADS=c4 TAG=${TAG} bash scripts/bench_all.sh
