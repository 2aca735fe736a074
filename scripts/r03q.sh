set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03q}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_tr -o run --output-format csv -- python3 scripts/qsplit_probe.py > gpurun_out/${T}.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/${T}.log; exit 1; }
grep -E "equal|qsplit|rel-RMS|speech moves" gpurun_out/${T}.log
f=$(find gpurun_out/${T}_tr -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
ev = sorted((int(r["Start_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1])))
names = [n for _, n in ev]
for i, n in enumerate(names):
    if "attn" in n or "init_state" in n or "nlc_to_ncl" in n:
        print(i, n[:100])
PY
rm -rf gpurun_out/${T}_tr
