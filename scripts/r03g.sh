set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03g}
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/${T}_trace -o run --output-format csv -- python3 bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline --no-f32-subrecord --no-profile > gpurun_out/${T}_trace.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/${T}_trace.log; exit 1; }
k=$(find gpurun_out/${T}_trace -name '*kernel_trace.csv' | head -1)
m=$(find gpurun_out/${T}_trace -name '*memory_copy_trace.csv' | head -1)
python3 - "$k" "$m" > gpurun_out/${T}_timeline.txt <<'PY'
import csv, sys
ev = []
for r in csv.DictReader(open(sys.argv[1])):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:90]))
if sys.argv[2]:
    for r in csv.DictReader(open(sys.argv[2])):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C %s %s bytes" % (r.get("Direction", "?"), r.get("Size", "?"))))
ev.sort()
t0 = ev[0][0]
# the last pass: from the last mk_kernel backwards to the previous mk_kernel
mk = [i for i, e in enumerate(ev) if "mk_kernel<unsigned short, 3, 17>" in e[2]]
a, b = (mk[-2] + 1, mk[-1] + 3) if len(mk) > 1 else (0, len(ev))
print("events between the last two loops (start us, duration us, what):")
for s, e, n in ev[a:b]:
    print("%10.1f %9.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, n))
PY
cat gpurun_out/${T}_timeline.txt | head -150
rm -rf gpurun_out/${T}_trace
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-f32-subrecord > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
