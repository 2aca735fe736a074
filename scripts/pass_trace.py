"""One sampling pass in kernel order (GPU box): every kernel / copy between the end of the
second-to-last persistent-loop launch and the end of the last one, with start offset, duration and
the idle gap in front of it.  Run the bench under the tracer, then report:
    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 bench.py --workload c5 \
        --steps 3 --warmup 1 --no-cpu-baseline --no-f32-subrecord --no-subrecords
    python3 scripts/pass_trace.py DIR"""
import collections
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
loops = [i for i, e in enumerate(ev) if any(k in e[2] for k in ("mk_kernel", "psk_kernel", "lk_kernel", "mr_kernel"))
         and e[1] - e[0] > 1e6]
a, b = loops[-2], loops[-1]
t0 = ev[a][1]
prev = t0
busy = collections.Counter()
count = collections.Counter()
for s, e, n in ev[a + 1:b + 1]:
    print("%9.1f %8.1f gap %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, n[:100]))
    key = n.split("(")[0][-60:]
    busy[key] += (e - s) / 1e3
    count[key] += 1
    prev = max(prev, e)
print("\nper kernel name (us, calls):")
for k, v in busy.most_common():
    print("%9.1f %4d  %s" % (v, count[k], k))
print("pass span %.1f us (loop end to loop end), kernel busy %.1f us" % ((ev[b][1] - t0) / 1e3, sum(busy.values())))
