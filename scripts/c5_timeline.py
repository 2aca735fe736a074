"""Summarise a rocprofv3 kernel trace of the C5 bench: per psk_kernel launch its start/end and the
encoder kernels running before / during it (gaps show what the pass spends outside the loop)."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
psk = [r for r in rows if "psk_kernel" in r["Kernel_Name"]]
prev_end = None
for r in psk:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    enc_in = [x for x in rows if "enc_" in x["Kernel_Name"] and s <= int(x["Start_Timestamp"]) < e]
    gap = (s - prev_end) / 1e3 if prev_end else 0
    between = [x for x in rows if prev_end and prev_end <= int(x["Start_Timestamp"]) < s]
    btime = sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in between) / 1e3
    names = sorted({x["Kernel_Name"][:40] for x in between})
    print(f"psk start {(s - t0) / 1e6:9.3f} ms dur {(e - s) / 1e6:7.3f} ms gap-before {gap:8.1f} us "
          f"(kernels in gap {len(between)}, busy {btime:.1f} us) enc kernels during {len(enc_in)}")
    if len(between) < 12:
        for x in between:
            print("    ", x["Kernel_Name"][:60], (int(x["Start_Timestamp"]) - s) / 1e3,
                  (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
    prev_end = e
