"""Per-kernel PMC table of the encoder's SECOND call (scripts/enc_once.py under rocprofv3 --pmc):
    python3 scripts/enc_pmc.py DIR [DIR ...]   (each DIR one --pmc pass, counter_collection.csv inside)"""
import csv
import glob
import sys
from collections import OrderedDict

rows = OrderedDict()   # (dispatch order within the 2nd call, kernel) -> {counter: value}
for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        continue
    disp = OrderedDict()
    for r in csv.DictReader(open(f[0])):
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        disp.setdefault(k, {})
        disp[k][r["Counter_Name"]] = disp[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    keys = sorted(disp)
    half = keys[len(keys) // 2:]            # the second (measured) call's dispatches
    for i, k in enumerate(half):
        rows.setdefault((i, k[1]), {}).update(disp[k])
for (i, name), c in rows.items():
    short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
    print(f"{i:3d} {short:60s} " + " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))
