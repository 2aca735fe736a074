"""Summarise rocprofv3 --pmc passes (scripts/pmc.sh) per kernel: mean counter value per dispatch.

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE (KiB) reports half the bytes of a
wide coalesced read on gfx950, so hbm_read_bytes = 2 x 1024 x FETCH_SIZE; WRITE_SIZE (KiB) is exact
for 16-B-per-lane stores.  Both count L2 -> fabric requests, Infinity-Cache hits included.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(root, tag, workload=None):
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, f"{tag}_*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in sorted(glob.glob(os.path.join(root, f"{tag}_*", "**", "*kernel_trace.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    for k, cs in per.items():
        short = k.split("(")[0]
        if not any(s in short for s in ("ggd", "mk_kernel", "kb_kernel")):
            continue
        e = {c: sum(v) / len(v) for c, v in cs.items()}
        e["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in e:
            e["hbm_read_bytes"] = 2 * 1024 * e["FETCH_SIZE"]
        if "WRITE_SIZE" in e:
            e["hbm_write_bytes"] = 1024 * e["WRITE_SIZE"]
        if dur.get(k):
            e["avg_duration_ns"] = sum(dur[k]) / len(dur[k])
        out[k] = e
    if workload:
        out["_workload"] = workload
    # the kernels' source hash at collection time: bench.py uses the summary's traffic only while
    # csrc/ still hashes to this (a stale summary is reported as such, never silently reused)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    import bench
    out["_csrc"] = bench.csrc_hash()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
