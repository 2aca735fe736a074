"""One bf16 encoder call at B clips under rocprofv3 --kernel-trace: print the last call's kernels
in order with durations (run as: rocprofv3 --kernel-trace -d DIR -o run --output-format csv --
python3 scripts/enc_trace.py B; then python3 scripts/enc_trace.py --report DIR)."""
import csv
import glob
import os
import sys

if sys.argv[1] == "--report":
    f = glob.glob(os.path.join(sys.argv[2], "**", "*kernel_trace.csv"), recursive=True)[0]
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                 r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Workgroup_Size_X", "?"),
                 r.get("LDS_Block_Size", r.get("Lds_Size", "?")))
                for r in csv.DictReader(open(f)))
    st = [i for i, e in enumerate(ev) if "enc_stft_power" in e[2] or "enc_stft_mel" in e[2]]
    a = st[-1]
    t0 = ev[a][0]
    tot = 0.0
    for s, e, n, gx, wx, lds in ev[a:]:
        tot += (e - s) / 1e3
        print("%9.1f %7.1f  grid %8s wg %4s lds %6s  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gx, wx, lds, n[:110]))
    print("sum of kernel durations %.1f us, span %.1f us" % (tot, (ev[-1][1] - t0) / 1e3))
    sys.exit(0)

import torch as th  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
model, _, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
enc = model.encoder()
B = int(sys.argv[1])
wav = th.randn(B, 32000, device="cuda:0") * 0.1
for _ in range(3):
    enc(wav)
th.cuda.synchronize()
print("done", flush=True)
