"""Arrival skew at the persistent loop's clip-group barriers (GPU box, diag library).

For clip group 0, every barrier of the second stamped step: the spread of its 8 workgroups'
arrival times, which one arrives last, and workgroup 0's exit after that last arrival."""
import os as _os
_os.environ["GGD_DIAG"] = "1"
import ctypes
import os
import sys

import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
native = __import__(ge.PKG_NAME + ".native", fromlist=["x"])
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
dev = th.device("cuda:0")
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device=dev)
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
wav = th.randn(32, 32000, device=dev) * 0.1
ctx, _ = model.prepare(wav, 40)
B, NSTEP = 2 * 17 * 2, 2
NS = B + 1 + 16 * 17 * NSTEP


def diag(what, p, n_out=1):
    arr = (ctypes.c_int32 * len(p))(*p)
    out = (ctypes.c_double * max(n_out, 1))()
    native.check(ctx.h, ctx.lib.ggd_diag(ctx.h, what, arr, len(p), 1, ctypes.cast(out, ctypes.c_void_p)), "diag")
    return list(out)


# the row-block loop (bf16, round 6): 16 barriers per step -- the last layer's KD runs inside KE
names = [f"L{li}{ph}" for li in range(4) for ph in ("ABCD" if li < 3 else "ABC")] + ["E"]
NPH = len(names)
diffusion.p_sample_loop(model, (32, 123, 40), model_kwargs={"wav": wav}, seed=1, extras=False, n_steps=5)
for rep in range(3):
    diag(10, [1])
    diffusion.p_sample_loop(model, (32, 123, 40), model_kwargs={"wav": wav}, seed=1, extras=False, n_steps=5)
    t = diag(10, [2, NS], NS)
    step = 1
    cells = []
    tot_skew = tot_exit = 0.0
    for e, nm in enumerate(names):
        ep = NPH * step + e
        arr = [t[B + 1 + 2 * (8 * ep + p)] for p in range(8)]
        ex = [t[B + 1 + 2 * (8 * ep + p) + 1] for p in range(8)]
        lo, hi = min(arr), max(arr)
        last = arr.index(hi)
        tot_skew += (hi - lo) / 100.0
        tot_exit += (min(ex) - hi) / 100.0
        cells.append(f"{nm} skew {(hi - lo) / 100:4.2f} last p{last} exit +{(min(ex) - hi) / 100:4.2f}..{(max(ex) - hi) / 100:4.2f}")
    print(f"rep {rep}: skew sum {tot_skew:5.2f} us, last-arrival->exit sum {tot_exit:5.2f} us")
    for i in range(0, len(cells), 4):
        print("   " + " | ".join(cells[i:i + 4]))
diag(10, [0])
