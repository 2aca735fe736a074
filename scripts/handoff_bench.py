"""Clip-group hand-off inside one launch: XCD-local groups vs groups spread over XCDs (GPU box).

ggd_diag what=5 mode 6 (csrc/ggd_diag.hip mb_xcdsync_kernel): 256 workgroups of 512 threads,
groups of 8; each round every member writes kb KiB and gathers all 8 slices of its group.
Cost per round = slope of the launch time over the number of rounds.
"""
import os as _os
_os.environ["GGD_DIAG"] = "1"  # ggd_diag lives in libggd_diag.so only (native.py)
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
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
wav = th.randn(32, 32000, device="cuda:0") * 0.1
ctx, n = model.prepare(wav, 40)
lib = ctx.lib

VARS = {0: "8K x8, xcd-local, plain loads", 1: "8K x8, xcd-local, sc0 loads", 2: "8K x8, xcd-local, sc1 loads",
        3: "8K x8, xcd-local, sc1 loads + sc1 stores", 4: "8K x8, spread, sc1 loads + sc1 stores",
        5: "8K x8, spread, sc0 loads", 6: "16K x8, xcd-local, sc0 loads",
        7: "16K x8, xcd-local, sc1 loads + sc1 stores", 8: "16K x8, spread, sc1 loads + sc1 stores"}


def run(var, rounds, iters=20):
    arr = (ctypes.c_int32 * 4)(6, rounds | (var << 20), 256, 16)
    out = (ctypes.c_double * 4)()
    native.check(ctx.h, lib.ggd_diag(ctx.h, 5, arr, 4, iters, ctypes.cast(out, ctypes.c_void_p)), "diag")
    return out[0], int(out[1]), int(out[2]), int(out[3])


for var, name in VARS.items():
    t1 = run(var, 1)
    t2 = run(var, 65)
    per = (t2[0] - t1[0]) / 64
    print(f"{name:42s}: launch+1 round {t1[0]:7.2f} us, per round {per:6.2f} us, "
          f"errors {t1[1] + t2[1]}, misplaced {t1[2] + t2[2]}, timeouts {t1[3] + t2[3]}", flush=True)
