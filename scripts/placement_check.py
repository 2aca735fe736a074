"""Persistent loop placement A/B (GPU box): placement 0 (XCD-local clip groups: plain hand-off
stores, L2 flag barriers), 1 (workgroup part p of every clip on XCD p, write-through) and 2 (a
clip's 8 workgroups on one XCD, write-through).  Samples must be bit-identical; prints us/step
and, for placement 0, how many launches ran XCD-local / fell back to write-through."""
import os as _os
_os.environ["GGD_DIAG"] = "1"  # ggd_diag lives in libggd_diag.so only (native.py)
import ctypes
import os
import sys
import time

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


def diag(ctx, what, v, n_out=1):
    arr = (ctypes.c_int32 * 1)(v)
    out = (ctypes.c_double * n_out)()
    native.check(ctx.h, ctx.lib.ggd_diag(ctx.h, what, arr, 1, n_out, ctypes.cast(out, ctypes.c_void_p)), "diag")
    return list(out) if n_out > 1 else out[0]


n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
wav = th.randn(n, 32000, device=dev, generator=th.Generator(device=dev).manual_seed(n)) * 0.1
ctx, _ = model.prepare(wav, 40)
res = {}
for rep in range(2):
    for place in (0, 1, 2):
        diag(ctx, 12, place)
        f = lambda: diffusion.p_sample_loop(model, (n, 123, 40), model_kwargs={"wav": wav}, seed=11, extras=False,
                                            n_steps=steps)["sample"]
        out = f()
        th.cuda.synchronize()
        t0 = time.perf_counter()
        out = f()
        th.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        res[place] = out.clone()
        xl = diag(ctx, 13, 0, 2)
        print(f"rep {rep} placement {place}: {dt:8.2f} ms ({dt / steps * 1e3:6.1f} us/step) xl/fallback {xl}", flush=True)
print("identical:", bool(th.equal(res[0], res[1])) and bool(th.equal(res[0], res[2])), flush=True)
diag(ctx, 12, 0)
