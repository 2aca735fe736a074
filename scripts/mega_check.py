"""Persistent reverse loop (ggd_mega.hip) vs the per-phase launches: identical samples, time (GPU box)."""
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
dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
dev = th.device("cuda:0")
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype=dtype, device=dev)
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))


def use_mega(ctx, on):
    arr = (ctypes.c_int32 * 1)(0 if on else 1)
    out = ctypes.c_double()
    native.check(ctx.h, ctx.lib.ggd_diag(ctx.h, 9, arr, 1, 1, ctypes.cast(ctypes.byref(out), ctypes.c_void_p)), "diag9")
    return out.value


for n, steps in ((32, 1000), (8, 200), (1, 50), (3, 50)):
    wav = th.randn(n, 32000, device=dev, generator=th.Generator(device=dev).manual_seed(n)) * 0.1
    ctx, _ = model.prepare(wav, 40)
    res = {}
    for on in (True, False):
        cap = use_mega(ctx, on)
        f = lambda: diffusion.p_sample_loop(model, (n, 123, 40), model_kwargs={"wav": wav}, seed=11, extras=False,
                                            n_steps=steps)["sample"]
        out = f()
        th.cuda.synchronize()
        t0 = time.perf_counter()
        out2 = f()
        th.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        res[on] = (out.clone(), dt, bool(th.equal(out, out2)))
    a, b = res[True][0], res[False][0]
    print(f"n={n:2d} steps={steps:4d} capacity={cap:.0f}: persistent {res[True][1]:8.2f} ms "
          f"({res[True][1] / steps * 1e3:6.1f} us/step, repeat-identical {res[True][2]}), per-phase {res[False][1]:8.2f} ms "
          f"({res[False][1] / steps * 1e3:6.1f} us/step); identical {bool(th.equal(a, b))}, "
          f"max|diff| {float((a - b).abs().max()):.3e}, finite {bool(th.isfinite(a).all())}", flush=True)
    use_mega(ctx, True)
# extras path: last step through the per-phase kernels
wav = th.randn(32, 32000, device=dev) * 0.1
out = {}
for on in (True, False):
    ctx, _ = model.prepare(wav, 40)
    use_mega(ctx, on)
    r = diffusion.p_sample_loop(model, (32, 123, 40), model_kwargs={"wav": wav}, seed=5, n_steps=30)
    out[on] = {k: v.clone() for k, v in r.items()}
use_mega(ctx, True)
print("extras identical:", all(bool(th.equal(out[True][k], out[False][k])) for k in out[True]), flush=True)
