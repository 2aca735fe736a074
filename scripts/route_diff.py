"""psk_kernel vs mk_kernel after k steps on the same inputs (GPU box): where do they differ?"""
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
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
dev = th.device("cuda:0")
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device=dev)
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
n = 4
wav = th.randn(n, 32000, device=dev, generator=th.Generator(device=dev).manual_seed(3)) * 0.1
x = th.randn(n, 123, 40, device=dev, generator=th.Generator(device=dev).manual_seed(4))
ctx, _ = model.prepare(wav, 40)


def route(mode):
    arr = (ctypes.c_int32 * 1)(mode)
    out = ctypes.c_double()
    assert ctx.lib.ggd_diag(ctx.h, 7, arr, 1, 1, ctypes.cast(ctypes.byref(out), ctypes.c_void_p)) == 0


for steps in (1, 2):
    outs = {}
    for name, mode in (("psk", 0), ("mk", 1)):
        route(mode)
        r = diffusion.p_sample_loop(model, (n, 123, 40), {"wav": wav}, noise=x, seed=5, extras=True, n_steps=steps)
        outs[name] = r["sample"].float().cpu()
        outs[name + "_eps"] = r["eps"].float().cpu()
        outs[name + "_x0"] = r["pred_x_start"].float().cpu()
    route(2)
    d = (outs["psk"] - outs["mk"]).abs()
    print(f"steps {steps}: max {d.max().item():.3e} mean {d.mean().item():.3e}")
    print("  per clip  ", [round(v, 4) for v in d.amax(dim=(1, 2)).tolist()])
    print("  per frame ", [round(v, 3) for v in d.amax(dim=(0, 1)).tolist()])
    print("  per chan>0.05", [i for i, v in enumerate(d.amax(dim=(0, 2)).tolist()) if v > 0.05])
    for key in ("_eps", "_x0"):
        d = (outs["psk" + key] - outs["mk" + key]).abs()
        print(f"  {key}: max {d.max().item():.3e}; per frame", [round(v, 3) for v in d.amax(dim=(0, 1)).tolist()])
