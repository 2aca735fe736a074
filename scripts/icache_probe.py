"""One persistent-loop sample and one per-phase sample of 200 steps (for rocprofv3 --pmc)."""
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
dev = th.device("cuda:0")
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device=dev)
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
wav = th.randn(32, 32000, device=dev) * 0.1
ctx, _ = model.prepare(wav, 40)
for mode in (0, 1):
    arr = (ctypes.c_int32 * 1)(mode)
    out = ctypes.c_double()
    native.check(ctx.h, ctx.lib.ggd_diag(ctx.h, 9, arr, 1, 1, ctypes.cast(ctypes.byref(out), ctypes.c_void_p)), "d9")
    diffusion.p_sample_loop(model, (32, 123, 40), model_kwargs={"wav": wav}, seed=3, extras=False, n_steps=200)
    th.cuda.synchronize()
print("done")
