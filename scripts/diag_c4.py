"""C4-shape (L = 160, 128,000-sample wav) kernel latencies via ggd_diag on the generic path:
attention (query-split vs one workgroup per head) and one full denoise step (eager launches)."""
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
dtype = sys.argv[1] if len(sys.argv) > 1 else "fp8"
L = int(sys.argv[2]) if len(sys.argv) > 2 else 160
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype=dtype, device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
wav = th.randn(32, 800 * L, device="cuda:0") * 0.1
ctx, n = model.prepare(wav, L)
ctx.set_schedule(diffusion.betas, diffusion.timestep_map)
lib = ctx.lib


def diag(what, params, iters=100):
    arr = (ctypes.c_int32 * len(params))(*params)
    out = ctypes.c_double()
    native.check(ctx.h, lib.ggd_diag(ctx.h, what, arr, len(params), iters, ctypes.cast(ctypes.byref(out), ctypes.c_void_p)), "diag")
    return out.value


print(f"dtype={dtype} L={L} n=32")
for cross in (0, 1):
    for nq in (0, 1):
        print(f"attention {'cross' if cross else 'self '} {'one WG per head' if nq else 'query-split    '}: "
              f"{diag(1, [cross, 32, nq]):8.2f} us")
print(f"full denoise step (eager): {diag(2, [32], iters=20):8.2f} us")
