"""Sampling time per denoise step on the three fused routes (GPU box): the persistent clip-group
loop (mk_kernel, 8 workgroups per clip), the one-workgroup-per-clip loop (psk_kernel) and the
per-phase launches, for several batch sizes; plus the bf16 agreement of the routes' samples."""
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
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100


def diag(ctx, what, p):
    arr = (ctypes.c_int32 * len(p))(*p)
    out = ctypes.c_double()
    native.check(ctx.h, ctx.lib.ggd_diag(ctx.h, what, arr, len(p), 1, ctypes.cast(ctypes.byref(out), ctypes.c_void_p)), "diag")
    return out.value


for B in [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "32,64,128,256").split(",")]:
    wav = th.randn(B, 32000, device=dev) * 0.1
    ctx, _ = model.prepare(wav, 40)
    res = {}
    for route in ("mega", "persist", "phases"):
        diag(ctx, 7, [0 if route == "persist" else 1])
        diag(ctx, 9, [1 if route == "phases" else 0])
        run = lambda: diffusion.p_sample_loop(model, (B, 123, 40), {"wav": wav}, seed=3, n_steps=steps,
                                              extras=False)["sample"]
        run()
        th.cuda.synchronize()
        t0 = time.perf_counter()
        out = run()
        th.cuda.synchronize()
        res[route] = (time.perf_counter() - t0) / steps * 1e6, out
    diag(ctx, 7, [2])
    diag(ctx, 9, [0])
    ref = res["mega"][1]
    line = f"B={B:4d}: " + "  ".join(
        f"{k} {v[0]:8.1f} us/step (rel diff {((v[1] - ref).norm() / ref.norm()).item():.1e})" for k, v in res.items())
    print(line, flush=True)
