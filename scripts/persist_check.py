"""Persistent per-clip sampler vs the per-step launch path: agreement and speed (bf16, C2 shape)."""
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
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0, perturb=True))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
g = th.Generator().manual_seed(61)
wav = (th.randn(B, 32000, generator=g) * 0.1).cuda()
ctx, _ = model.prepare(wav, 40)
lib = ctx.lib
out = ctypes.c_double()
arr = (ctypes.c_int32 * 1)


def diag(what, v):
    res = (ctypes.c_double * 17)()
    native.check(ctx.h, lib.ggd_diag(ctx.h, what, arr(v), 1, 1, ctypes.cast(res, ctypes.c_void_p)), "diag")
    return list(res)


print("persistent available:", diag(7, 0)[0])


def run(persist, n_steps, seed=3):
    diag(7, 0 if persist else 1)
    th.cuda.synchronize()
    t0 = time.perf_counter()
    r = diffusion.p_sample_loop(model, (B, 123, 40), {"wav": wav}, seed=seed, n_steps=n_steps)["sample"]
    th.cuda.synchronize()
    return r, time.perf_counter() - t0


def rel(a, b):
    return (((a - b) ** 2).mean().sqrt() / (b ** 2).mean().sqrt()).item()


for n in (1, 2, 10):
    p, _ = run(True, n)
    q, _ = run(False, n)
    print(f"n_steps={n:4d}: rel-RMS persistent vs per-step {rel(p, q):.3e}  max|d| {(p - q).abs().max().item():.3e}"
          f"  finite {bool(th.isfinite(p).all())}", flush=True)
for n in (1000,):
    run(True, n)
    p, tp = run(True, n)
    q, tq = run(False, n)
    print(f"n_steps={n}: rel-RMS {rel(p, q):.3e}; wall persistent {tp * 1e3:.1f} ms ({tp / n * 1e6:.1f} us/step), "
          f"per-step path {tq * 1e3:.1f} ms ({tq / n * 1e6:.1f} us/step)", flush=True)
diag(8, 1)
run(True, 1)
st = diag(8, 2)
print("persistent phases (us, iteration 0, wg 0): emb|layers...|out+update", [round(v, 2) for v in st[:5]])
f = st[5:16]
print("CA head 1 of layer 0 (us from its start): Qgemm+refill, kv_store, kv_load, bar, conv, bar, attn",
      [round(f[i + 1] - f[0], 3) for i in range(7)], "vmcnt(0) drain", round(f[8] - f[0], 3),
      "pmma", round(f[9] - f[8], 3))
