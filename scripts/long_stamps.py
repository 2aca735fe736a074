"""Phase times of the long-clip persistent loop (ggd_long.hip) at the C4 shape: barrier stamps of
clip group 0 (ggd_diag what = 16, libggd_diag.so) over the first steps of a DDPM loop.
Usage: GGD_DIAG=1 python scripts/long_stamps.py [dtype] [n_clips] [steps]"""
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
dtype = sys.argv[1] if len(sys.argv) > 1 else "fp8"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 32
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
L = 160
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype=dtype, device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
wav = (th.randn(n, 800 * L, generator=th.Generator().manual_seed(0)) * 0.1).cuda()
ctx, _ = model.prepare(wav, L)
lib = ctx.lib


def diag(what, p0):
    arr = (ctypes.c_int32 * 1)(p0)
    out = (ctypes.c_double * 64)()
    rc = lib.ggd_diag(ctx.h, what, ctypes.cast(arr, ctypes.c_void_p), 1, 1, ctypes.cast(out, ctypes.c_void_p))
    assert rc == 0, rc
    return list(out)


names = ["self-attn", "chain A", "cross-attn", "chain B"]
for rep in range(2):
    diag(16, 1)
    out = diffusion.p_sample_loop(model, (n, 123, L), {"wav": wav}, seed=5, n_steps=steps, extras=False)
    th.cuda.synchronize()
    st = diag(16, 2)
diag(16, 0)
b0 = 4 * model.arch["n_layers"]  # step 1 starts after barrier b0
print("self-attn step 1 L0 sub-phases (us from the phase start): staged %.1f, convs %.1f, wave-0 tiles %.1f, barrier %.1f"
      % (st[56] - st[b0], st[57] - st[b0], st[58] - st[b0], st[b0 + 1] - st[b0]))
print("cross-attn step 1 L0 sub-phases: staged %.1f, convs %.1f, wave-0 tiles %.1f, barrier %.1f"
      % (st[60] - st[b0 + 2], st[61] - st[b0 + 2], st[62] - st[b0 + 2], st[b0 + 3] - st[b0 + 2]))
nl = model.arch["n_layers"]
per = 4 * nl
print(f"{dtype} n={n}: loop start -> barrier j (us):", [round(v, 1) for v in st[:2 + per * 2]])
for k in range(1, steps):
    base = per * k  # stamp of the barrier before step k's first phase
    seg = [st[base + j + 1] - st[base + j] for j in range(per) if st[base + j + 1] > 0]
    if len(seg) < per:
        break
    tot = st[base + per] - st[base]
    print(f"step {k}: {tot:.1f} us;", ", ".join(f"{names[j % 4]} L{j // 4} {v:.1f}" for j, v in enumerate(seg)))
    for j in range(4):
        print(f"   {names[j]:10s} mean {sum(seg[j::4]) / nl:.1f} us")
