"""Stage stamps inside the long loop's chain B (diag variant with sub-stamps, see the round-6 notes in
profiles/r06aa_long_chain_stamps.txt): step 0, layer 0 (R F1 F2 P) and the last layer (R F1 F2 PO E P2
+ update).  Usage: GGD_DIAG=1 GGD_LIB=<diag variant> python scripts/long_chain_stamps.py"""
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
n, L = 32, 160
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype="fp8", device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
wav = (th.randn(n, 800 * L, generator=th.Generator().manual_seed(0)) * 0.1).cuda()
ctx, _ = model.prepare(wav, L)


def diag(what, p0):
    arr = (ctypes.c_int32 * 1)(p0)
    out = (ctypes.c_double * 64)()
    rc = ctx.lib.ggd_diag(ctx.h, what, ctypes.cast(arr, ctypes.c_void_p), 1, 1, ctypes.cast(out, ctypes.c_void_p))
    assert rc == 0, rc
    return list(out)


for rep in range(3):
    diag(16, 1)
    diffusion.p_sample_loop(model, (n, 123, L), {"wav": wav}, seed=5, n_steps=2, extras=False)
    th.cuda.synchronize()
    st = diag(16, 2)
    nl = model.arch["n_layers"]
    b0, b1 = st[4 * nl - 1], st[4 * nl]  # last layer's chain B: from its barrier to the next
    names = ["R", "F1(+LN3)", "F2", "PO(+LN_out)", "E(+update)", "P2(+LN1)"]
    t = [st[36 + i] for i in range(6)] + [b1]
    print(f"rep {rep} last-layer chain B {b1 - b0:.1f} us: entry {st[42] - b0:.2f}, staged {st[44] - b0:.2f}, " +
          ", ".join(f"{names[i]} {t[i + 1] - t[i]:.2f}" for i in range(6)) + f" | update done at {st[43] - b0:.2f}, end {st[45] - b0:.2f}")
    a0, a1 = st[3], st[4]
    t = [st[50 + i] for i in range(4)] + [st[59]]
    print(f"      layer-0 chain B {a1 - a0:.1f} us: R start {st[50] - a0:.2f}, " +
          ", ".join(f"{nm} {t[i + 1] - t[i]:.2f}" for i, nm in enumerate(["R", "F1(+LN3)", "F2", "P(+LN1)"])) +
          f" | end {st[59] - a0:.2f}")
diag(16, 0)
