import os, sys, ctypes
os.environ["GGD_DIAG"] = "1"
sys.path.insert(0, "/root/repo")
import torch as th
import __graft_entry__ as ge
pkg = ge.load_package()
n, L = 32, 160
cfg = pkg.load_config("/root/repo/configs/beat-ours.json")
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype="fp8", device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
wav = (th.randn(n, 800 * L, generator=th.Generator().manual_seed(0)) * 0.1).cuda()
ctx, _ = model.prepare(wav, L)
def diag(what, p0):
    arr = (ctypes.c_int32 * 1)(p0); out = (ctypes.c_double * 64)()
    assert ctx.lib.ggd_diag(ctx.h, what, ctypes.cast(arr, ctypes.c_void_p), 1, 1, ctypes.cast(out, ctypes.c_void_p)) == 0
    return list(out)
for rep in range(3):
    diag(16, 1)
    diffusion.p_sample_loop(model, (n, 123, L), {"wav": wav}, seed=5, n_steps=3, extras=False)
    th.cuda.synchronize()
    st = diag(16, 2)
    b0 = 16
    print(f"rep {rep}: self-attn step 1 L0: staged {st[56]-st[b0]:.2f}, conv pass 1 done {st[59]-st[b0]:.2f}, pass 2 done {st[57]-st[b0]:.2f}, tiles {st[58]-st[b0]:.2f}, phase {st[b0+1]-st[b0]:.2f}")
diag(16, 0)
