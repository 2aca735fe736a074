"""C4-shape denoise calls (32 clips x 160 frames, fp8 weights) for counter passes over the generic
one-way route: 5 eps evaluations through ggd_denoise (a few hundred dispatches, no sampling loop).
Usage: python scripts/chain_probe.py [dtype] [route]   route: chain (default) | gemm"""
import os
import sys

import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
dtype = sys.argv[1] if len(sys.argv) > 1 else "fp8"
route = sys.argv[2] if len(sys.argv) > 2 else "chain"
L, n = 160, 32
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype=dtype, device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
g = th.Generator().manual_seed(0)
wav = (th.randn(n, 800 * L, generator=g) * 0.1).cuda()
x = th.randn(n, 123, L, generator=g).cuda()
t = th.randint(0, 1000, (n,), generator=g).cuda()
ctx, _ = model.prepare(wav, L)
if route == "gemm":
    assert ctx.lib.ggd_set_route(ctx.h, 5, 1) == 0   # GGD_ROUTE_GEMM_LAUNCHES
for _ in range(5):
    eps = model(x, t, wav=wav)
th.cuda.synchronize()
print("eps rms", float(eps.float().pow(2).mean().sqrt()))
