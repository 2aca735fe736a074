"""Locate batch-dependence: encoder, memory, one denoise, sampling (full batch vs a slice)."""
import os
import sys

import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
for dtype in ("f32", "bf16"):
    model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype=dtype, device="cuda:0")
    model.load_state_dict(pkg.init_state_dict(model.arch, seed=0, perturb=True))
    g = th.Generator().manual_seed(61)
    wav = (th.randn(32, 32000, generator=g) * 0.1).cuda()
    x = th.randn(32, 123, 40, generator=g).cuda()
    t = th.randint(0, 1000, (32,), generator=g).cuda()
    enc = model.encoder()
    zf, zp = enc(wav), enc(wav[8:16].clone())
    print(dtype, "encoder", [(a[8:16] - b).abs().max().item() for a, b in zip(zf, zp)])
    ef = model(x, t, wav=wav)
    ep = model(x[8:16].clone(), t[8:16].clone(), wav=wav[8:16].clone())
    print(dtype, "eps", (ef[8:16] - ep).abs().max().item(), ef.abs().max().item())
    for n_steps in (1, 2, 10, 1000):
        full = diffusion.p_sample_loop(model, (32, 123, 40), {"wav": wav}, seed=3, n_steps=n_steps)["sample"]
        part = diffusion.p_sample_loop(model, (8, 123, 40), {"wav": wav[8:16].clone()}, seed=3, clip_offset=8,
                                       n_steps=n_steps)["sample"]
        print(dtype, "sample n_steps", n_steps, (part - full[8:16]).abs().max().item(), full.abs().max().item())
