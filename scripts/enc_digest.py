"""sha256 of the speech encoder's token outputs on fixed inputs (GPU box): a kernel rewrite that keeps
the accumulation order must print the same digests before and after.
    python3 scripts/enc_digest.py"""
import hashlib
import os
import sys

import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
for dtype in ("bf16", "f32"):
    model, _, _, _, _ = pkg.create_model(123, cfg.Model, dtype=dtype, device="cuda:0")
    model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
    enc = model.encoder()
    for B, T in ((8, 32000), (128, 32000), (4, 128000)):
        wav = th.randn(B, T, generator=th.Generator().manual_seed(B + T)).cuda() * 0.1
        out = enc(wav)
        h = hashlib.sha256()
        for z in out:
            h.update(z.detach().float().cpu().numpy().tobytes())
        print(f"{dtype} B={B} T={T}: {h.hexdigest()[:16]}", flush=True)
