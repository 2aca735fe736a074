"""Speech-encoder wall time per call (HIP, bf16) for a few batch sizes (GPU box)."""
import os
import sys
import time

import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
model, _, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
enc = model.encoder()
for B, Tw in ((32, 32000), (128, 32000), (32, 128000)):
    wav = th.randn(B, Tw, device="cuda:0") * 0.1
    enc(wav)
    th.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        enc(wav)
    th.cuda.synchronize()
    print(f"encoder B={B} wav={Tw}: {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms/call", flush=True)
