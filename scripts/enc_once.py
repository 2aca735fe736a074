"""One speech-encoder call at B clips after one warm-up call (GPU box), for profiler passes:
    python3 scripts/enc_once.py [B] [WAV_LEN]"""
import os
import sys

import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
T = int(sys.argv[2]) if len(sys.argv) > 2 else 32000
pkg = ge.load_package()
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
model, _, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
enc = model.encoder()
wav = th.randn(B, T, generator=th.Generator().manual_seed(0)).cuda() * 0.1
enc(wav)
th.cuda.synchronize()
enc(wav)
th.cuda.synchronize()
print("done", flush=True)
