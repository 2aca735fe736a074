"""Training-step throughput of the HIP training path (beat-ours, batch 64 = Train.batch_size of
the reference config): Trainer.step = loss + backward + grad norm + AdamW + lr step on synthetic
poses / wavs.  argv: B, steps, mode ("full": the HA2G encoder trained too, as the reference does;
"frozen": speech tokens from the frozen HIP encoder computed once)."""
import os
import sys
import time

import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
tr = __import__(ge.PKG_NAME + ".training", fromlist=["x"])
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
mode = sys.argv[3] if len(sys.argv) > 3 else "full"
sched = {"type": "noamxf", "warmup_steps": "4k", "d_model": 256}
model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, lr=1.0, weight_decay=0.0, is_training=True,
                                             device="cuda:0", scheduler_params=sched, train_encoder=mode == "full")
trainer = tr.Trainer(model, diffusion, None, lr=1.0, weight_decay=0.0, scheduler_params=sched)
g = th.Generator(device="cuda").manual_seed(0)
poses = th.randn(B, 40, 123, device="cuda", generator=g)
wav = th.randn(B, 32000, device="cuda", generator=g) * 0.1
batch = {"pose": poses, "wav": wav} if mode == "full" else {"pose": poses, "speech_tokens": model.speech_encoder()(wav)}
for _ in range(3):
    trainer.step(batch)
th.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    res = trainer.step(batch)
th.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
print(f"train step ({mode}) B={B}: {dt * 1e3:.2f} ms/step, {B / dt:.1f} clips/s, loss {res['loss']:.4f}, "
      f"grad_norm {res['grad_norm']:.4f}, {model.flat.numel()} trainable params")
