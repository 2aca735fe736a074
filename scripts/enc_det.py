"""Encoder determinism probe: same input twice, with and without MIOpen deterministic flags."""
import os
import sys

import torch as th
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
model, _, _, _, _ = pkg.create_model(123, cfg.Model, dtype="f32", device="cuda:0")
model.load_state_dict(pkg.init_state_dict(model.arch, seed=0, perturb=True))
enc = model.encoder()
g = th.Generator().manual_seed(61)
wav = (th.randn(8, 32000, generator=g) * 0.1).cuda()


def run():
    return [z.clone() for z in enc(wav)]


for det in (False, True):
    with th.backends.cudnn.flags(enabled=True, benchmark=False, deterministic=det):
        a = run()
        b = run()
    print("deterministic", det, [(x - y).abs().max().item() for x, y in zip(a, b)])
with th.backends.cudnn.flags(enabled=False):
    a = run()
    b = run()
print("cudnn disabled", [(x - y).abs().max().item() for x, y in zip(a, b)])
# locate: mel, first conv, linear
m1, m2 = enc.mel(wav), enc.mel(wav)
print("mel", (m1 - m2).abs().max().item())
x = th.randn(8, 256, 16, 8, device="cuda")
w = th.randn(64, 256, 3, 3, device="cuda")
c1, c2 = F.conv2d(x, w, padding=1), F.conv2d(x, w, padding=1)
print("conv 3x3 256->64", (c1 - c2).abs().max().item())
ps = F.pixel_shuffle(x, 2)
print("pixel_shuffle ok", ps.shape)
y = th.randn(8, 60, 1024, device="cuda")
wl = th.randn(32, 1024, device="cuda")
print("linear", (F.linear(y, wl) - F.linear(y, wl)).abs().max().item())
