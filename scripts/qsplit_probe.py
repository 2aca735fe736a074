"""Whole-clip vs query-split attention on the bf16 launch route at L = 100 (GPU box): the two
outputs, their difference, and (under rocprofv3 --kernel-trace) which attention kernels ran."""
import os
import sys

import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
arch = pkg.arch_from_config(cfg.Model, 123)
sd = pkg.init_state_dict(arch, seed=0, perturb=True)
model, _, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device="cuda:0")
model.load_state_dict(sd)
g = th.Generator().manual_seed(81)
n, L = 3, 100
wav = th.randn(n, 80000, generator=g) * 0.1
x = th.randn(n, 123, L, generator=g)
t = th.randint(0, 1000, (n,), generator=g)
ctx, _ = model.prepare(wav.cuda(), L)
a = model(x.cuda(), t.cuda(), wav=wav.cuda()).cpu()
th.cuda.synchronize()
print("--- qsplit on", flush=True)
assert ctx.lib.ggd_set_route(ctx.h, 6, 1) == 0
b = model(x.cuda(), t.cuda(), wav=wav.cuda()).cpu()
th.cuda.synchronize()
ctx.lib.ggd_set_route(ctx.h, 6, 0)
print("equal", th.equal(a, b), "max|diff|", (a - b).abs().max().item(), "rms", a.pow(2).mean().sqrt().item(), flush=True)
from oracle import ref_denoiser  # noqa: E402
from tests.conftest import oracle_cfg  # noqa: E402
om = ref_denoiser.OracleModel(sd, oracle_cfg(arch), cache_speech=True)
ref = om(x, t, wav=wav)
rr = lambda p, q: ((p - q).pow(2).mean().sqrt() / q.pow(2).mean().sqrt()).item()
print("rel-RMS clip vs oracle", rr(a, ref), "qsplit vs oracle", rr(b, ref), flush=True)
# the same with a different speech batch: does the output move with the speech?
wav2 = th.randn(n, 80000, generator=g) * 0.1
model.prepare(wav2.cuda(), L)
c2 = model(x.cuda(), t.cuda(), wav=wav2.cuda()).cpu()
print("speech moves the GPU output by", rr(c2, a), "oracle:", rr(om(x, t, wav=wav2), ref), flush=True)
