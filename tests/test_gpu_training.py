"""Training path on the GPU (…_amd/training.py over include/ggd_train.h) against torch / the oracle.

Op level: every HIP forward / backward kernel against torch's own CPU autograd of the same op
(f32; max|diff| <= 1e-4 relative to the operand scale).  Model level: one training step's loss
and the gradients of every trainable parameter against torch autograd through the CPU oracle's
restated model (oracle/ref_denoiser.denoise, gaussian_diffusion.py:531-569's mse) on identical
x_start / t / noise and identical frozen speech tokens: loss rel <= 1e-5, each gradient
max|diff| <= 2e-3 x max|grad|.  Optimizer: AdamW against torch.optim.AdamW; two Trainer steps
(noamxf schedule) against the oracle step with torch.optim.AdamW.
"""
import math

import numpy as np
import pytest
import torch as th
import torch.nn.functional as F

from oracle import ref_denoiser
from tests.conftest import oracle_cfg

pytestmark = pytest.mark.gpu

D_POSE, L, WAV = 123, 40, 32000


@pytest.fixture(scope="module")
def tr(pkg):
    import importlib
    return importlib.import_module(pkg.__name__ + ".training")


def close(got, want, tol=1e-4):
    got, want = got.detach().cpu(), want.detach().cpu()
    scale = max(1.0, want.abs().max().item())
    err = (got - want).abs().max().item()
    assert err <= tol * scale, (err, scale)


@pytest.mark.parametrize("shape", [(77, 45, 133), (96, 130, 3000)])   # the second one runs split-K
@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0), (1, 1)])
def test_gemm_variants(tr, ta, tb, shape):
    g = th.Generator().manual_seed(ta * 2 + tb)
    M, N, K = shape
    A = th.randn(K, M, generator=g) if ta else th.randn(M, K, generator=g)
    B = th.randn(N, K, generator=g) if tb else th.randn(K, N, generator=g)
    C = th.randn(M, N, generator=g)
    bias = th.randn(N, generator=g)
    want = 0.5 * ((A.t() if ta else A) @ (B.t() if tb else B)) + 0.25 * C + bias
    Cd = C.cuda()
    tr.gemm(ta, tb, M, N, K, A.cuda(), M if ta else K, B.cuda(), K if tb else N, Cd, N, alpha=0.5, beta=0.25,
            bias=bias.cuda())
    close(Cd, want, 1e-5)


def test_linear_layernorm_act_backward(tr):
    g = th.Generator().manual_seed(3)
    x = th.randn(5, 7, 96, generator=g)
    w = th.randn(160, 96, generator=g) * 0.1
    b = th.randn(160, generator=g)
    lg, lb = th.randn(160, generator=g), th.randn(160, generator=g)
    dy = th.randn(5, 7, 160, generator=g)

    def run(lin, ln, act, tensors):
        xx, ww, bb, gg, bt = [t.clone().requires_grad_(True) for t in tensors]
        y = act(ln(lin(xx, ww, bb), gg, bt))
        y.backward(dy.to(xx.device))
        return [y] + [t.grad for t in (xx, ww, bb, gg, bt)]

    for act_hip, act_ref in ((tr.squared_relu, lambda u: F.relu(u) ** 2), (tr.silu, F.silu)):
        got = run(tr.linear, tr.layer_norm, act_hip, [t.cuda() for t in (x, w, b, lg, lb)])
        want = run(F.linear, lambda u, a, c: F.layer_norm(u, (160,), a, c, 1e-5), act_ref, [x, w, b, lg, lb])
        for a, c in zip(got, want):
            close(a, c, 1e-4)


def test_seqconv_and_attention_backward(tr):
    g = th.Generator().manual_seed(4)
    n, Lq, Lk, H, dk = 3, 40, 32, 8, 32
    q = th.randn(n, Lq, H * dk, generator=g)
    k = th.randn(n, Lk, H * dk, generator=g)
    v = th.randn(n, Lk, H * dk, generator=g)
    w = th.randn(dk, 1, 3, generator=g)
    bc = th.randn(dk, generator=g)
    do = th.randn(n, Lq, H * dk, generator=g)
    scale = 1 / math.sqrt(dk)

    def conv_ref(x, w_, b_):  # transformer.py:28-44: padding 2, crop 1 each side
        y = x.reshape(n, -1, H, dk).permute(0, 2, 3, 1).reshape(n * H, dk, -1)
        y = F.conv1d(y, w_, b_, padding=2, groups=dk)[:, :, 1:-1]
        return y.reshape(n, H, dk, -1).permute(0, 3, 1, 2).reshape(n, -1, H * dk)

    def attn_ref(q_, k_, v_):
        qh, kh, vh = (t.reshape(n, -1, H, dk).transpose(1, 2) for t in (q_, k_, v_))
        p = th.softmax(qh @ kh.transpose(-1, -2) * scale, dim=-1)
        return (p @ vh).transpose(1, 2).reshape(n, -1, H * dk)

    def run(conv, attn, dev):
        ts = [t.to(dev).clone().requires_grad_(True) for t in (q, k, v, w, bc)]
        qq, kk, vv, ww, bb = ts
        o = attn(conv(qq, ww, bb), kk, vv)
        o.backward(do.to(dev))
        return [o] + [t.grad for t in ts]

    got = run(lambda x, w_, b_: tr._SeqConv.apply(x, w_, b_, H), lambda a, b_, c: tr._Attention.apply(a, b_, c, H, scale),
              "cuda")
    want = run(conv_ref, attn_ref, "cpu")
    for a, c in zip(got, want):
        close(a, c, 1e-4)


def test_adamw_matches_torch(tr, pkg, beat_cfg):
    arch = pkg.arch_from_config(beat_cfg.Model, D_POSE)
    sd = pkg.init_state_dict(arch, seed=0)
    model = tr.TrainableModel(arch, sd, "cuda")
    ref = model.flat.detach().cpu().clone().requires_grad_(True)
    opt_ref = th.optim.AdamW([ref], lr=3e-3, weight_decay=0.01)
    opt = tr.AdamW(model, lr=3e-3, weight_decay=0.01)
    g = th.Generator().manual_seed(5)
    for _ in range(3):
        grad = th.randn(ref.shape, generator=g) * 1e-2
        ref.grad = grad.clone()
        opt_ref.step()
        model.flat_grad.copy_(grad)
        opt.step()
    close(model.flat, ref, 2e-6)
    gn = tr.grad_norm(model)
    want = grad.double().norm().item()   # f64: a long f32 CPU reduction drifts by ~1e-4
    assert abs(gn - want) <= 1e-5 * want, (gn, want)


@pytest.fixture(scope="module")
def train_setup(pkg, beat_cfg, tr):
    arch = pkg.arch_from_config(beat_cfg.Model, D_POSE)
    sd = pkg.init_state_dict(arch, seed=0, perturb=True)
    enc_model, diffusion, _, _, _ = pkg.create_model(D_POSE, beat_cfg.Model, dtype="f32", device="cuda:0")
    enc_model.load_state_dict(sd)
    diffusion = pkg.create_diffusion(beat_cfg.Model.Diffusion.to_dict(), True)
    n = 3
    g = th.Generator().manual_seed(7)
    wav = th.randn(n, WAV, generator=g) * 0.1
    z = enc_model.encoder()(wav.cuda())
    return arch, sd, diffusion, n, g, z


def _oracle_loss(arch, sd_ref, diffusion, x0, t, noise, z_cpu):
    idx = t.numpy()
    ca = th.from_numpy(diffusion.sqrt_alphas_cumprod[idx]).float().reshape(-1, 1, 1)
    cb = th.from_numpy(diffusion.sqrt_one_minus_alphas_cumprod[idx]).float().reshape(-1, 1, 1)
    x_t = ca * x0 + cb * noise
    cfg = oracle_cfg(arch)
    speech = ref_denoiser.speech_memory(sd_ref, cfg, z_cpu)
    eps = ref_denoiser.denoise(sd_ref, cfg, x_t, t, speech=speech)
    return ((eps - noise) ** 2).mean(dim=(1, 2)).mean()


def test_training_step_gradients_match_oracle(tr, train_setup):
    arch, sd, diffusion, n, g, z = train_setup
    model = tr.TrainableModel(arch, sd, "cuda")
    x0 = th.randn(n, D_POSE, L, generator=g)
    t = th.tensor([999, 417, 3])
    noise = th.randn(n, D_POSE, L, generator=g)
    model.zero_grad()
    out = tr.training_losses(diffusion, model, x0.cuda(), t.cuda(), {"speech_tokens": z}, noise=noise.cuda())
    loss = out["mse"].mean()
    loss.backward()
    names = list(model.params)
    sd_ref = {k: v.detach().float().clone() for k, v in sd.items()}
    for k in names:
        sd_ref[k].requires_grad_(True)
    want = _oracle_loss(arch, sd_ref, diffusion, x0, t, noise, tuple(a.cpu() for a in z))
    want.backward()
    assert abs(loss.item() - want.item()) <= 1e-5 * want.item(), (loss.item(), want.item())
    # The key conv biases get an exactly-zero gradient (softmax over keys is invariant to a bias
    # added to every key): both sides hold rounding noise there, so every error is measured
    # against max(max|grad| of the tensor, 1e-4 x the largest gradient of the model).
    floor = 1e-4 * max(sd_ref[k].grad.abs().max().item() for k in names)
    worst = []
    for k in names:
        gg, gr = model.params[k].grad.cpu(), sd_ref[k].grad
        assert gr is not None, k
        s = max(gr.abs().max().item(), floor)
        e = (gg - gr).abs().max().item() / s
        worst.append((e, k, gr.abs().max().item()))
    worst.sort(reverse=True)
    print("\nworst gradient errors (max|diff| / scale, tensor, max|grad|):", worst[:6])
    for k in names:
        if k.endswith("key.1.conv.bias"):
            assert sd_ref[k].grad.abs().max().item() <= 1e-3 * floor / 1e-4
    assert worst[0][0] <= 2e-3, worst[:6]


def test_speed_loss_gradients_match_oracle(tr, train_setup):
    """mse + the reference's speed losses (trainer.py:172-193) through pred_x_start: gradients of the
    HIP model vs the oracle's torch autograd on the same loss, and Trainer accepts the terms."""
    arch, sd, diffusion, n, g, z = train_setup
    params = {"speed_loss": 0.5, "speed_l1_loss": 1.0, "speed_constraint_loss": 0.1}
    model = tr.TrainableModel(arch, sd, "cuda")
    x0 = th.randn(n, D_POSE, L, generator=g)
    t = th.tensor([640, 201, 37])
    noise = th.randn(n, D_POSE, L, generator=g)
    model.zero_grad()
    out = tr.training_losses(diffusion, model, x0.cuda(), t.cuda(), {"speech_tokens": z}, noise=noise.cuda())
    terms, extra = tr.speed_losses(x0.cuda(), out["pred_x_start"], params)
    loss = out["mse"].mean() + extra
    loss.backward()
    names = list(model.params)
    sd_ref = {k: v.detach().float().clone() for k, v in sd.items()}
    for k in names:
        sd_ref[k].requires_grad_(True)
    idx = t.numpy()
    ext = lambda a: th.from_numpy(a[idx]).float().reshape(-1, 1, 1)
    x_t = ext(diffusion.sqrt_alphas_cumprod) * x0 + ext(diffusion.sqrt_one_minus_alphas_cumprod) * noise
    cfg = oracle_cfg(arch)
    speech = ref_denoiser.speech_memory(sd_ref, cfg, tuple(a.cpu() for a in z))
    eps = ref_denoiser.denoise(sd_ref, cfg, x_t, t, speech=speech)
    px0 = ext(diffusion.sqrt_recip_alphas_cumprod) * x_t - ext(diffusion.sqrt_recipm1_alphas_cumprod) * eps
    want_terms, want_extra = tr.speed_losses(x0, px0, params)
    want = ((eps - noise) ** 2).mean(dim=(1, 2)).mean() + want_extra
    want.backward()
    for k in ("speed", "speed_l1", "speed_constraint"):
        assert abs(terms[k].item() - want_terms[k].item()) <= 1e-4 * abs(want_terms[k].item()) + 1e-7, k
    assert abs(loss.item() - want.item()) <= 1e-5 * want.item(), (loss.item(), want.item())
    floor = 1e-4 * max(sd_ref[k].grad.abs().max().item() for k in names)
    worst = max(((model.params[k].grad.cpu() - sd_ref[k].grad).abs().max().item()
                 / max(sd_ref[k].grad.abs().max().item(), floor), k) for k in names)
    print("\nworst gradient error with the speed losses:", worst)
    assert worst[0] <= 2e-3, worst
    trainer = tr.Trainer(model, diffusion, speech_encoder=None, lr=1e-4, loss_params=params)
    res = trainer.step({"pose": x0.transpose(1, 2).cuda(), "speech_tokens": z}, noise=noise.cuda(), t=t.cuda())
    assert np.isfinite(res["loss"]) and res["loss"] > 0


def test_trainer_steps_match_torch_adamw(tr, train_setup):
    arch, sd, diffusion, n, g, z = train_setup
    sched = {"type": "noamxf", "warmup_steps": "4k", "d_model": 256}
    model = tr.TrainableModel(arch, sd, "cuda")
    trainer = tr.Trainer(model, diffusion, speech_encoder=None, lr=1.0, weight_decay=0.0, scheduler_params=sched)
    names = list(model.params)
    sd_ref = {k: v.detach().float().clone() for k, v in sd.items()}
    params = [sd_ref[k].requires_grad_(True) for k in names]
    opt = th.optim.AdamW(params, lr=1.0, weight_decay=0.0)
    noam = lambda step: 256 ** -0.5 * min((step + 1) ** -0.5, (step + 1) * 4000 ** -1.5)   # lr_scheduler.py NoamLR
    z_cpu = tuple(a.cpu() for a in z)
    for step in range(2):
        x0 = th.randn(n, D_POSE, L, generator=g)
        t = th.randint(0, 1000, (n,), generator=g)
        noise = th.randn(n, D_POSE, L, generator=g)
        res = trainer.step({"pose": x0.transpose(1, 2).cuda(), "speech_tokens": z}, noise=noise.cuda(), t=t.cuda())
        for grp in opt.param_groups:
            grp["lr"] = noam(step)
        opt.zero_grad()
        loss = _oracle_loss(arch, sd_ref, diffusion, x0, t, noise, z_cpu)
        loss.backward()
        opt.step()
        assert abs(res["loss"] - loss.item()) <= 1e-4 * loss.item()
        assert abs(res["lr"] - noam(step + 1)) <= 1e-12
    got = th.cat([model.params[k].detach().cpu().reshape(-1) for k in names])
    want = th.cat([sd_ref[k].detach().reshape(-1) for k in names])
    start = th.cat([sd[k].float().reshape(-1) for k in names])
    d_got, d_want = got - start, want - start
    rel = ((d_got - d_want).norm() / d_want.norm()).item()
    assert rel <= 2e-2, rel   # AdamW's m / sqrt(v) amplifies f32 summation-order noise where g ~ 0
    ck = trainer.checkpoint()
    assert set(ck) >= {"model_state_dict", "optimizer_state_dict", "lr_scheduler_state_dict", "train_step"}


def test_create_model_training_surface(pkg, beat_cfg, tr):
    """create_model(is_training=True) returns the reference's 5-tuple (model_creation.py:51-191)."""
    model, diffusion, opt, sampler, sched = pkg.create_model(
        D_POSE, beat_cfg.Model, lr=1.0, weight_decay=0.0, is_training=True, device="cuda:0",
        scheduler_params={"type": "noamxf", "warmup_steps": "4k", "d_model": 256})
    assert isinstance(model, tr.TrainableModel) and isinstance(opt, tr.AdamW)
    assert diffusion.num_timesteps == 1000 and sampler.num_timesteps == 1000
    assert sched.get_last_lr()[0] == pytest.approx(256 ** -0.5 * 4000 ** -1.5)
    n_train = sum(p.numel() for p in model.parameters())
    assert n_train == model.flat.numel()
    wav = th.randn(2, WAV, generator=th.Generator().manual_seed(9)) * 0.1
    trainer = tr.Trainer(model, diffusion, None, lr=1.0, weight_decay=0.0,
                         scheduler_params={"type": "noamxf", "warmup_steps": "4k", "d_model": 256})
    poses = th.randn(2, L, D_POSE, generator=th.Generator().manual_seed(10))
    before = model.flat.clone()
    res = trainer.step({"pose": poses.cuda(), "wav": wav.cuda()})   # speech tokens from the frozen HIP encoder
    assert np.isfinite(res["loss"]) and res["grad_norm"] > 0
    assert not th.equal(before, model.flat)


def test_checkpoint_roundtrip_resumes_identically(pkg, beat_cfg, tr, train_setup, tmp_path):
    """formats.save_checkpoint (trainer.py:200-212 layout) -> load_checkpoint -> Trainer.load_checkpoint:
    the resumed trainer's next step equals the uninterrupted one bit for bit."""
    import importlib
    fm = importlib.import_module(pkg.__name__ + ".formats")
    arch, sd, diffusion, n, g, z = train_setup
    sched = {"type": "noamxf", "warmup_steps": "4k", "d_model": 256}
    mk = lambda: tr.Trainer(tr.TrainableModel(arch, sd, "cuda"), diffusion, None, lr=1.0, weight_decay=0.0,
                            scheduler_params=sched)
    a = mk()
    gg = th.Generator().manual_seed(21)
    batches = [({"pose": th.randn(n, L, D_POSE, generator=gg).cuda(), "speech_tokens": z},
                th.randn(n, D_POSE, L, generator=gg).cuda(), th.randint(0, 1000, (n,), generator=gg).cuda())
               for _ in range(2)]
    a.step(batches[0][0], noise=batches[0][1], t=batches[0][2])
    path = tmp_path / "chkpt_gpu0_seed0.pt"
    fm.save_checkpoint(str(path), a)
    b = mk()
    b.load_checkpoint(fm.load_checkpoint(str(path), map_location="cuda:0"))
    ra = a.step(batches[1][0], noise=batches[1][1], t=batches[1][2])
    rb = b.step(batches[1][0], noise=batches[1][1], t=batches[1][2])
    assert ra == rb and th.equal(a.model.flat, b.model.flat)


# ------------------------------------------------------------------------------------------
# speech-encoder training (train-mode SE-ResNet34 on NHWC activations)
# ------------------------------------------------------------------------------------------
# (1, 32): im2col route (conv1); the others: the implicit GEMMs, incl. a 64-column tile spanning taps
# (16 input channels) and stride-2 dgrad parity cases
@pytest.mark.parametrize("cin,cout,k,stride,pad,bias", [(1, 32, 3, 1, 1, True), (32, 64, 3, 2, 1, False),
                                                         (32, 64, 1, 2, 0, False), (64, 64, 2, 1, 0, True),
                                                         (16, 32, 3, 1, 1, True), (64, 128, 3, 2, 1, False),
                                                         (128, 16, 1, 1, 0, True)])
def test_conv2d_nhwc_matches_torch(tr, cin, cout, k, stride, pad, bias):
    g = th.Generator().manual_seed(cin + cout + k)
    x = th.randn(3, 17, 13, cin, generator=g)                         # NHWC
    w = th.randn(cout, cin, k, k, generator=g) * 0.2
    b = th.randn(cout, generator=g) if bias else None
    dy_shape = (3, (17 + 2 * pad - k) // stride + 1, (13 + 2 * pad - k) // stride + 1, cout)
    dy = th.randn(*dy_shape, generator=g)

    def ref(xx, ww, bb):
        return F.conv2d(xx.permute(0, 3, 1, 2), ww, bb, stride=stride, padding=pad).permute(0, 2, 3, 1)

    def run(fn, dev):
        ts = [t.to(dev).clone().requires_grad_(True) if t is not None else None for t in (x, w, b)]
        y = fn(*ts)
        y.backward(dy.to(dev))
        return [y] + [t.grad for t in ts if t is not None]

    got = run(lambda a, c, d: tr._Conv2d.apply(a, c, d, stride, pad), "cuda")
    want = run(ref, "cpu")
    for a, c in zip(got, want):
        close(a, c, 2e-5)


def test_batchnorm_se_shuffle_flatten_match_torch(tr):
    g = th.Generator().manual_seed(12)
    x = th.randn(3, 8, 6, 32, generator=g) * 2 + 1
    gam, bet = th.randn(32, generator=g), th.randn(32, generator=g)
    sc = th.rand(3, 32, generator=g)
    dy = th.randn(3, 16, 12, 8, generator=g)

    def ref(xx, gg, bb, ss):
        y = F.batch_norm(xx.permute(0, 3, 1, 2), None, None, gg, bb, True, 0.0, 1e-5)
        pooled = y.mean(dim=(2, 3))
        y = y * th.sigmoid(ss + pooled)[:, :, None, None]
        y = F.pixel_shuffle(F.relu(y), 2)                                  # (3, 8, 16, 12)
        return y.permute(0, 2, 3, 1)

    def hip(xx, gg, bb, ss):
        y = tr._BatchNorm2d.apply(xx, gg, bb, [])
        pooled = tr._ChanMean.apply(y)
        y = tr._ChanScale.apply(y, tr._Sigmoid.apply(tr.add(ss, pooled)))
        return tr._PixelShuffle.apply(tr.relu(y).contiguous(), 2)

    def run(fn, dev):
        ts = [t.to(dev).clone().requires_grad_(True) for t in (x, gam, bet, sc)]
        y = fn(*ts)
        y.backward(dy.to(dev))
        return [y] + [t.grad for t in ts]

    for a, c in zip(run(hip, "cuda"), run(ref, "cpu")):
        close(a, c, 1e-4)
    h = th.randn(2, 5, 7, 3, generator=g)
    flat = tr._HeadFlatten.apply(h.cuda()).cpu()
    assert th.equal(flat, h.permute(0, 3, 1, 2).reshape(2, 15, 7).transpose(1, 2))   # ResNetSE34V2.py:161-163


@pytest.fixture(scope="module")
def enc_setup(pkg, beat_cfg, tr):
    arch = pkg.arch_from_config(beat_cfg.Model, D_POSE)
    sd = pkg.init_state_dict(arch, seed=0, perturb=True)
    diffusion = pkg.create_diffusion(beat_cfg.Model.Diffusion.to_dict(), True)
    wav = th.randn(3, WAV, generator=th.Generator().manual_seed(17)) * 0.1
    return arch, sd, diffusion, wav


def test_encoder_training_gradients_match_oracle(tr, enc_setup):
    """The HA2G encoder in train mode (BatchNorm on batch statistics) from the same front-end image:
    speech tokens and every encoder parameter gradient of L = sum_l <z_l, R_l> against torch autograd
    through the oracle.  Deep train-mode BN chains amplify f32 summation-order differences, so the
    yardstick is an f64 oracle run: our error vs f64 must stay within 4x the f32 oracle's own error
    vs f64 (or 1e-3 of the tensor's gradient scale).  The running statistics follow
    nn.BatchNorm2d's momentum-0.1 update."""
    arch, sd, diffusion, wav = enc_setup
    model = tr.TrainableModel(arch, sd, "cuda", train_encoder=True)
    img = model.speech_encoder().frontend(wav.cuda())
    z = model.encode(img=img)
    g = th.Generator().manual_seed(19)
    R = [th.randn(zi.shape, generator=g) for zi in z]
    model.zero_grad()
    sum((zi * r.cuda()).sum() for zi, r in zip(z, R)).backward()
    names = [k for k in model.params if k.startswith("speech_encoder.")]

    def oracle(dtype):
        sdr = {k: v.detach().to(dtype).clone() if v.is_floating_point() else v for k, v in sd.items()}
        for k in names:
            sdr[k].requires_grad_(True)
        zr = ref_denoiser.speech_encoder_from_image(sdr, img.cpu().to(dtype), train=True)
        sum((zi * r.to(dtype)).sum() for zi, r in zip(zr, R)).backward()
        return zr, {k: sdr[k].grad for k in names}

    z64, g64 = oracle(th.float64)
    z32, g32 = oracle(th.float32)
    for a, b, c in zip(z, z32, z64):
        e_ours = (a.detach().cpu().double() - c).abs().max().item()
        e_ref = (b.detach().double() - c).abs().max().item()
        assert e_ours <= max(4 * e_ref, 1e-5 * c.abs().max().item()), (e_ours, e_ref)
    worst = []
    for k in names:
        s_ = g64[k].abs().max().item()
        e_ours = (model.params[k].grad.cpu().double() - g64[k]).abs().max().item() / s_
        e_ref = (g32[k].double() - g64[k]).abs().max().item() / s_
        worst.append((e_ours / max(4 * e_ref, 1e-3), e_ours, e_ref, k))
    worst.sort(reverse=True)
    print("\nencoder gradients (ratio to bound, ours vs f64, f32 oracle vs f64):", worst[:5])
    assert worst[0][0] <= 1.0, worst[:5]
    # running statistics of the first BN: 0.9 init + 0.1 batch stats of relu(conv1(img))
    r = "speech_encoder.wav_encoder.feat_extractor."
    a = F.relu(F.conv2d(img.cpu()[:, None], sd[r + "conv1.weight"].float(), sd[r + "conv1.bias"].float(), padding=1))
    rm = 0.9 * sd[r + "bn1.running_mean"] + 0.1 * a.mean(dim=(0, 2, 3))
    rv = 0.9 * sd[r + "bn1.running_var"] + 0.1 * a.var(dim=(0, 2, 3), unbiased=True)
    close(model.buffers[r + "bn1.running_mean"], rm, 1e-4)
    close(model.buffers[r + "bn1.running_var"], rv, 1e-4)
    assert int(model.buffers[r + "bn1.num_batches_tracked"]) == int(sd[r + "bn1.num_batches_tracked"]) + 1


def test_training_step_with_encoder_matches_oracle_loss(tr, enc_setup):
    """One full training step with the encoder trained: the loss (train-mode encoder + decoder) and
    the decoder's gradients against the oracle from the same front-end image."""
    arch, sd, diffusion, wav = enc_setup
    model = tr.TrainableModel(arch, sd, "cuda", train_encoder=True)
    n = wav.shape[0]
    g = th.Generator().manual_seed(18)
    x0 = th.randn(n, D_POSE, L, generator=g)
    t = th.tensor([911, 250, 7])
    noise = th.randn(n, D_POSE, L, generator=g)
    model.zero_grad()
    out = tr.training_losses(diffusion, model, x0.cuda(), t.cuda(), {"wav": wav.cuda()}, noise=noise.cuda())
    loss = out["mse"].mean()
    loss.backward()
    img = model.speech_encoder().frontend(wav.cuda()).cpu()
    sd_ref = {k: v.detach().float().clone() for k, v in sd.items()}
    dec = [k for k in model.params if not k.startswith("speech_encoder.")]
    for k in dec:
        sd_ref[k].requires_grad_(True)
    z_ref = ref_denoiser.speech_encoder_from_image(sd_ref, img, train=True)
    want = _oracle_loss(arch, sd_ref, diffusion, x0, t, noise, z_ref)
    want.backward()
    assert abs(loss.item() - want.item()) <= 1e-4 * want.item(), (loss.item(), want.item())
    floor = 1e-4 * max(sd_ref[k].grad.abs().max().item() for k in dec)
    worst = max((model.params[k].grad.cpu() - sd_ref[k].grad).abs().max().item()
                / max(sd_ref[k].grad.abs().max().item(), floor) for k in dec)
    assert worst <= 2e-3, worst


# ------------------------------------------------------------------------------------------
# checkpoints written by training feed the sampler (main.py:113-115: strict load of
# chkpt["model_state_dict"]); optimizer state in torch.optim.AdamW's layout (trainer.py:203, 218)
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("train_encoder", [False, True])
def test_trained_checkpoint_loads_into_sampler(pkg, beat_cfg, tr, tmp_path, train_encoder):
    import importlib
    fm = importlib.import_module(pkg.__name__ + ".formats")
    arch = pkg.arch_from_config(beat_cfg.Model, D_POSE)
    sd = pkg.init_state_dict(arch, seed=0, perturb=True)
    diffusion = pkg.create_diffusion(beat_cfg.Model.Diffusion.to_dict(), True)
    model = tr.TrainableModel(arch, sd, "cuda", train_encoder=train_encoder)
    trainer = tr.Trainer(model, diffusion, None, lr=1e-3, weight_decay=0.0)
    g = th.Generator().manual_seed(31)
    wav = th.randn(3, WAV, generator=g) * 0.1
    trainer.step({"pose": th.randn(3, L, D_POSE, generator=g).cuda(), "wav": wav.cuda()})
    path = tmp_path / "chkpt_gpu0_seed0.pt"
    fm.save_checkpoint(str(path), trainer)
    trained = {k: v.cpu() for k, v in model.state_dict().items()}
    assert list(trained) == list(sd)                    # the reference module tree's full key set, in order
    sampler, _, _, _, _ = pkg.create_model(D_POSE, beat_cfg.Model, dtype="f32", device="cuda:0")
    fm.load_model_checkpoint(sampler, str(path), strict=True)
    x = th.randn(3, D_POSE, L, generator=g)
    t = th.tensor([999, 500, 0])
    eps = sampler(x.cuda(), t.cuda(), wav=wav.cuda()).cpu()
    want = ref_denoiser.OracleModel(trained, oracle_cfg(arch), cache_speech=True)(x, t, wav=wav)
    assert (eps - want).abs().max().item() <= 1e-4
    if train_encoder:   # the step moved the encoder's BN statistics; the sampler sees the moved ones
        k = "speech_encoder.wav_encoder.feat_extractor.bn1.running_mean"
        assert not th.equal(trained[k], sd[k]) and int(trained[k.replace("running_mean", "num_batches_tracked")]) == 1


def test_eval_mode_uses_running_statistics(pkg, beat_cfg, tr):
    """TrainableModel.eval() (model.eval(), trainer.py:252): the encoder normalises with the running
    statistics and a forward leaves them unchanged; train() restores batch statistics."""
    arch = pkg.arch_from_config(beat_cfg.Model, D_POSE)
    sd = pkg.init_state_dict(arch, seed=0, perturb=True)
    model = tr.TrainableModel(arch, sd, "cuda", train_encoder=True)
    g = th.Generator().manual_seed(41)
    wav = th.randn(2, WAV, generator=g) * 0.1
    x = th.randn(2, D_POSE, L, generator=g)
    t = th.tensor([10, 900])
    before = {k: v.clone() for k, v in model.buffers.items()}
    model.eval()
    with th.no_grad():
        e1 = model(x.cuda(), t.cuda(), wav=wav.cuda()).cpu()
    assert all(th.equal(before[k], v) for k, v in model.buffers.items())
    want = ref_denoiser.OracleModel(sd, oracle_cfg(arch), cache_speech=True)(x, t, wav=wav)
    assert (e1 - want).abs().max().item() <= 1e-4            # eval-mode BN = the oracle's running stats
    model.train()
    with th.no_grad():
        model(x.cuda(), t.cuda(), wav=wav.cuda())
    k = "speech_encoder.wav_encoder.feat_extractor.bn1.running_mean"
    assert not th.equal(before[k], model.buffers[k])


def test_optimizer_state_is_torch_adamw_layout(pkg, beat_cfg, tr):
    """Our AdamW's state_dict loads into torch.optim.AdamW over the reference parameter order and
    both take the same next step; and a torch AdamW state loads back into ours."""
    arch = pkg.arch_from_config(beat_cfg.Model, D_POSE)
    sd = pkg.init_state_dict(arch, seed=0)
    model = tr.TrainableModel(arch, sd, "cuda")
    opt = tr.AdamW(model, lr=3e-3, weight_decay=0.01)
    g = th.Generator().manual_seed(6)
    for _ in range(2):
        model.flat_grad.copy_(th.randn(model.flat.shape, generator=g) * 1e-2)
        opt.step()
    st = opt.state_dict()
    params = [p.detach().cpu().clone().requires_grad_(True) for p in model.params.values()]
    ref = th.optim.AdamW(params, lr=3e-3, weight_decay=0.01)
    ref.load_state_dict(st)
    grad = th.randn(model.flat.shape, generator=g) * 1e-2
    off = 0
    for p in params:
        p.grad = grad[off:off + p.numel()].view(p.shape).clone()
        off += p.numel()
    ref.step()
    model.flat_grad.copy_(grad)
    opt.step()
    close(model.flat, th.cat([p.detach().reshape(-1) for p in params]), 2e-6)
    opt2 = tr.AdamW(tr.TrainableModel(arch, sd, "cuda"), lr=3e-3, weight_decay=0.01)
    opt2.load_state_dict(ref.state_dict())
    assert opt2.step_count == 3
    close(opt2.exp_avg, opt.exp_avg, 1e-6)
    close(opt2.exp_avg_sq, opt.exp_avg_sq, 1e-6)


# ------------------------------------------------------------------------------------------
# the inpaint model's training inputs (trainer.py:139-146, model.py:120-166)
# ------------------------------------------------------------------------------------------
def test_inpaint_training_gradients_match_oracle_and_checkpoint_samples(pkg, beat_cfg, tr):
    """Speech2GestureModelInpaint trained the reference's way: the trainer builds inpaint_pose = the
    clip's poses and inpaint_mask = 1 on the first pose_seed_len frames (trainer.py:139-146); the
    model adds proj([pose * mask, mask]) to x (model.py:152-166).  Loss and every gradient (the proj
    MLP's included) against torch autograd through the oracle; then a Trainer step's checkpoint loads
    strictly into the inpaint sampler and its eps matches the oracle on the trained weights."""
    cfg = dict(beat_cfg.Model.to_dict(), type="inpaint")   # beat-ours with Model.type "inpaint"
    arch = pkg.arch_from_config(cfg, D_POSE)
    assert arch["type"] == "inpaint"
    seed_len = int(cfg["Generate"]["pose_seed_len"])
    sd = pkg.init_state_dict(arch, seed=0, perturb=True)
    g = th.Generator().manual_seed(53)
    for k in [k for k in sd if k.startswith("proj.")]:   # GLIDE zero init would give proj.0 / proj.2 zero gradients
        sd[k] = th.randn(sd[k].shape, generator=g) * 0.05
    sampler, _, _, _, _ = pkg.create_model(D_POSE, cfg, dtype="f32", device="cuda:0")
    sampler.load_state_dict(sd)
    n = 3
    wav = th.randn(n, WAV, generator=g) * 0.1
    z = sampler.encoder()(wav.cuda())
    diffusion = pkg.create_diffusion(beat_cfg.Model.Diffusion.to_dict(), True)
    model = tr.TrainableModel(arch, sd, "cuda", pose_seed_len=seed_len)
    assert "proj.0.weight" in model.params and "blend_layer.weight" not in model.params
    trainer = tr.Trainer(model, diffusion, None, lr=1e-3, weight_decay=0.0)
    poses = th.randn(n, L, D_POSE, generator=g)
    t = th.tensor([901, 333, 12])
    noise = th.randn(n, D_POSE, L, generator=g)
    model.zero_grad()
    terms = trainer._compute_loss({"pose": poses.cuda(), "speech_tokens": z}, noise=noise.cuda(), t=t.cuda())
    terms["loss"].backward()
    names = list(model.params)
    sd_ref = {k: v.detach().float().clone() for k, v in sd.items()}
    for k in names:
        sd_ref[k].requires_grad_(True)
    x0 = poses.transpose(1, 2)
    idx = t.numpy()
    ext = lambda a: th.from_numpy(a[idx]).float().reshape(-1, 1, 1)
    x_t = ext(diffusion.sqrt_alphas_cumprod) * x0 + ext(diffusion.sqrt_one_minus_alphas_cumprod) * noise
    ocfg = oracle_cfg(arch)
    mask = th.zeros(L, n, 1)
    mask[:seed_len] = 1.0
    speech = ref_denoiser.speech_memory(sd_ref, ocfg, tuple(a.cpu() for a in z))
    eps = ref_denoiser.denoise(sd_ref, ocfg, x_t, t, speech=speech, inpaint_pose=poses.transpose(0, 1),
                               inpaint_mask=mask)
    want = ((eps - noise) ** 2).mean(dim=(1, 2)).mean()
    want.backward()
    loss = terms["loss"].item()
    assert abs(loss - want.item()) <= 1e-5 * want.item(), (loss, want.item())
    floor = 1e-4 * max(sd_ref[k].grad.abs().max().item() for k in names)
    worst = max(((model.params[k].grad.cpu() - sd_ref[k].grad).abs().max().item()
                 / max(sd_ref[k].grad.abs().max().item(), floor), k) for k in names)
    print("\ninpaint: worst gradient error", worst,
          "| proj.0.weight max|grad|", sd_ref["proj.0.weight"].grad.abs().max().item())
    assert sd_ref["proj.0.weight"].grad.abs().max().item() > 0
    assert worst[0] <= 2e-3, worst
    # one full Trainer step, then the checkpoint into the inpaint sampler (main.py:113-115)
    res = trainer.step({"pose": poses.cuda(), "speech_tokens": z}, noise=noise.cuda(), t=t.cuda())
    assert np.isfinite(res["loss"])
    trained = {k: v.cpu() for k, v in model.state_dict().items()}
    assert set(trained) == set(sd)
    assert not th.equal(trained["proj.0.weight"], sd["proj.0.weight"])
    sampler.load_state_dict(trained, strict=True)
    xs = th.randn(n, D_POSE, L, generator=g)
    ts = th.tensor([999, 500, 0])
    got = sampler(xs.cuda(), ts.cuda(), wav=wav.cuda(), inpaint_pose=poses.transpose(0, 1).cuda(),
                  inpaint_mask=mask.cuda()).cpu()
    ref = ref_denoiser.OracleModel(trained, ocfg, cache_speech=True)(xs, ts, wav=wav, inpaint_pose=poses.transpose(0, 1),
                                                                       inpaint_mask=mask)
    assert (got - ref).abs().max().item() <= 1e-4


def test_twoway_decoder_training_gradients_match_oracle_and_checkpoint_samples(pkg, beat_cfg, tr):
    """The two-way CrossAttention decoder (nn.py:381-447, the tedexp configuration's decoder) trained
    under the default model (memory concat on time, model.py:41-73): one step's loss and every
    gradient -- the memory stream's self-attention / feed-forward, the joint attention, the last
    layer without feed_forward_mem -- against torch autograd through the oracle's twoway_decoder;
    then a Trainer step's checkpoint loads strictly into the two-way sampler and its eps matches the
    oracle on the trained weights."""
    cfg = beat_cfg.Model.to_dict()
    cfg = dict(cfg, type="default", Decoder=dict(cfg["Decoder"], type="cross_attention", n_layers=2))
    arch = pkg.arch_from_config(cfg, D_POSE)
    assert arch["decoder"] == "cross_attention" and arch["type"] == "default"
    sd = pkg.init_state_dict(arch, seed=0, perturb=True)
    assert "pose_decoder.layers.0.feed_forward_mem.layer1.weight" in sd
    assert "pose_decoder.layers.1.feed_forward_mem.layer1.weight" not in sd   # last layer (nn.py:408-418)
    g = th.Generator().manual_seed(61)
    sampler, _, _, _, _ = pkg.create_model(D_POSE, cfg, dtype="f32", device="cuda:0")
    sampler.load_state_dict(sd)
    n = 2
    wav = th.randn(n, WAV, generator=g) * 0.1
    z = sampler.encoder()(wav.cuda())
    diffusion = pkg.create_diffusion(beat_cfg.Model.Diffusion.to_dict(), True)
    model = tr.TrainableModel(arch, sd, "cuda")
    assert "pose_decoder.layers.0.self_attn_mem.output.weight" in model.params
    trainer = tr.Trainer(model, diffusion, None, lr=1e-3, weight_decay=0.0)
    x0 = th.randn(n, D_POSE, L, generator=g)
    t = th.tensor([811, 40])
    noise = th.randn(n, D_POSE, L, generator=g)
    model.zero_grad()
    out = tr.training_losses(diffusion, model, x0.cuda(), t.cuda(), {"speech_tokens": z}, noise=noise.cuda())
    loss = out["mse"].mean()
    loss.backward()
    names = list(model.params)
    sd_ref = {k: v.detach().float().clone() for k, v in sd.items()}
    for k in names:
        sd_ref[k].requires_grad_(True)
    want = _oracle_loss(arch, sd_ref, diffusion, x0, t, noise, tuple(a.cpu() for a in z))
    want.backward()
    assert abs(loss.item() - want.item()) <= 1e-5 * want.item(), (loss.item(), want.item())
    floor = 1e-4 * max(sd_ref[k].grad.abs().max().item() for k in names)
    worst = sorted(((model.params[k].grad.cpu() - sd_ref[k].grad).abs().max().item()
                    / max(sd_ref[k].grad.abs().max().item(), floor), k) for k in names)[::-1]
    print("\ntwo-way: worst gradient errors", worst[:4])
    assert sd_ref["pose_decoder.layers.0.feed_forward_mem.layer2.weight"].grad.abs().max().item() > 0
    assert worst[0][0] <= 2e-3, worst[:4]
    res = trainer.step({"pose": x0.transpose(1, 2).cuda(), "speech_tokens": z}, noise=noise.cuda(), t=t.cuda())
    assert np.isfinite(res["loss"])
    trained = {k: v.cpu() for k, v in model.state_dict().items()}
    assert set(trained) == set(sd)
    sampler.load_state_dict(trained, strict=True)
    xs = th.randn(n, D_POSE, L, generator=g)
    ts = th.tensor([999, 0])
    got = sampler(xs.cuda(), ts.cuda(), wav=wav.cuda()).cpu()
    ref = ref_denoiser.OracleModel(trained, oracle_cfg(arch), cache_speech=True)(xs, ts, wav=wav)
    assert (got - ref).abs().max().item() <= 1e-4
