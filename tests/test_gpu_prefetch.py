"""Speech-encoder prefetch on a side HIP stream (model.prefetch_speech / Generator.generate_batches):
outputs must equal the inline-encoded calls bit for bit (same kernels, only the stream differs)."""
import os

import pytest
import torch as th

import __graft_entry__ as ge

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_generate_batches_matches_generate_sample():
    pkg = ge.load_package()
    cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
    model, _, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device="cuda:0")
    model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
    diffusion = pkg.create_diffusion(dict(cfg.Model.Diffusion, timestep_respacing="ddim10"), False)
    gen = pkg.Generator(model, diffusion)
    g = th.Generator(device="cuda:0").manual_seed(7)
    wavs = [th.randn(6, 32000, device="cuda:0", generator=g) * 0.1 for _ in range(3)]
    shape = (6, 123, 40)
    outs = gen.generate_batches(shape, wavs, sample_alg="ddim", device="cuda:0", seed=11)
    th.cuda.synchronize()
    model._release()  # fresh contexts: no cached speech memory
    for wav, out in zip(wavs, outs):
        ref = gen.generate_sample(shape, wav, sample_alg="ddim", device="cuda:0", progress=False, seed=11)
        assert th.equal(out, ref)


@pytest.mark.gpu
def test_prefetch_out_of_order_and_inline_calls():
    """A prefetched batch sampled after an inline-encoded one (the inline encoder waits for the
    side stream: both share the encoder context's buffers)."""
    pkg = ge.load_package()
    cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
    model, _, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device="cuda:0")
    model.load_state_dict(pkg.init_state_dict(model.arch, seed=0))
    diffusion = pkg.create_diffusion(dict(cfg.Model.Diffusion, timestep_respacing="ddim5"), False)
    gen = pkg.Generator(model, diffusion)
    g = th.Generator(device="cuda:0").manual_seed(9)
    w1, w2 = (th.randn(4, 32000, device="cuda:0", generator=g) * 0.1 for _ in range(2))
    shape = (4, 123, 40)
    model.prefetch_speech(w2)
    o1 = gen.generate_sample(shape, w1, device="cuda:0", progress=False, seed=3)  # inline encode
    o2 = gen.generate_sample(shape, w2, device="cuda:0", progress=False, seed=3)  # prefetched
    th.cuda.synchronize()
    assert not model._pending
    model._release()
    assert th.equal(o1, gen.generate_sample(shape, w1, device="cuda:0", progress=False, seed=3))
    assert th.equal(o2, gen.generate_sample(shape, w2, device="cuda:0", progress=False, seed=3))


@pytest.mark.gpu
def test_prefetch_beside_persistent_loop_matches_oracle():
    """The next batch's encoder on the side stream WHILE the clip-group persistent loop runs
    (C2 shape, 32 clips: the loop needs every one of its 256 workgroups resident, the encoder's
    kernels hold CUs meanwhile).  One non-blocking run: no status error (ggd_sync), the output
    equals the run without the prefetch bit for bit, and eps / the sample match the oracle."""
    import numpy as np
    from oracle import ref_denoiser, ref_diffusion
    from tests.conftest import oracle_cfg
    pkg = ge.load_package()
    cfg = pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))
    model, diffusion, _, _, _ = pkg.create_model(123, cfg.Model, dtype="bf16", device="cuda:0")
    sd = pkg.init_state_dict(model.arch, seed=0, perturb=True)
    model.load_state_dict(sd)
    n, L, steps = 32, 40, 6
    g = th.Generator().manual_seed(13)
    w1, w2 = (th.randn(n, 32000, generator=g) * 0.1 for _ in range(2))
    x = th.randn(n, 123, L, generator=g)
    zs = th.randn(steps, n, 123, L, generator=g)
    w1d, w2d, xd, zd = w1.cuda(), w2.cuda(), x.cuda(), zs.cuda()
    run = lambda pre: diffusion.p_sample_loop(model, (n, 123, L), {"wav": w1d}, noise=xd, step_noise=zd,
                                              n_steps=steps, prefetch_wav=pre)
    with_pre = run(w2d)
    model.sync()                                   # raises if the loop reported a status error
    assert len(model._pending) == 1                # w2's tokens wait for their sampling call
    model._release()
    plain = run(None)
    model.sync()
    for k in ("sample", "eps"):
        assert th.equal(with_pre[k], plain[k]), k
    ids = np.array([0, 17, 31])
    om = ref_denoiser.OracleModel(sd, oracle_cfg(model.arch), cache_speech=True)
    sch = ref_diffusion.make_schedule("linear", 1000, "")
    want = ref_diffusion.sample_loop(sch, om, (len(ids), 123, L), {"wav": w1[ids]},
                                     ref_diffusion.InjectedNoise(x[ids], zs[:, ids]), "ddpm", x_T=x[ids],
                                     n_steps=steps)
    rr = lambda a, b: (((a - b) ** 2).mean().sqrt() / (b ** 2).mean().sqrt()).item()
    assert rr(with_pre["eps"].cpu()[ids], want["eps"]) <= 1e-2
    assert rr(with_pre["sample"].cpu()[ids], want["sample"]) <= 5e-2
