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
