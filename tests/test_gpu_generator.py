"""The Generator drivers of models/generator.py on the HIP sampler, against the CPU oracle.

  * generate_sample called twice with two HOST wav batches of one shape (main.py:171-196 calls it
    once per test batch): each result must be that batch's own -- the speech-memory cache must
    never serve the previous batch's memory (the freed device copy's block is reused);
  * generate_sequence (generator.py:80-195): windows, seed-pose inpainting, cross-fade;
  * eval_infer_time_ddim (generator.py:47-78): timing harness contract.

f32 tolerance as the other f32 sampling tests: max|diff| <= 1e-3 after the steps run.
"""
import numpy as np
import pytest
import torch as th

from oracle import ref_denoiser, ref_diffusion
from tests.conftest import oracle_cfg

pytestmark = pytest.mark.gpu

D_POSE, L, WAV = 123, 40, 32000


@pytest.fixture(scope="module")
def setup(pkg, beat_cfg):
    arch = pkg.arch_from_config(beat_cfg.Model, D_POSE)
    sd = pkg.init_state_dict(arch, seed=0, perturb=True, bounded=True)
    om = ref_denoiser.OracleModel(sd, oracle_cfg(arch), cache_speech=False)
    model, diffusion, _, _, _ = pkg.create_model(D_POSE, beat_cfg.Model, dtype="f32", device="cuda:0")
    model.load_state_dict(sd)
    return model, diffusion, om, pkg.Generator(model, diffusion)


def test_generate_sample_two_host_batches(pkg, beat_cfg, setup):
    """Two calls, two host wavs of equal shape: outputs match the oracle each and differ.

    Whole DDIM-50 loops.  With random weights the speech moves the poses by ~6e-3 (max), so the
    tolerance here is 1e-4 (f32 HIP vs oracle measured ~1e-6 on this loop) and the two batches'
    oracle outputs must differ by more than 10x that: a stale memory fails the oracle check."""
    model, _, om, _ = setup
    diffusion = pkg.create_diffusion(dict(beat_cfg.Model.Diffusion.to_dict(), timestep_respacing="ddim50"), False)
    gen = pkg.Generator(model, diffusion)
    n, seed = 2, 17
    sch = ref_diffusion.make_schedule("linear", 1000, "ddim50")
    g = th.Generator().manual_seed(90)
    wav_a = th.randn(n, WAV, generator=g) * 0.1
    wav_b = th.randn(n, WAV, generator=g) * 0.1
    outs, wants = [], []
    for wav in (wav_a, wav_b):  # host tensors: each call makes (and frees) its own device copy
        got = gen.generate_sample((n, D_POSE, L), wav, sample_alg="ddim", device="cuda:0", progress=False,
                                  seed=seed).cpu()
        want = ref_diffusion.generate_sample(sch, om, (n, D_POSE, L), wav, ref_diffusion.PhiloxNoise(seed, np.arange(n)),
                                             sample_alg="ddim")
        err = (got - want).abs().max().item()
        assert err <= 1e-4, err
        outs.append(got)
        wants.append(want)
    assert (wants[0] - wants[1]).abs().max().item() > 1e-3  # different speech -> different poses
    assert (outs[0] - outs[1]).abs().max().item() > 1e-3


def test_model_protocol_two_host_batches(setup):
    """The same through the model protocol itself (per-step callers pass host wavs)."""
    model, _, om, _ = setup
    n = 2
    g = th.Generator().manual_seed(91)
    x = th.randn(n, D_POSE, L, generator=g)
    t = th.tensor([900, 12])
    for k in range(3):
        wav = th.randn(n, WAV, generator=g) * 0.1
        eps = model(x.cuda(), t.cuda(), wav=wav).cpu()
        ref = om(x, t, wav=wav)
        assert (eps - ref).abs().max().item() <= 1e-4, k


def test_prefetch_keyed_wav_is_pinned(setup):
    """A prefetched batch that is never sampled must not be served to a later tensor that
    lands at the same address."""
    model, _, om, _ = setup
    n = 2
    g = th.Generator().manual_seed(92)
    x = th.randn(n, D_POSE, L, generator=g)
    t = th.tensor([500, 3])
    w1 = (th.randn(n, WAV, generator=g) * 0.1).cuda()
    model.prefetch_speech(w1)
    del w1  # the pending entry keeps the block; a new tensor cannot reuse its address
    w2_host = th.randn(n, WAV, generator=g) * 0.1
    w2 = w2_host.cuda()
    eps = model(x.cuda(), t.cuda(), wav=w2).cpu()
    assert (eps - om(x, t, wav=w2_host)).abs().max().item() <= 1e-4
    model._pending.clear()


@pytest.mark.parametrize("with_init,smooth", [(True, True), (False, False), (True, False)])
def test_generate_sequence_vs_oracle(pkg, beat_cfg, setup, with_init, smooth):
    """3 windows of 40 frames (seed 10, stride 30) over a 5 s wav, reduced n_steps per window."""
    model, diffusion, om, gen = setup
    n, steps, seed, seed_len, tf = 2, 3, 23, 10, 0.575
    g = th.Generator().manual_seed(93)
    wav = th.randn(n, 80000, generator=g) * 0.1      # seq_len = 100 frames -> 3 windows
    init = th.randn(n, seed_len, D_POSE, generator=g) if with_init else None
    got = gen.generate_sequence(wav, 16000, D_POSE, 20, L, seed_len, smooth_trans=smooth, trans_factor=tf,
                                init_poses=init, sample_alg="ddim", batch_size=64, device="cuda:0",
                                progress=False, seed=seed, n_steps=steps).cpu()
    sch = ref_diffusion.make_schedule("linear", 1000, "")
    want = ref_diffusion.generate_sequence(sch, om, wav, 16000, D_POSE, 20, L, seed_len,
                                           lambda k: ref_diffusion.PhiloxNoise(seed, np.arange(n)),
                                           smooth_trans=smooth, trans_factor=tf, init_poses=init,
                                           sample_alg="ddim", n_steps=steps)
    assert got.shape == (n, 100, D_POSE) == want.shape
    err = (got - want).abs().max().item()
    assert err <= 1e-3, err


def test_generate_sequence_batches(setup):
    """batch_size smaller than the number of sequences: batches are independent and concatenated."""
    _, _, _, gen = setup
    n, steps, seed = 3, 2, 5
    wav = th.randn(n, 48000, generator=th.Generator().manual_seed(94)) * 0.1
    kw = dict(smooth_trans=True, trans_factor=None, init_poses=None, sample_alg="ddpm", device="cuda:0",
              progress=False, seed=seed, n_steps=steps)
    whole = gen.generate_sequence(wav, 16000, D_POSE, 20, L, 10, batch_size=64, **kw).cpu()
    split = gen.generate_sequence(wav, 16000, D_POSE, 20, L, 10, batch_size=2, **kw).cpu()
    assert whole.shape == (n, 60, D_POSE)
    # clip ids restart at 0 in each batch, so batch 2's clip 0 uses clip 0's noise: compare
    # batch 1 (clips 0, 1) exactly and batch 2 against a lone run of its sequence
    assert (split[:2] - whole[:2]).abs().max().item() <= 1e-5
    lone = gen.generate_sequence(wav[2:], 16000, D_POSE, 20, L, 10, batch_size=64, **kw).cpu()
    assert (split[2:] - lone).abs().max().item() <= 1e-5


def test_eval_infer_time_ddim(pkg, beat_cfg, setup):
    """generator.py:47-78: (mean_ms, std_ms) over timed DDIM loops of a respaced diffusion."""
    model, _, _, _ = setup
    diffusion = pkg.create_diffusion(dict(beat_cfg.Model.Diffusion.to_dict(), timestep_respacing="ddim50"), False)
    gen = pkg.Generator(model, diffusion)
    wav = (th.randn(1, WAV, generator=th.Generator().manual_seed(95)) * 0.1).cuda()
    mean_ms, std_ms = gen.eval_infer_time_ddim((1, D_POSE, L), {"wav": wav}, repetitions=3, device="cuda:0")
    assert np.isfinite(mean_ms) and mean_ms > 0 and std_ms >= 0
    with pytest.raises(ValueError):
        gen.eval_infer_time_ddim((1, D_POSE, L), {"wav": wav}, sample_alg="bogus", repetitions=1)


def test_eval_bpd_matches_oracle_f32(pkg, beat_cfg):
    """Generator.eval_bpd -> calc_bpd_loop (generator.py:197-216, gaussian_diffusion.py:571-678) on the
    HIP denoiser (f32) against the oracle restatement, identical per-t noise; respaced to 20 steps
    so the oracle finishes in seconds.  Tolerance: total / prior bpd and every vb / mse term rel <= 1e-3."""
    from oracle import ref_denoiser, ref_diffusion
    from tests.conftest import oracle_cfg
    arch = pkg.arch_from_config(beat_cfg.Model, 123)
    sd = pkg.init_state_dict(arch, seed=0, perturb=True)
    model, _, _, _, _ = pkg.create_model(123, beat_cfg.Model, dtype="f32", device="cuda:0")
    model.load_state_dict(sd)
    diffusion = pkg.create_diffusion(dict(beat_cfg.Model.Diffusion.to_dict(), timestep_respacing="20"), False)
    gen = pkg.Generator(model, diffusion)
    g = th.Generator().manual_seed(31)
    n = 2
    poses = th.randn(n, 40, 123, generator=g) * 0.5
    wavs = th.randn(n, 32000, generator=g) * 0.1
    noise = th.randn(diffusion.num_timesteps, n, 123, 40, generator=g)
    got = gen.eval_bpd(poses.cuda(), wavs.cuda(), noise=noise.cuda())
    om = ref_denoiser.OracleModel(sd, oracle_cfg(arch), cache_speech=True)
    sch = ref_diffusion.make_schedule("linear", 1000, "20")
    want = ref_diffusion.calc_bpd_loop(sch, om, poses.transpose(1, 2), {"wav": wavs}, noise)
    for k in ("total_bpd", "prior_bpd", "vb", "x_start_mse", "mse"):
        a, b = got[k].cpu(), want[k]
        assert a.shape == b.shape, k
        err = ((a - b).abs() - 1e-3 * b.abs() - 1e-5 * b.abs().max()).max().item()
        assert err <= 0, (k, (a - b).abs().max().item(), b.abs().max().item())
