"""Known-answer tests pinning the CPU oracle (and the package's host-side math) on CPU.

Pins: (1) structural numbers produced by the one reference import that ran
(parameter counts, speech-token lengths); (2) published Philox4x32-10
known-answer vectors (Random123 kat_vectors); (3) closed-form schedule values
(gaussian_diffusion.py:20-40,87-143; respace.py:13-68).
"""
import math

import numpy as np
import pytest
import torch as th

from oracle import philox, ref_denoiser, ref_diffusion
from tests.conftest import oracle_cfg


def test_parameter_counts_match_reference(pkg, beat_cfg):
    arch = pkg.arch_from_config(beat_cfg.Model, 123)
    sd = pkg.init_state_dict(arch, seed=0)
    assert pkg.count_parameters(sd) == 10_340_087
    assert pkg.count_parameters(sd, "speech_encoder.") == 5_665_148
    assert pkg.count_parameters(sd, "pose_decoder.") == 4_346_491
    assert pkg.count_parameters(sd, "blend_layer.") == 196_864
    assert pkg.count_parameters(sd, "diffusion_step_encoder.") == 131_584


@pytest.mark.parametrize("n_wav,lens", [(32000, (31, 30, 30)), (128000, (125, 124, 126)), (36266, (35, 34, 34))])
def test_speech_token_lengths(pkg, beat_cfg, n_wav, lens):
    arch = pkg.arch_from_config(beat_cfg.Model, 123)
    sd = pkg.init_state_dict(arch, seed=0)
    z = ref_denoiser.speech_encoder(sd, th.randn(1, n_wav) * 0.1)
    assert tuple(a.shape[1] for a in z) == lens
    enc = __import__("importlib").import_module(pkg.__name__ + ".encoder")
    assert enc.speech_len("s2g_v2", n_wav) == max(lens)
    assert enc.speech_len("default", n_wav) == sum(lens)


@pytest.mark.parametrize("ctr,key,want", [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox_known_answers(ctr, key, want):
    out = philox.philox4x32_10(np.array([ctr[0]], np.uint32), ctr[1], ctr[2], ctr[3], key[0], key[1])
    assert tuple(int(o[0]) for o in out) == want


def test_philox_normals_are_standard():
    z = philox.normal_block(123, np.arange(64), 7, philox.TAG_STEP, 4920)
    assert abs(float(z.mean())) < 0.01 and abs(float(z.std()) - 1) < 0.01
    z2 = philox.normal_block(123, np.arange(64), 8, philox.TAG_STEP, 4920)
    assert not np.array_equal(z, z2)
    # a clip's draws do not depend on which other clips are drawn with it
    z3 = philox.normal_block(123, np.arange(10, 12), 7, philox.TAG_STEP, 4920)
    assert np.array_equal(z3, z[10:12])


def test_linear_schedule_closed_form(pkg):
    b = ref_diffusion.named_betas("linear", 1000)
    assert b[0] == pytest.approx(1e-4) and b[-1] == pytest.approx(0.02)
    sch = ref_diffusion.make_schedule("linear", 1000, "")
    # alpha_bar_T of the Ho et al. linear schedule
    assert sch.alphas_cumprod[-1] == pytest.approx(4.0358e-05, rel=1e-3)
    assert sch.posterior_log_variance_clipped[0] == sch.posterior_log_variance_clipped[1]
    d = pkg.create_diffusion({"type": "gaussian", "noise_schedule": "linear", "diffusion_steps": 1000,
                              "timestep_respacing": "", "model_var_type": "fixed_small"}, False)
    for name in ("sqrt_recip_alphas_cumprod", "sqrt_recipm1_alphas_cumprod", "posterior_mean_coef1",
                 "posterior_mean_coef2", "posterior_log_variance_clipped", "posterior_variance"):
        np.testing.assert_array_equal(getattr(d, name), getattr(sch, name))


def test_respacing(pkg):
    s = ref_diffusion.spaced_steps(1000, "ddim50")
    assert s == set(range(0, 1000, 20))
    s50 = ref_diffusion.spaced_steps(1000, "50")
    assert len(s50) == 50 and min(s50) == 0 and max(s50) == 999
    assert len(ref_diffusion.spaced_steps(1000, "fast27")) == 27
    assert ref_diffusion.spaced_steps(300, "10,15,20") == pkg.space_timesteps(300, "10,15,20")
    with pytest.raises(ValueError):
        ref_diffusion.spaced_steps(10, "ddim7")
    sch = ref_diffusion.make_schedule("linear", 1000, "ddim50")
    assert sch.num_timesteps == 50 and sch.timestep_map[-1] == 980
    # respaced alphas_cumprod are the kept subset of the originals
    full = ref_diffusion.make_schedule("linear", 1000, "")
    np.testing.assert_allclose(sch.alphas_cumprod, full.alphas_cumprod[::20], rtol=1e-12)
    d = pkg.create_diffusion({"type": "gaussian", "noise_schedule": "linear", "diffusion_steps": 1000,
                              "timestep_respacing": "ddim50", "model_var_type": "fixed_small"}, False)
    np.testing.assert_array_equal(d.betas, sch.betas)
    assert d.timestep_map == sch.timestep_map


def test_step_embedding_and_pe():
    e = ref_denoiser.step_embedding(th.tensor([0, 7]), 256)
    assert th.allclose(e[0, :128], th.ones(128)) and th.allclose(e[0, 128:], th.zeros(128))
    assert e[1, 0].item() == pytest.approx(math.cos(7.0), abs=1e-6)
    pe = ref_denoiser.positional_table(256, 50)
    assert pe.shape == (50, 1, 256)
    assert pe[3, 0, 0].item() == pytest.approx(math.sin(3.0), abs=1e-6)
    assert pe[3, 0, 1].item() == pytest.approx(math.cos(3.0), abs=1e-6)


def test_mel_filterbank_htk(pkg):
    fb = ref_denoiser.mel_filterbank()
    assert fb.shape == (513, 128)
    assert (fb >= 0).all() and fb.max() <= 1.0 + 1e-6
    # every filter is a triangle with one peak
    assert ((fb > 0).sum(0) > 0).all()
    sd = pkg.init_state_dict(pkg.arch_from_config(
        {"type": "s2g_v2", "d_model": 256, "Decoder": {"type": "oneway_cross_attention", "heads": 8, "n_layers": 1}},
        123), seed=0)
    assert th.equal(sd["speech_encoder.wav2spec.1.mel_scale.fb"], fb)


def test_depthwise_conv_centered():
    """SpatialDepthWiseConv: out[i] = b + w0 x[i-1] + w1 x[i] + w2 x[i+1] (transformer.py:28-44)."""
    L, N, H, dk = 5, 2, 2, 4
    x = th.randn(L, N, H, dk)
    w = th.randn(dk, 1, 3)
    b = th.randn(dk)
    y = ref_denoiser._depthwise_seq_conv({"c.conv.weight": w, "c.conv.bias": b}, "c", x)
    xp = th.cat([th.zeros(1, N, H, dk), x, th.zeros(1, N, H, dk)])
    want = b + w[:, 0, 0] * xp[:-2] + w[:, 0, 1] * xp[1:-1] + w[:, 0, 2] * xp[2:]
    assert th.allclose(y, want, atol=1e-6)


def test_encoder_hoisting_is_exact(pkg, beat_cfg):
    """Recomputing the encoder each step (reference) == computing it once (the build)."""
    arch = pkg.arch_from_config(beat_cfg.Model, 123)
    sd = pkg.init_state_dict(arch, seed=0, perturb=True)
    cfg = oracle_cfg(arch)
    wav = th.randn(2, 32000) * 0.1
    x = th.randn(2, 123, 40)
    t = th.tensor([5, 900])
    a = ref_denoiser.OracleModel(sd, cfg, cache_speech=False)(x, t, wav=wav)
    b = ref_denoiser.OracleModel(sd, cfg, cache_speech=True)(x, t, wav=wav)
    assert th.equal(a, b)


@pytest.mark.parametrize("n_wav,lens", [(32000, (31, 30, 30)), (128000, (125, 124, 126)), (36266, (35, 34, 34))])
def test_hip_encoder_token_lengths(pkg, n_wav, lens):
    """ggd_enc_lengths (host-side geometry, no device call) against the structural KATs."""
    import ctypes
    native = __import__(pkg.__name__ + ".native", fromlist=["x"])
    lib = native.load()
    h = ctypes.c_void_p()
    assert lib.ggd_enc_create(0, 256, n_wav, 4, native.BF16, ctypes.byref(h)) == 0
    try:
        t = [ctypes.c_int32() for _ in range(3)]
        assert lib.ggd_enc_lengths(h, *[ctypes.byref(x) for x in t]) == 0
        assert tuple(x.value for x in t) == lens
        # a finalize without weights names the first missing tensor
        assert lib.ggd_enc_load_weight(h, b"pose_decoder.emb_x.weight", None, 0) == native.GGD_IGNORED
    finally:
        lib.ggd_enc_destroy(h)


def test_two_way_decoder_oracle_runs(pkg, tedexp_cfg):
    """Config C1 plumbing: tedexp (legacy schema) -> default model + two-way decoder on CPU."""
    arch = pkg.arch_from_config(tedexp_cfg.Model, 126)
    assert arch == {"type": "default", "d_model": 512, "decoder": "cross_attention", "heads": 8,
                    "n_layers": 10, "d_pose": 126}
    sd = pkg.init_state_dict(arch, seed=0)
    om = ref_denoiser.OracleModel(sd, oracle_cfg(arch), cache_speech=True)
    wav = th.randn(1, int(16000 * 34 / 15)) * 0.1
    sch = ref_diffusion.make_schedule("linear", 1000, "50")
    out = ref_diffusion.sample_loop(sch, om, (1, 126, 34), {"wav": wav}, ref_diffusion.TorchNoise(0), "ddpm",
                                    n_steps=2)
    assert out["sample"].shape == (1, 126, 34) and th.isfinite(out["sample"]).all()
