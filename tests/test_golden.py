"""Golden vectors (tests/golden/beat_c2_small.npz, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces its committed vectors (drift guard; the reference itself
cannot be run -- SURVEY.md 8c -- so these pin the restatement, "parity unpinned" against the
reference's own numerics).  GPU: the HIP path (f32 parity mode, through libggd's C ABI) against
the same vectors: eps max|diff| <= 1e-4, 5 DDPM / DDIM steps on the counter noise <= 1e-3.
"""
import os

import numpy as np
import pytest
import torch as th

from oracle import philox, ref_diffusion
from tests.golden import make_golden as mg

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "beat_c2_small.npz"))


def test_inputs_regenerate():
    wav, x, t = mg.inputs()
    assert np.array_equal(wav[:, :256].numpy(), GOLD["wav_head"])
    assert np.array_equal(x.numpy(), GOLD["x"]) and np.array_equal(t.numpy(), GOLD["t"])


def test_noise_and_schedule_vectors():
    z = philox.clip_noise(3, [5], 0, philox.TAG_XT, mg.D_POSE, mg.L)[0, :4]
    assert np.array_equal(z, GOLD["noise_xT_clip5"])
    z = philox.clip_noise(3, [0, 1], 7, philox.TAG_STEP, mg.D_POSE, mg.L)[:, :2]
    assert np.array_equal(z, GOLD["noise_step7_clips01"])
    sch = ref_diffusion.make_schedule("linear", 1000, "")
    assert np.array_equal(np.asarray(sch.posterior_mean_coef1[[0, 1, 500, 999]]), GOLD["sched_coef1"])
    assert np.array_equal(np.asarray(sch.posterior_log_variance_clipped[[0, 1, 500, 999]]), GOLD["sched_logvar"])


def test_oracle_eps_and_steps_reproduce(pkg):
    _, _, om = mg.build(pkg)
    res = mg.compute(om)
    for k in ("eps", "ddpm5_sample", "ddim5_sample", "ddpm5_pred_x_start"):
        np.testing.assert_allclose(res[k], GOLD[k], rtol=1e-5, atol=1e-5, err_msg=k)


@pytest.mark.gpu
def test_hip_f32_matches_golden(pkg, beat_cfg):
    arch, sd, _ = mg.build(pkg)
    model, diffusion, _, _, _ = pkg.create_model(mg.D_POSE, beat_cfg.Model, dtype="f32", device="cuda:0")
    model.load_state_dict(sd)
    wav, x, t = mg.inputs()
    eps = model(x.cuda(), t.cuda(), wav=wav.cuda()).cpu().numpy()
    assert np.abs(eps - GOLD["eps"]).max() <= 1e-4
    for alg, loop in (("ddpm", diffusion.p_sample_loop), ("ddim", diffusion.ddim_sample_loop)):
        out = loop(model, (2, mg.D_POSE, mg.L), model_kwargs={"wav": wav.cuda()}, seed=3, clip_offset=0, n_steps=5)
        err = np.abs(out["sample"].cpu().numpy() - GOLD[f"{alg}5_sample"]).max()
        assert err <= 1e-3, (alg, err)
