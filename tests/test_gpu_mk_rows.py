"""The clip-group persistent loops' KE by frame rows (ggd_phases.h ker_phase, round 4; ggd_rows.hip ke_rows).

Workgroup p of a clip updates frames [p L / 8, (p + 1) L / 8) and computes their next-step layer-0
rows (emb_x + PE); the Philox quads stay in the reference's (C, L) element order, so a quad can
straddle two frame blocks (L = 34, 38: blocks of 4 and 5 frames) and, when L % 4 != 0, two
channels.  Whole short trajectories on the counter-noise stream (no injected noise: the Philox
draws are the kernel's own) against oracle/ref_diffusion.py with oracle/philox.py, and the XCD-local
launch must have run (GGD_INFO_XL_LAUNCHES), i.e. not a fallback route.
(models/modules/gaussian_diffusion.py:300-412, models/model.py:12-15.)
"""
import ctypes

import numpy as np
import pytest
import torch as th

from oracle import ref_denoiser, ref_diffusion
from tests.conftest import oracle_cfg

pytestmark = pytest.mark.gpu

D_POSE = 123
ROUTE_PER_CLIP = 0
INFO_XL_LAUNCHES, INFO_ROWS_LOOP = 3, 9


def rel_rms(a, b):
    return (((a - b) ** 2).mean().sqrt() / (b ** 2).mean().sqrt()).item()


@pytest.fixture(scope="module")
def weights(pkg, beat_cfg):
    arch = pkg.arch_from_config(beat_cfg.Model, D_POSE)
    return arch, pkg.init_state_dict(arch, seed=0, perturb=True)


# bf16: the row-block loop (ggd_rows.hip; rows = 1), f32: the head / chunk loop (ggd_mega.hip; rows = 0).
# L = 38 / 44: blocks of 4 and 5 / 5 and 6 frames; L = 56: 4 row tiles and 45 memory keys (two more key
# tiles in the row-block cross-attention; the LDS-DMA'd out-projection share clamped to what fits)
@pytest.mark.parametrize("dtype,L,n,rows", [("f32", 34, 2, 0), ("bf16", 38, 3, 1), ("bf16", 40, 2, 1),
                                            ("bf16", 44, 2, 1), ("bf16", 56, 2, 1), ("bf16", 64, 2, 1)])
def test_frame_block_update_matches_oracle(pkg, beat_cfg, weights, dtype, L, n, rows):
    arch, sd = weights
    model, diffusion, _, _, _ = pkg.create_model(D_POSE, beat_cfg.Model, dtype=dtype, device="cuda:0")
    model.load_state_dict(sd)
    wav = th.randn(n, 16000 * L // 20, generator=th.Generator().manual_seed(L)) * 0.1
    seed, off, steps = 77, 3, 3
    ctx, _ = model.prepare(wav.cuda(), L)
    try:
        assert ctx.lib.ggd_set_route(ctx.h, ROUTE_PER_CLIP, 1) == 0   # never the per-clip loops
        out = diffusion.p_sample_loop(model, (n, D_POSE, L), {"wav": wav.cuda()}, seed=seed, clip_offset=off,
                                      n_steps=steps, sync=True)["sample"].cpu()
        v = ctypes.c_double()
        assert ctx.lib.ggd_route_info(ctx.h, INFO_XL_LAUNCHES, ctypes.cast(ctypes.byref(v), ctypes.c_void_p)) == 0
        assert v.value >= 1, "the clip-group loop did not run"
        assert ctx.lib.ggd_route_info(ctx.h, INFO_ROWS_LOOP, ctypes.cast(ctypes.byref(v), ctypes.c_void_p)) == 0
        assert int(v.value) == rows
    finally:
        ctx.lib.ggd_set_route(ctx.h, ROUTE_PER_CLIP, 0)
    om = ref_denoiser.OracleModel(sd, oracle_cfg(arch), cache_speech=True)
    sch = ref_diffusion.make_schedule("linear", 1000, "")
    noise = ref_diffusion.PhiloxNoise(seed, np.arange(off, off + n))
    want = ref_diffusion.sample_loop(sch, om, (n, D_POSE, L), {"wav": wav}, noise, "ddpm", n_steps=steps)["sample"]
    if dtype == "f32":
        assert (out - want).abs().max().item() <= 1e-3
    else:   # a missed or misplaced element would be off by about one step's noise (sigma ~ 0.14)
        assert rel_rms(out, want) <= 2e-2 and (out - want).abs().max().item() <= 0.1
