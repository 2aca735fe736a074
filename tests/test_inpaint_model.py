"""CPU checks of the Speech2GestureModelInpaint surface (Model.type "inpaint", models/model.py:118-166)."""
import pytest
import torch as th

from oracle import ref_denoiser
from tests.conftest import oracle_cfg


@pytest.fixture(scope="module")
def archs(pkg, beat_cfg):
    mp = beat_cfg.Model.to_dict()
    out = {}
    for ty in ("default", "inpaint"):
        mp["type"] = ty
        out[ty] = pkg.arch_from_config(mp, 123)
    return out


def test_inpaint_parameter_count(pkg, archs):
    """proj = Linear(C+1, d) + Linear(d, d) + Linear(d, C) on top of the default model (model.py:135-142)."""
    d, C = 256, 123
    n_def = sum(th.Size(s).numel() for s, _ in pkg.parameter_shapes(archs["default"]).values())
    n_inp = sum(th.Size(s).numel() for s, _ in pkg.parameter_shapes(archs["inpaint"]).values())
    assert n_inp - n_def == (C + 1) * d + d + d * d + d + d * C + C


def test_zero_initialised_projection_is_identity(pkg, archs):
    """GLIDE zero init (model.py:144-151): a freshly built inpaint model equals the default model."""
    sd = pkg.init_state_dict(archs["inpaint"], seed=0)
    assert all(float(sd[k].abs().max()) == 0.0 for k in sd if k.startswith("proj."))
    g = th.Generator().manual_seed(3)
    x, t = th.randn(2, 123, 40, generator=g), th.tensor([5, 700])
    wav = th.randn(2, 32000, generator=g) * 0.1
    pose, mask = th.randn(40, 2, 123, generator=g), th.ones(40, 2, 1)
    a = ref_denoiser.OracleModel(sd, oracle_cfg(archs["inpaint"]), cache_speech=True)(
        x, t, wav=wav, inpaint_pose=pose, inpaint_mask=mask)
    sd_def = {k: v for k, v in sd.items() if not k.startswith("proj.")}
    b = ref_denoiser.OracleModel(sd_def, oracle_cfg(archs["default"]), cache_speech=True)(x, t, wav=wav)
    assert th.equal(a, b)
