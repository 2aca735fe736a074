"""CPU tests: config surface, host-side update math, and that libggd.so loads with every ABI symbol."""
import ctypes
import importlib
import os
import re

import numpy as np
import pytest
import torch as th

from tests.conftest import ROOT


def test_json_config_attribute_access(pkg, beat_cfg):
    assert beat_cfg.Model.d_model == 256
    assert beat_cfg.Model.Decoder.type == "oneway_cross_attention"
    assert beat_cfg.Meta.name == "beat-ours"
    with pytest.raises(KeyError):
        _ = beat_cfg.Model.no_such_key


def test_json_config_roundtrip(pkg, beat_cfg, tmp_path):
    p = tmp_path / "c.json"
    beat_cfg.dump(str(p))
    again = pkg.JsonConfig(str(p))
    assert again.to_dict() == beat_cfg.to_dict()


def test_legacy_schema_adapter(pkg, tedexp_cfg):
    m = tedexp_cfg.Model
    assert m.type == "default" and m.d_model == 512 and m.dropout_prob == 0.0
    assert m.Decoder.type == "cross_attention" and m.Decoder.heads == 8 and m.Decoder.n_layers == 10
    assert m.Diffusion.diffusion_steps == 1000 and m.Diffusion.model_var_type == "fixed_small"
    assert m.Generate.pose_seed_len == 4
    raw = pkg.JsonConfig(os.path.join(ROOT, "configs", "tedexp-ours.json"))
    with pytest.raises(KeyError):
        _ = raw.Model.d_model  # the reference's create_model fails exactly here (model_creation.py:66)


def test_create_model_surface(pkg, beat_cfg, tedexp_cfg):
    out = pkg.create_model(123, beat_cfg.Model)
    assert len(out) == 5
    model, diffusion = out[:2]
    assert diffusion.num_timesteps == 1000 and diffusion.timestep_map[-1] == 999
    assert model.arch["n_layers"] == 4
    model2, _, _, _, _ = pkg.create_model(126, tedexp_cfg.Model)  # legacy params accepted
    assert model2.arch["decoder"] == "cross_attention"
    with pytest.raises(ValueError):
        pkg.create_model(123, dict(beat_cfg.Model.to_dict(), type="unet"))
    with pytest.raises(ValueError):   # the training path runs on the GPU only (no CPU fallback)
        pkg.create_model(123, beat_cfg.Model, is_training=True, device="cpu")
    with pytest.raises(ValueError):   # and rejects model types the reference does not have
        pkg.create_model(123, dict(beat_cfg.Model.to_dict(), type="unet"), is_training=True, device="cuda")


def test_load_state_dict_checks_names_and_shapes(pkg, beat_cfg):
    model, _, _, _, _ = pkg.create_model(123, beat_cfg.Model)
    sd = pkg.init_state_dict(model.arch, seed=0)
    model.load_state_dict(sd)
    bad = dict(sd)
    bad.pop("blend_layer.bias")
    with pytest.raises(RuntimeError):
        model.load_state_dict(bad)
    bad = dict(sd)
    bad["pose_decoder.emb_x.weight"] = th.zeros(3, 3)
    with pytest.raises(RuntimeError):
        model.load_state_dict(bad)


def test_generator_rejects_unknown_algorithm(pkg, beat_cfg):
    model, diffusion, _, _, _ = pkg.create_model(123, beat_cfg.Model)
    gen = pkg.Generator(model, diffusion)
    with pytest.raises(ValueError):
        gen._choose_sample_func("plms")
    with pytest.raises(ValueError):
        gen.tensor2dtype(th.zeros(1), "half")
    assert isinstance(gen.tensor2dtype(th.zeros(2), "array"), np.ndarray)


def test_inpaint_denoise_matches_reference_formula(pkg):
    """InpaintDenoise.__call__ == generator.py:272-281 on random data (oracle restatement)."""
    from oracle import ref_diffusion
    n, L, C = 2, 40, 5
    g = th.Generator().manual_seed(0)
    poses, x0 = th.randn(n, L, C, generator=g), th.randn(n, C, L, generator=g)
    masks = th.ones(n, L, 1)
    masks[:, 10:] = 0
    trans = ref_diffusion.trans_ramp(0.575, 10, L)
    assert trans.shape == (1, L, 1)
    want = ref_diffusion.make_denoise_fn(poses, masks, trans)(x0)
    got = pkg.InpaintDenoise(poses, masks, trans.reshape(L))(x0)
    assert th.equal(got, want)


def _header_symbols(diag=False):
    """Function declarations of include/ggd.h (comments stripped); the GGD_DIAG block only with diag."""
    txt = "".join(open(os.path.join(ROOT, "include", h)).read() for h in ("ggd.h", "ggd_train.h"))
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    if not diag:
        txt = re.sub(r"#ifdef GGD_DIAG.*?#endif", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ggd_[a-z0-9_]+)\s*\(", txt)))


def test_library_loads_and_exports_every_header_symbol(pkg):
    native = importlib.import_module(pkg.__name__ + ".native")
    if native.is_stale():
        native.build()
    lib = native.load()
    syms = _header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(native.EXPORTS)
    assert lib.ggd_version().decode().startswith("ggd")


def test_diagnostics_stay_out_of_the_product_library(pkg):
    """ggd_diag (microbenchmarks, stamps) is exported by libggd_diag.so only."""
    import ctypes
    native = importlib.import_module(pkg.__name__ + ".native")
    if native.is_stale():
        native.build()
    assert "ggd_diag" in _header_symbols(diag=True) and "ggd_diag" not in _header_symbols()
    assert not hasattr(ctypes.CDLL(native.PRODUCT_LIB), "ggd_diag")
    diag = ctypes.CDLL(native.DIAG_LIB)
    for s in _header_symbols(diag=True):
        assert hasattr(diag, s), s


def test_abi_struct_layouts_match_header(pkg, tmp_path):
    """Every field offset and the size of the ctypes mirrors equal what a C compiler makes of
    include/ggd.h (gcc on a generated probe)."""
    import subprocess
    native = importlib.import_module(pkg.__name__ + ".native")
    lines = []
    for cname, py in (("ggd_desc", native.Desc), ("ggd_sample_args", native.SampleArgs)):
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    src = tmp_path / "probe.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "ggd.h"\nint main(void) {\n' +
                   "\n".join(lines) + "\nreturn 0;\n}\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        s, f, v = line.split()
        got[(s, f)] = int(v)
    for cname, py in (("ggd_desc", native.Desc), ("ggd_sample_args", native.SampleArgs)):
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)


def test_null_context_is_an_argument_error(pkg):
    native = importlib.import_module(pkg.__name__ + ".native")
    lib = native.load()
    assert lib.ggd_create(0, None, None) == native.GGD_ERR_ARG
    assert lib.ggd_destroy(None) == native.GGD_OK
    assert lib.ggd_last_error(None) == b"null context"
