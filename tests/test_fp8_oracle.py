"""CPU checks of the fp8 e4m3fn restatement (oracle/fp8.py) the GGD_FP8W parity tests rely on.

Known answers are from the OCP 8-bit floating point specification's e4m3 table (bias 7, no
infinities, max 448 = 0x7e, NaN 0x7f, min subnormal 2^-9 = 0x01, min normal 2^-6 = 0x08)."""
import numpy as np
import torch as th

from oracle import fp8

KAT = [(0.0, 0x00), (1.0, 0x38), (-1.0, 0xB8), (448.0, 0x7E), (-448.0, 0xFE), (2.0 ** -9, 0x01),
       (2.0 ** -6, 0x08), (1.125, 0x39), (1.75, 0x3E), (0.5, 0x30), (240.0, 0x77), (3.0, 0x44)]


def test_e4m3_known_answers():
    x = np.array([v for v, _ in KAT], np.float32)
    codes = fp8.e4m3_encode(x)
    assert [int(c) for c in codes] == [c for _, c in KAT]
    np.testing.assert_array_equal(fp8.e4m3_decode(codes), x)


def test_e4m3_rounding_and_saturation():
    # ties to even: 1.0625 sits between 1.0 (m=0) and 1.125 (m=1) -> 1.0; 1.1875 -> 1.25 (m=2)
    got = fp8.e4m3_decode(fp8.e4m3_encode(np.array([1.0625, 1.1875, 500.0, 1e9, -1e9, 2.0 ** -11], np.float32)))
    np.testing.assert_array_equal(got, np.array([1.0, 1.25, 448.0, 448.0, -448.0, 0.0], np.float32))
    assert fp8.e4m3_encode(np.array([np.nan], np.float32))[0] == 0x7F


def test_e4m3_roundtrip_all_codes():
    codes = np.array([c for c in range(256) if (c & 0x7F) != 0x7F], np.uint8)
    vals = fp8.e4m3_decode(codes)
    back = fp8.e4m3_encode(vals)
    # +0 / -0 both decode to zero; every other code round-trips exactly
    np.testing.assert_array_equal(back[vals != 0], codes[vals != 0])


def test_quantize_rows_error_bound():
    g = th.Generator().manual_seed(0)
    w = (th.randn(64, 256, generator=g) * 0.05).numpy()
    codes, scale, deq = fp8.quantize_rows(w)
    assert codes.dtype == np.uint8 and scale.shape == (64,)
    assert np.abs(deq).max(axis=1).round(6).tolist() == np.abs(w).max(axis=1).round(6).tolist()  # amax exact
    rel = np.sqrt(((deq - w) ** 2).mean() / (w ** 2).mean())
    assert rel < 0.04, rel      # 3 mantissa bits: ~2-3 % RMS relative error


def test_step_linear_selection(pkg, beat_cfg):
    arch = pkg.arch_from_config(beat_cfg.Model, 123)
    sd = pkg.init_state_dict(arch, seed=0)
    names = fp8.step_linear_names(sd)
    # per layer: q, k, v, SA out, CA q, CA out, FFN 1, FFN 2 -> 8; plus emb_x and out_layers.1
    assert len(names) == 8 * arch["n_layers"] + 2
    assert not any("cross_attn.key" in n or "cross_attn.value" in n for n in names)
    dq = fp8.dequantized_state_dict(sd)
    assert set(dq) == set(sd)
    for k in names:
        assert not th.equal(dq[k], sd[k])


def test_mx_e4m3_blocks():
    """MX activations (the fp8-MFMA long loop's quantiser, ggd_chainlib.h mx_scale_byte / mx_mul):
    per 32-value block the max lands in [128, 256) (scale 2^(E - 7)), powers of two and small
    integers times the scale survive exactly, every value keeps e4m3's 2^-4 relative step, an
    all-zero block stays zero and blocks do not see each other's scale."""
    g = th.Generator().manual_seed(3)
    x = th.randn(6, 96, generator=g) * th.tensor([1e-3, 1.0, 300.0]).repeat_interleave(32)
    y = fp8.mx_e4m3(x)
    rel = ((y - x).abs() / x.abs().clamp_min(1e-30))
    # normals of the block keep a 3-bit mantissa (round to nearest: <= 2^-4 relative); values below
    # max / 2^13 may go subnormal, the random data here has none
    assert float(rel.max()) <= 2.0 ** -4 + 1e-7
    blocks = x.reshape(6, 3, 32)
    m = blocks.abs().amax(-1)
    e = th.floor(th.log2(m))
    scaled = (blocks / (2.0 ** (e - 7))[..., None]).abs().amax(-1)
    assert bool(((scaled >= 128) & (scaled < 256)).all())
    z = th.zeros(2, 64)
    z[1, 32:] = th.tensor([2.0 ** k for k in range(-8, 24)])
    assert th.equal(fp8.mx_e4m3(z)[0], z[0])
    assert th.equal(fp8.mx_e4m3(z)[1, 32:][-14:], z[1, 32:][-14:])   # within 2^13 of the block max: exact
