"""Block-scaled fp8 (MX) MFMA arithmetic pinned value by value (ggd_mx_linear, ggd_mx_layernorm,
include/ggd.h).  ggd_mx_layernorm runs the long loop's own LayerNorm-into-MX device function
(lk_layernorm_mx: the block -> lane map, the 8-lane block max, the scale byte, the packing order);
ggd_mx_linear the quantiser and the MFMA chunk of its MX stages.

The long-clip loop's GGD_ROUTE_FP8_MFMA stages (csrc/ggd_long.hip over ggd_chainlib.h mx_scale_byte /
mx_mul / mx_pack4 / ch_mma_mx) quantise activations to e4m3 with one e8m0 scale per 32 values and
multiply them with per-channel e4m3 weights.  Model-level tests (test_gpu_fullsize.py) can only bound
that route's drift from the f32 oracle; this one runs the same device functions on one Linear and
compares with the numpy restatement (oracle/fp8.py mx_e4m3, e4m3_decode) in float64.
  * The quantisation itself is pinned bit for bit (identity weights: out = the quantised values).
  * The Linear: products of two e4m3 values scaled by powers of two are exact, so what is left is the
    block-scaled MFMA's own accumulation.  Measured on MI355X (gpurun_out r05k, 9 cases): max error
    3e-6 .. 6.5e-6 relative to sum |a_q| |w_q| when the row's blocks share a magnitude, up to 3.3e-5
    when they span 2^32 -- the instruction's internal sum is narrower than an f32 chain.  Tolerance
    2e-5 (same-magnitude blocks) / 1e-4 (2^32 spread), still 600x below one e4m3 code step (2^-4).
"""
import numpy as np
import pytest
import torch as th

from oracle import fp8

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib(pkg):
    from importlib import import_module
    native = import_module(pkg.__name__ + ".native")
    return native.load()


def run(lib, a, codes, scale, bias):
    M, K = a.shape
    N = codes.shape[0]
    ad, cd, sd, bd = a.cuda(), th.from_numpy(codes).cuda(), th.from_numpy(scale).cuda(), bias.cuda()
    out = th.full((M, N), float("nan"), device="cuda")
    rc = lib.ggd_mx_linear(M, N, K, ad.data_ptr(), cd.data_ptr(), sd.data_ptr(), bd.data_ptr(), out.data_ptr(), None)
    assert rc == 0, rc
    return out.cpu()


@pytest.mark.parametrize("spread", [0, 4, 32])
@pytest.mark.parametrize("M,N,K", [(32, 64, 256), (45, 128, 1024), (96, 192, 512)])
def test_mx_linear_matches_the_restated_quantisation(lib, M, N, K, spread):
    g = th.Generator().manual_seed(M + N + K)
    # rows whose 32-value blocks differ in magnitude by up to 2^spread (MX scales across the row),
    # zero blocks, tiny values that land in e4m3's subnormal range inside a block with a large max
    lo = -(spread * 5) // 8
    e = th.randint(lo, lo + spread + 1, (M, K // 32, 1), generator=g).float()
    a = th.randn(M, K, generator=g) * th.exp2(e).expand(M, K // 32, 32).reshape(M, K)
    a[0, :32] = 0.0
    a[1, 32:64] *= th.exp2(-th.arange(32).float())
    w = (th.randn(N, K, generator=g) * 0.05).numpy()
    codes, scale, _ = fp8.quantize_rows(w)
    bias = th.randn(N, generator=g)
    got = run(lib, a, codes, scale, bias).double()
    aq = fp8.mx_e4m3(a).double()
    wq = th.from_numpy(fp8.e4m3_decode(codes)).double()
    acc = aq @ wq.t()
    want = acc * th.from_numpy(scale).double() + bias.double()
    mag = aq.abs() @ wq.abs().t() * th.from_numpy(scale).double() + bias.double().abs()
    err = ((got - want).abs() / mag.clamp_min(1e-30)).max().item()
    print(f"mx_linear {M}x{N}x{K} spread {spread}: max rel err {err:.2e}")
    assert err <= (1e-4 if spread > 4 else 2e-5), err


def test_mx_quantisation_is_bit_exact(lib):
    """Identity e4m3 weights (code 0x38 = 1.0, scale 1, bias 0): out = the quantised activations
    themselves, so every value of mx_e4m3 is compared bit for bit -- subnormal e4m3 codes, zero
    blocks, round-to-nearest-even ties, and blocks whose max sits on a power of two."""
    K = 256
    g = th.Generator().manual_seed(11)
    rows = [th.randn(K, generator=g) * th.exp2(th.randint(-20, 12, (K // 32, 1), generator=g).float()).expand(
        K // 32, 32).reshape(K) for _ in range(24)]
    ramp = th.exp2(-th.arange(K).float() / 16.0) * 3.0           # every exponent a block spans, subnormals
    ties = (th.arange(K).float() % 32 + 0.5) / 4.0 * 2.0 ** -3     # exact e4m3 midpoints
    pow2 = th.where(th.arange(K) % 32 == 0, 256.0, 1.0 + th.arange(K).float() % 32 / 64.0)
    a = th.stack(rows + [ramp, -ramp, ties, -ties, pow2, th.zeros(K), ramp * 2.0 ** -100, ties * 2.0 ** 60])
    codes = np.where(np.eye(K, dtype=bool), 0x38, 0).astype(np.uint8)
    got = run(lib, a, codes, np.ones(K, np.float32), th.zeros(K))
    want = fp8.mx_e4m3(a)
    bad = (got != want).nonzero()
    for r, k in bad[:12].tolist():
        print(f"row {r} k {k}: in {a[r, k].item():.9g} gpu {got[r, k].item():.9g} oracle {want[r, k].item():.9g}")
    assert bad.shape[0] == 0, bad.shape[0]


def test_mx_linear_rejects_bad_shapes(lib):
    for M, N, K in ((32, 64, 128), (32, 60, 256), (0, 64, 256), (32, 64, 2048)):
        assert lib.ggd_mx_linear(M, N, K, 1, 1, 1, 1, 1, None) == -1


def test_mx_layernorm_scales_exact_and_codes_within_rounding(lib):
    """The long loop's LayerNorm into its MX A image (lk_layernorm_mx, ggd_mx_layernorm) against a
    float64 restatement: LN (two-pass statistics, eps 1e-5, nn.py:141-147) then per (row, 32
    columns) the block max -> e8m0 scale 2^(E - 7) and e4m3 codes of y / scale.  The kernel's f32
    statistics differ from float64 in the last bits, so: every scale byte equal unless the block max
    sits within 1e-5 of a power of two; every code equal unless y / scale sits within 1e-5 relative of
    an e4m3 rounding boundary (then one code step apart) -- which pins the block -> lane map, the
    scale choice and the packing order of the stage."""
    g = th.Generator().manual_seed(5)
    rows = th.randn(32, 256, generator=g) * th.exp2(th.randint(-6, 6, (32, 1), generator=g).float()) + \
        th.randn(32, 1, generator=g) * 3.0
    gamma = th.randn(256, generator=g) * th.exp2(th.randint(-3, 3, (256,), generator=g).float())
    beta = th.randn(256, generator=g) * 0.5
    codes = th.zeros(32, 256, dtype=th.uint8, device="cuda")
    scales = th.zeros(32, 8, dtype=th.uint8, device="cuda")
    rd, gd, bd = rows.cuda(), gamma.cuda(), beta.cuda()
    assert lib.ggd_mx_layernorm(rd.data_ptr(), gd.data_ptr(), bd.data_ptr(), codes.data_ptr(), scales.data_ptr(),
                                None) == 0
    codes, scales = codes.cpu().numpy(), scales.cpu().numpy()
    x = rows.double().numpy()
    mu = x.mean(1, keepdims=True)
    var = ((x - mu) ** 2).mean(1, keepdims=True)
    y = (x - mu) / np.sqrt(var + 1e-5) * gamma.double().numpy() + beta.double().numpy()
    yb = y.reshape(32, 8, 32)
    m = np.abs(yb).max(-1)
    e = np.floor(np.log2(m))
    want_sb = np.clip(e + 127 - 7, 2, 253).astype(np.int64)
    near_pow2 = np.abs(m / np.exp2(e) - 1.0) < 1e-5
    bad_sb = (scales.astype(np.int64) != want_sb) & ~near_pow2
    assert not bad_sb.any(), np.argwhere(bad_sb)[:5]
    mul = np.exp2(127.0 - scales.astype(np.float64))[:, :, None]
    v = (yb * mul).reshape(32, 256).astype(np.float32)
    want = fp8.e4m3_encode(v)
    got_val = fp8.e4m3_decode(codes).astype(np.float64)
    want_val = fp8.e4m3_decode(want).astype(np.float64)
    diff = codes != want
    # a mismatch must be a rounding-boundary case: one e4m3 step apart and y / scale within 1e-5 of the midpoint
    if diff.any():
        step = np.abs(got_val - want_val)[diff]
        mid = (np.abs(got_val) + np.abs(want_val))[diff] / 2
        assert np.all(np.abs(np.abs(v.astype(np.float64)[diff]) - mid) <= 1e-5 * mid + 1e-12), \
            (np.argwhere(diff)[:5], step[:5])
    print(f"mx layernorm: {int(diff.sum())} of 8192 codes at a rounding boundary, scales exact")
    assert diff.sum() <= 16


def _ffn_up_inputs(seed):
    """Operands whose FFN-up sums are exact in f32 (integers below 2^15 before the power-of-two
    channel scale), so that the kernel's result is fully determined and every byte can be compared:
    A = e4m3 integers in [-8, 8] with block scales 2^-1 .. 2^2, W = e4m3 integers in [-4, 4], per-channel
    scales 2^-6 .. 2^-2, bias multiples of 1/16; about half the pre-activations negative (ReLU zeros),
    one row and one 32-column block of weights all zero (zero blocks: scale byte 2)."""
    rng = np.random.default_rng(seed)
    a_codes = fp8.e4m3_encode(rng.integers(-8, 9, (32, 256)).astype(np.float32))
    a_scales = rng.integers(126, 130, (32, 8)).astype(np.uint8)
    a_codes[7] = 0
    w_codes = fp8.e4m3_encode(rng.integers(-4, 5, (1024, 256)).astype(np.float32))
    w_codes[64:96] = 0
    wscale = np.exp2(rng.integers(-6, -1, 1024)).astype(np.float32)
    bias = (rng.integers(-256, 257, 1024) / 16.0).astype(np.float32)
    bias[64:96] = 0.0
    return a_codes, a_scales, w_codes, wscale, bias


def _run_ffn_up(lib, a_codes, a_scales, w_codes, wscale, bias):
    dev = [th.from_numpy(np.ascontiguousarray(v)).cuda() for v in (a_codes, a_scales, w_codes, wscale, bias)]
    h_codes = th.full((32, 1024), 0x7f, dtype=th.uint8, device="cuda")
    h_scales = th.full((32, 32), 0xff, dtype=th.uint8, device="cuda")
    rc = lib.ggd_mx_ffn_up(*[t.data_ptr() for t in dev], h_codes.data_ptr(), h_scales.data_ptr(), None)
    assert rc == 0, rc
    return h_codes.cpu().numpy(), h_scales.cpu().numpy()


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_mx_ffn_up_epilogue_bit_exact(lib, seed):
    """The long loop's FFN-up stage on block-scaled fp8 MFMA -- the transposed MFMA chunk and the
    ReLU^2 epilogue that quantises the hidden rows (lk_relu2_mx: the lane's two column tiles x its 4
    lane rows as one 32-column block via lanerow_max4, the e8m0 byte, mx_pack4's byte order, the
    scale placement) -- run by ggd_mx_ffn_up on one 32-row block: every one of the 32,768 e4m3 codes
    and 1,024 scale bytes equals oracle/fp8.py mx_ffn_up.  A deliberately wrong block -> lane map
    (blocks of 16 or 64 columns), a plain ReLU, or the blocks shifted by 16 columns each disagree."""
    a_codes, a_scales, w_codes, wscale, bias = _ffn_up_inputs(seed)
    got_c, got_s = _run_ffn_up(lib, a_codes, a_scales, w_codes, wscale, bias)
    want_c, want_s = fp8.mx_ffn_up(a_codes, a_scales, w_codes, wscale, bias)
    bad_s = np.argwhere(got_s != want_s)
    bad_c = np.argwhere(got_c != want_c)
    for r, k in bad_c[:8].tolist():
        print(f"code row {r} col {k}: gpu {got_c[r, k]:#04x} oracle {want_c[r, k]:#04x}")
    assert len(bad_s) == 0, bad_s[:8]
    assert len(bad_c) == 0, len(bad_c)
    assert (want_s == 2).any() and (want_c == 0).mean() > 0.3 and (want_s > 2).mean() > 0.5  # cases covered
    # sensitivity: the wrong maps / activation are told apart
    for kw in (dict(block_cols=16), dict(block_cols=64), dict(square=False)):
        wc, ws = fp8.mx_ffn_up(a_codes, a_scales, w_codes, wscale, bias, **kw)
        assert (wc != got_c).any() or ws.shape != got_s.shape or (ws != got_s).any(), kw
    shifted = np.roll(fp8.mx_ffn_up(np.roll(a_codes, 0, 1), a_scales, np.roll(w_codes, 16, 0), np.roll(wscale, 16),
                                    np.roll(bias, 16))[0], -16, 1)
    assert (shifted != got_c).any()


def test_mx_ffn_up_rejects_null_pointers(lib):
    assert lib.ggd_mx_ffn_up(0, 0, 0, 0, 0, 0, 0, None) == -1
