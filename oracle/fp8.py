"""OCP fp8 e4m3fn weight quantization, restated for the parity tests -- TEST INFRASTRUCTURE ONLY.

The reference has no fp8 path (it is fp32 throughout, SURVEY.md 8 preamble); BASELINE.json
configs[3] asks for fp8 weights on the long-clip config.  The HIP context's GGD_FP8W mode
(include/ggd.h) stores every Linear that runs inside a denoise step as e4m3fn bytes with one f32
scale per output channel (amax / 448) -- ggd_api.hip ``f2e4m3_host`` / ``pack_lin``.  This
module restates that quantization in numpy so the oracle can run the SAME dequantized weights
(q * scale) in fp32: the tests then bound the HIP fp8 path against (a) the oracle on the
dequantized weights (bf16-activation tolerance) and (b) the oracle on the original weights
(the fp8 tolerance of SURVEY.md 8d).

e4m3fn: sign, 4 exponent bits (bias 7), 3 mantissa bits, no infinities, 0x7f / 0xff NaN,
largest finite 448 (0x7e), subnormals m * 2^-9.  Rounding: nearest even, saturating.
"""
import re

import numpy as np
import torch as th

E4M3_MAX = 448.0


def e4m3_encode(x):
    """float32 array -> uint8 e4m3fn codes (round to nearest even, saturate to +-448)."""
    x = np.asarray(x, np.float32)
    sign = np.where(np.signbit(x), 0x80, 0).astype(np.uint8)
    a = np.abs(x).astype(np.float64)
    out = np.zeros(x.shape, np.uint8)
    sub = a < 2.0 ** -6
    out[sub] = np.rint(a[sub] * 2.0 ** 9).astype(np.uint8)          # 0 .. 8 (8 = 2^-6, normal)
    nor = ~sub
    e = np.floor(np.log2(np.where(nor, a, 1.0)))
    m = np.rint((np.where(nor, a, 1.0) / 2.0 ** e - 1.0) * 8.0)       # np.rint: ties to even
    carry = m == 8
    e = np.where(carry, e + 1, e)
    m = np.where(carry, 0, m)
    code = ((e + 7).astype(np.int64) << 3) | m.astype(np.int64)
    sat = (e > 8) | ((e == 8) & (m > 6)) | (a >= E4M3_MAX)
    code = np.where(sat, 0x7e, code)
    out[nor] = code[nor].astype(np.uint8)
    out = out | sign
    out[np.isnan(x)] = 0x7f
    return out


def e4m3_decode(code):
    """uint8 e4m3fn codes -> float32 values (NaN for 0x7f / 0xff)."""
    c = np.asarray(code, np.uint8).astype(np.int64)
    s = np.where(c & 0x80, -1.0, 1.0)
    e = (c >> 3) & 0xF
    m = c & 0x7
    v = np.where(e == 0, m * 2.0 ** -9, (1.0 + m / 8.0) * 2.0 ** (e - 7))
    v = np.where((c & 0x7F) == 0x7F, np.nan, v)
    return (s * v).astype(np.float32)


def quantize_rows(w):
    """Per-output-channel (row) quantization of a torch Linear weight [out][in]:
    returns (codes uint8 [out][in], scale f32 [out], dequantized f32 [out][in])."""
    w = np.asarray(w, np.float32)
    amax = np.abs(w).max(axis=1)
    scale = np.where(amax > 0, amax / np.float32(E4M3_MAX), np.float32(1.0)).astype(np.float32)
    codes = e4m3_encode(w / scale[:, None])
    deq = e4m3_decode(codes) * scale[:, None]
    return codes, scale, deq.astype(np.float32)


# the Linears a GGD_FP8W context evaluates inside every denoise step (ggd_api.hip
# ggd_finalize_weights, pack_lin(..., step = true)); the one-way decoder's cross-attention
# key / value projections act on the step-invariant memory and stay bf16
_STEP_LINEARS = [
    r"pose_decoder\.emb_x\.weight",
    r"pose_decoder\.out_layers\.1\.weight",
    r"pose_decoder\.layers\.\d+\.self_attn(_mem)?\.(query|key|value)\.0\.linear\.weight",
    r"pose_decoder\.layers\.\d+\.self_attn(_mem)?\.output\.weight",
    r"pose_decoder\.layers\.\d+\.cross_attn\.query\.0\.linear\.weight",
    r"pose_decoder\.layers\.\d+\.cross_attn\.output\.weight",
    r"pose_decoder\.layers\.\d+\.feed_forward(_mem)?\.layer[12]\.weight",
]
_TWOWAY_EXTRA = [r"pose_decoder\.layers\.\d+\.cross_attn\.(key|value)\.0\.linear\.weight"]


def step_linear_names(sd, twoway=False):
    pats = [re.compile(p) for p in _STEP_LINEARS + (_TWOWAY_EXTRA if twoway else [])]
    return [k for k in sd if any(p.fullmatch(k) for p in pats)]


def dequantized_state_dict(sd, twoway=False):
    """Copy of ``sd`` whose per-step Linear weights are replaced by their e4m3 dequantization."""
    out = dict(sd)
    for k in step_linear_names(sd, twoway):
        _, _, deq = quantize_rows(sd[k].detach().cpu().float().numpy())
        out[k] = th.from_numpy(deq)
    return out


# ------------------------------------------------------------------------------------------
# Block-scaled (MX) e4m3 activations of the long-clip loop's fp8-MFMA stages (GGD_ROUTE_FP8_MFMA,
# csrc/ggd_chainlib.h mx_scale_byte / mx_mul): blocks of 32 consecutive values along the last dim,
# scale 2^(E - 7) for the block max 1.f 2^E (biased exponent clamped to [2, 253]), values rounded to
# e4m3 (nearest even) after the exact power-of-two division.
# ------------------------------------------------------------------------------------------
def mx_e4m3(x):
    """fp32 tensor (last dim a multiple of 32) -> its MX-e4m3 dequantization, same shape."""
    shp = x.shape
    xb = x.detach().float().reshape(-1, shp[-1] // 32, 32).contiguous()
    m = xb.abs().amax(-1, keepdim=True)
    be = (m.view(th.int32) >> 23) & 0xFF
    sb = (be - 7).clamp(2, 253)
    mul = ((254 - sb) << 23).view(th.float32)     # 2^-(sb - 127): exact
    scale = ((sb) << 23).view(th.float32)         # 2^(sb - 127)
    q = e4m3_decode(e4m3_encode((xb * mul).numpy()))
    return (th.from_numpy(q) * scale).reshape(shp)


# the Linears whose INPUT the fp8-MFMA long loop quantises (self-attention Q / K / V of LN1, the
# cross-attention query of LN2, both FFN Linears); OUT_PROJ adds the attention out-projections
_MX_INPUTS = [r"pose_decoder\.layers\.\d+\.self_attn\.(query|key|value)\.0\.linear",
              r"pose_decoder\.layers\.\d+\.cross_attn\.query\.0\.linear",
              r"pose_decoder\.layers\.\d+\.feed_forward\.layer[12]"]
_MX_OUT_PROJ = [r"pose_decoder\.layers\.\d+\.(self_attn|cross_attn)\.output"]


class mx_activations:
    """Context manager: while active, oracle.ref_denoiser quantises the inputs of the Linears the
    fp8-MFMA long loop runs on block-scaled MFMA to MX-e4m3 (``out_proj``: the attention
    out-projections too).  Test infrastructure: the oracle of that route's exact arithmetic."""

    def __init__(self, out_proj=False, first_qkv=True):
        self.pats = [re.compile(p) for p in _MX_INPUTS + (_MX_OUT_PROJ if out_proj else [])]
        # first_qkv False: layer 0's self-attention Q / K / V stay unquantised (the loop's FIRST
        # iteration takes them from the bf16 chain launch in front of it, ggd_api.hip run_long)
        self.skip = [] if first_qkv else [re.compile(r"pose_decoder\.layers\.0\.self_attn\..*")]

    def _q(self, name, x):
        if any(p.fullmatch(name) for p in self.skip):
            return x
        return mx_e4m3(x) if any(p.fullmatch(name) for p in self.pats) else x

    def __enter__(self):
        from oracle import ref_denoiser
        self._prev = ref_denoiser.ACT_QUANT
        ref_denoiser.ACT_QUANT = self._q
        return self

    def __exit__(self, *exc):
        from oracle import ref_denoiser
        ref_denoiser.ACT_QUANT = self._prev
        return False


def mx_scale_bytes(m):
    """e8m0 scale bytes of blocks whose max |v| is ``m`` (float32 array): the biased exponent of m
    minus 7, clamped to [2, 253] (csrc/ggd_chainlib.h mx_scale_byte)."""
    be = (np.asarray(m, np.float32).view(np.int32) >> 23) & 0xFF
    return np.clip(be - 7, 2, 253).astype(np.uint8)


def mx_quantise_blocks(y, block_cols=32):
    """float32 rows (R, N) -> (e4m3 codes (R, N), e8m0 scale bytes (R, N / block_cols)), one scale per
    ``block_cols`` consecutive columns of a row (32: the MX block), values divided by the exact power
    of two 2^(sb - 127) in float32 and rounded to nearest even."""
    y = np.asarray(y, np.float32)
    R, N = y.shape
    yb = y.reshape(R, N // block_cols, block_cols)
    sb = mx_scale_bytes(np.abs(yb).max(-1))
    mul = ((254 - sb.astype(np.int32)) << 23).view(np.float32)[:, :, None]
    return e4m3_encode((yb * mul).reshape(R, N)), sb


def mx_ffn_up(a_codes, a_scales, w_codes, wscale, bias, square=True, block_cols=32):
    """The long loop's FFN-up stage on block-scaled fp8 (csrc/ggd_long.hip lk_relu2_mx after
    ch_mma_mx<2, true>): h = relu(a . w^T * wscale + bias)^2 (models/modules/transformer.py:8-16
    SquaredReLU, :151-154 FFN.layer1) from the MX A image (codes (R, K) with one e8m0 scale per 32 k)
    and per-output-channel e4m3 weights, then re-quantised per 32 hidden columns.  The product is
    summed in float64 (the tests pick operands whose sums are exact); the epilogue in float32, as the
    kernel.  Returns (codes (R, N), scales (R, N / 32)).  ``square`` / ``block_cols``: deliberately
    wrong variants for the tests' sensitivity checks."""
    a = e4m3_decode(a_codes).astype(np.float64)
    R, K = a.shape
    a = (a.reshape(R, K // 32, 32) * np.exp2(np.asarray(a_scales, np.float64) - 127.0)[:, :, None]).reshape(R, K)
    acc = (a @ e4m3_decode(w_codes).astype(np.float64).T).astype(np.float32)
    v = np.maximum(acc * np.asarray(wscale, np.float32) + np.asarray(bias, np.float32), np.float32(0.0))
    y = (v * v if square else v).astype(np.float32)
    return mx_quantise_blocks(y, block_cols)
