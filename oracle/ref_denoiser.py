"""Oracle: fp32 CPU restatement of the reference denoiser  eps = model(x_t, t, wav).

Test infrastructure only (see oracle/__init__.py).  Functional style: every
function reads parameters from a flat ``state_dict``-keyed mapping ``sd`` whose
names are the reference's own ``Speech2GestureModel*.state_dict()`` keys, so a
checkpoint written by the reference loads unchanged.

Layouts follow the reference: decoder activations are sequence-major
``(L, N, d)``; the model boundary is ``(N, C, L)``.
"""
import math

import torch as th
import torch.nn.functional as F


# ----------------------------------------------------------------------------
# small building blocks
# ----------------------------------------------------------------------------

# activation quantisation hook (oracle/fp8.py mx_activations): (linear name, input) -> input
ACT_QUANT = None


def _lin(sd, name, x):
    """nn.Linear: models/modules/transformer.py:51,73; models/nn.py:189-190,213."""
    if ACT_QUANT is not None:
        x = ACT_QUANT(name, x)
    return F.linear(x, sd[name + ".weight"], sd.get(name + ".bias"))


def _ln(sd, name, x):
    """nn.LayerNorm([d]) eps=1e-5 affine: models/nn.py:141-147,212."""
    return F.layer_norm(x, (x.shape[-1],), sd[name + ".weight"], sd[name + ".bias"], 1e-5)


def positional_table(d_model, max_len=5000):
    """Sinusoidal table (max_len, 1, d): models/modules/transformer.py:157-166.

    even columns sin(p * exp(-2i ln(1e4)/d)), odd columns cos of the same argument.
    """
    pos = th.arange(0, max_len, dtype=th.float32)[:, None]
    freq = th.exp(th.arange(0, d_model, 2, dtype=th.float32) * -(math.log(10000.0) / d_model))
    tab = th.zeros(max_len, d_model)
    tab[:, 0::2] = th.sin(pos * freq)
    tab[:, 1::2] = th.cos(pos * freq)
    return tab[:, None, :]


def step_embedding(t, dim, max_period=10000):
    """diffusion_step_embedding: models/nn.py:17-35 ([cos | sin], odd dim zero-padded)."""
    half = dim // 2
    freqs = th.exp(-math.log(max_period) * th.arange(0, half, dtype=th.float32) / half)
    arg = t[:, None].float() * freqs[None]
    emb = th.cat([th.cos(arg), th.sin(arg)], dim=-1)
    if dim % 2:
        emb = th.cat([emb, th.zeros_like(emb[:, :1])], dim=-1)
    return emb


def step_encoder(sd, t, d_model):
    """DiffusionStepEncoder.forward: models/nn.py:38-52 (Linear, SiLU, Linear, Dropout p=0)."""
    e = step_embedding(t, d_model)
    e = F.silu(_lin(sd, "diffusion_step_encoder.proj.0", e))
    return _lin(sd, "diffusion_step_encoder.proj.2", e)


# ----------------------------------------------------------------------------
# Primer-EZ multi-dconv-head attention: models/modules/transformer.py:19-126
# ----------------------------------------------------------------------------

def _depthwise_seq_conv(sd, name, x):
    """SpatialDepthWiseConv.forward: transformer.py:28-44.

    x: (L, N, H, dk).  One 3-tap filter per dk channel, shared by every head and
    clip; conv padding 2 then crop 1 on both sides (transformer.py:23-24,40) so
    out[i] = b + w0 x[i-1] + w1 x[i] + w2 x[i+1] with zeros outside.
    """
    L, N, H, dk = x.shape
    y = x.permute(1, 2, 3, 0).reshape(N * H, dk, L)
    y = F.conv1d(y, sd[name + ".conv.weight"], sd[name + ".conv.bias"], padding=2, groups=dk)
    y = y[:, :, 1:-1]
    return y.reshape(N, H, dk, L).permute(3, 0, 1, 2)


def _heads(sd, name, x, heads):
    """PrepareForMultiHeadAttention (+ SpatialDepthWiseConv): transformer.py:47-59,121-126."""
    y = _lin(sd, name + ".0.linear", x)
    y = y.reshape(*x.shape[:-1], heads, -1)
    return _depthwise_seq_conv(sd, name + ".1", y)


def mdha(sd, name, query, key, value, heads):
    """MultiDConvHeadAttention forward: transformer.py:88-118 (no mask, dropout 0).

    softmax runs over the key index j of scores[i, j, b, h] (transformer.py:72,113).
    """
    L, N, d = query.shape
    q = _heads(sd, name + ".query", query, heads)
    k = _heads(sd, name + ".key", key, heads)
    v = _heads(sd, name + ".value", value, heads)
    scale = 1.0 / math.sqrt(d // heads)
    s = th.einsum("ibhd,jbhd->ijbh", q, k)
    s = s * scale
    p = th.softmax(s, dim=1)
    o = th.einsum("ijbh,jbhd->ibhd", p, v).reshape(L, N, d)
    return _lin(sd, name + ".output", o)


def ffn(sd, name, x):
    """FeedForward with SquaredReLU: transformer.py:8-16,129-154."""
    h = F.relu(_lin(sd, name + ".layer1", x))
    return _lin(sd, name + ".layer2", h * h)


# ----------------------------------------------------------------------------
# decoders
# ----------------------------------------------------------------------------

def oneway_decoder(sd, x, memory, heads, n_layers, pe):
    """OnewayCrossAttention.forward: models/nn.py:216-228 with layers nn.py:154-174.

    x: (L, N, d_pose), memory: (Tm, N, d).  Positions restart at 0 for both
    streams (nn.py:222-223); memory is never normalised or updated.
    """
    p = "pose_decoder."
    x = _lin(sd, p + "emb_x", x)
    x = x + pe[: x.shape[0]]
    m = _lin(sd, p + "emb_mem", memory)
    m = m + pe[: m.shape[0]]
    for i in range(n_layers):
        q = p + f"layers.{i}."
        z = _ln(sd, q + "norm_self_attn", x)
        x = x + mdha(sd, q + "self_attn", z, z, z, heads)
        z = _ln(sd, q + "norm_cross_attn", x)
        x = x + mdha(sd, q + "cross_attn", z, m, m, heads)
        z = _ln(sd, q + "norm_ff", x)
        x = x + ffn(sd, q + "feed_forward", z)
    x = _ln(sd, p + "out_layers.0", x)
    return _lin(sd, p + "out_layers.1", x)


def twoway_decoder(sd, x, memory, heads, n_layers, pe):
    """CrossAttention.forward: models/nn.py:428-447 with layers nn.py:90-125.

    Joint positional encoding over [x; memory] (nn.py:438-442); each layer
    self-attends x and memory separately, then attends over the joint sequence,
    then feed-forwards x (and memory, except in the last layer, nn.py:408-418).
    """
    p = "pose_decoder."
    x = _lin(sd, p + "emb_x", x)
    m = _lin(sd, p + "emb_mem", memory)
    lx = x.shape[0]
    h = th.cat([x, m], dim=0)
    h = h + pe[: h.shape[0]]
    x, m = h[:lx], h[lx:]
    for i in range(n_layers):
        q = p + f"layers.{i}."
        z = _ln(sd, q + "norm_self_attn", x)
        x = x + mdha(sd, q + "self_attn", z, z, z, heads)
        z = _ln(sd, q + "norm_self_attn_mem", m)
        m = m + mdha(sd, q + "self_attn_mem", z, z, z, heads)
        h = th.cat([x, m], dim=0)
        z = _ln(sd, q + "norm_cross_attn", h)
        h = h + mdha(sd, q + "cross_attn", z, z, z, heads)
        x, m = h[:lx], h[lx:]
        z = _ln(sd, q + "norm_ff", x)
        x = x + ffn(sd, q + "feed_forward", z)
        if (q + "feed_forward_mem.layer1.weight") in sd:
            z = _ln(sd, q + "norm_ff_mem", m)
            m = m + ffn(sd, q + "feed_forward_mem", z)
    x = _ln(sd, p + "out_layers.0", x)
    return _lin(sd, p + "out_layers.1", x)


# ----------------------------------------------------------------------------
# HA2G speech encoder: models/modules/ha2g/speech_encoder.py:9-61
# ----------------------------------------------------------------------------

def pre_emphasis(wav, coef=0.97):
    """PreEmphasis: ha2g/model/utils.py:22-38 -- y[n] = x[n] - c x[n-1], reflect pad (y[0] = x[0] - c x[1])."""
    xp = F.pad(wav[:, None, :], (1, 0), mode="reflect")
    k = th.tensor([[[-coef, 1.0]]], dtype=wav.dtype)
    return F.conv1d(xp, k)[:, 0, :]


def hz_to_mel_htk(f):
    return 2595.0 * math.log10(1.0 + f / 700.0)


def mel_filterbank(n_freqs=513, f_min=0.0, f_max=8000.0, n_mels=128, sample_rate=16000):
    """torchaudio.functional.melscale_fbanks(norm=None, mel_scale='htk') semantics.

    Used by torchaudio.transforms.MelSpectrogram at ha2g/speech_encoder.py:20-25
    (torchaudio is absent in this image; restated from its documented algorithm):
    triangular filters between n_mels+2 points equally spaced on the HTK mel scale.
    Returns (n_freqs, n_mels).
    """
    all_freqs = th.linspace(0, sample_rate // 2, n_freqs)
    m_pts = th.linspace(hz_to_mel_htk(f_min), hz_to_mel_htk(f_max), n_mels + 2)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return th.clamp(th.min(down, up), min=0.0)


def mel_power_spectrogram(wav, window, fb, n_fft=1024, hop=512):
    """torchaudio MelSpectrogram(16000, n_fft=1024, hop=512, n_mels=128) forward.

    Spectrogram: stft(center=True, pad_mode='reflect', onesided, not normalised),
    |.|^2 via abs().pow(2); MelScale: (spec^T @ fb)^T.  Output (N, n_mels, frames).
    """
    spec = th.stft(wav, n_fft=n_fft, hop_length=hop, win_length=n_fft, window=window,
                   center=True, pad_mode="reflect", normalized=False, onesided=True,
                   return_complex=True)
    power = spec.abs().pow(2.0)
    return th.matmul(power.transpose(-1, -2), fb).transpose(-1, -2)


def _bn(sd, name, x, train=False):
    """BatchNorm2d (eps 1e-5): eval mode uses the running stats (main.py:116 calls model.eval());
    train mode (trainer.py:229 model.train()) normalises with the batch statistics."""
    if train:
        return F.batch_norm(x, None, None, sd[name + ".weight"], sd[name + ".bias"], True, 0.0, 1e-5)
    return F.batch_norm(x, sd[name + ".running_mean"], sd[name + ".running_var"],
                        sd[name + ".weight"], sd[name + ".bias"], False, 0.0, 1e-5)


def _conv(sd, name, x, stride=1, padding=0):
    return F.conv2d(x, sd[name + ".weight"], sd.get(name + ".bias"), stride=stride, padding=padding)


def _se_block(sd, name, x, stride, train=False):
    """SEBasicBlock.forward: ha2g/model/ResNetBlocks.py:21-37 (ReLU before BN after conv1)."""
    out = _conv(sd, name + ".conv1", x, stride=stride, padding=1)
    out = _bn(sd, name + ".bn1", F.relu(out), train)
    out = _bn(sd, name + ".bn2", _conv(sd, name + ".conv2", out, padding=1), train)
    # SELayer: ResNetBlocks.py:81-96
    y = out.mean(dim=(2, 3))
    y = F.relu(_lin(sd, name + ".se.fc.0", y))
    y = th.sigmoid(_lin(sd, name + ".se.fc.2", y))
    out = out * y[:, :, None, None]
    if (name + ".downsample.0.weight") in sd:
        res = _bn(sd, name + ".downsample.1", _conv(sd, name + ".downsample.0", x, stride=stride), train)
    else:
        res = x
    return F.relu(out + res)


def _head(sd, feat, conv, bn, fc, shuffle, train=False):
    """Low/mid/high heads: ResNetSE34V2.py:157-188 (PixelShuffle, conv, ReLU, BN, flatten c*H, Linear)."""
    if shuffle > 1:
        feat = F.pixel_shuffle(feat, shuffle)
    feat = _bn(sd, bn, F.relu(_conv(sd, conv, feat)), train)
    n, c, hgt, w = feat.shape
    feat = feat.reshape(n, c * hgt, w).transpose(1, 2)
    return _lin(sd, fc, feat)


def speech_encoder(sd, wav, train=False):
    """HA2GSpeechEncoder.forward: speech_encoder.py:37-61 -> (z_low, z_mid, z_high), each (N, T_i, d).
    train: BatchNorm on batch statistics (the training step's mode); the front end has no state."""
    p = "speech_encoder."
    x = pre_emphasis(wav)
    x = mel_power_spectrogram(x, sd[p + "wav2spec.1.spectrogram.window"], sd[p + "wav2spec.1.mel_scale.fb"])
    x = x + 1e-6
    x = F.instance_norm(x, eps=1e-5)  # InstanceNorm1d(128), no affine, per-instance stats
    return speech_encoder_from_image(sd, x, train)


def speech_encoder_from_image(sd, img, train=False):
    """The SE-ResNet + heads + projection of speech_encoder() from the InstanceNorm'd mel image
    (N, 128, F) (Hierarchical_WavEncoder / ResNetSE.forward: hierarchy_net.py:16-19,
    ResNetSE34V2.py:118-188, speech_encoder.py:59-61)."""
    p = "speech_encoder."
    r = p + "wav_encoder.feat_extractor."
    x = img[:, None]
    x = _bn(sd, r + "bn1", F.relu(_conv(sd, r + "conv1", x, padding=1)), train)
    feats = []
    for li, (nblk, stride) in enumerate(zip((3, 4, 6, 3), (1, 2, 2, 2))):
        for bi in range(nblk):
            x = _se_block(sd, r + f"layer{li + 1}.{bi}", x, stride if bi == 0 else 1, train)
        feats.append(x)
    low = _head(sd, feats[1], r + "conv_low", r + "bn_low", r + "fc_low", 1, train)
    mid = _head(sd, feats[2], r + "conv_mid", r + "bn_mid", r + "fc_mid", 2, train)
    high = _head(sd, feats[3], r + "conv_high", r + "bn_high", r + "fc_high", 4, train)
    proj = p + "wav_proj_layer"
    return _lin(sd, proj, low), _lin(sd, proj, mid), _lin(sd, proj, high)


# ----------------------------------------------------------------------------
# memory assembly + full model
# ----------------------------------------------------------------------------

def speech_memory(sd, cfg, z):
    """Step-invariant speech part of the memory, (Ts, N, d).

    s2g_v2: left zero-pad each level to the longest, concat on features, blend
    Linear(3d -> d) (models/model.py:97-106).  default: concat on time (model.py:55-68).
    """
    z_low, z_mid, z_high = z
    if cfg["type"] == "s2g_v2":
        longest = max(a.shape[1] for a in z)
        padded = [F.pad(a, (0, 0, longest - a.shape[1], 0)) for a in z]
        blend = _lin(sd, "blend_layer", th.cat(padded, dim=-1))
        return blend.transpose(0, 1)
    if cfg["type"] in ("default", "inpaint"):  # Speech2GestureModelInpaint inherits it (model.py:118-166)
        return th.cat([a.transpose(0, 1) for a in z], dim=0)
    raise ValueError(f"Unsupported model type {cfg['type']}")


def inpaint_projection(sd, inpaint_pose, inpaint_mask):
    """Speech2GestureModelInpaint.proj on [pose * mask, mask] (models/model.py:135-142, 160-162):
    Linear(C+1 -> d) SiLU Linear(d -> d) SiLU Linear(d -> C) (+ Dropout, identity in eval).
    inpaint_pose (L, N, C), inpaint_mask (L, N, 1) -> (L, N, C)."""
    x_inp = th.cat([inpaint_pose * inpaint_mask, inpaint_mask], dim=-1)
    h = F.silu(_lin(sd, "proj.0", x_inp))
    h = F.silu(_lin(sd, "proj.2", h))
    return _lin(sd, "proj.4", h)


def denoise(sd, cfg, x_t, t, wav=None, speech=None, pe=None, inpaint_pose=None, inpaint_mask=None):
    """Speech2GestureModelBase.forward + myforward: models/model.py:12-15,41-73,81-117.

    x_t (N, C, L) fp32, t (N,) int64 original timesteps -> eps (N, C, L).
    ``speech`` may carry precomputed speech memory (Ts, N, d); the reference
    recomputes the encoder inside every call (model.py:95-96) -- that is what
    ``wav`` does here.
    """
    d = cfg["d_model"]
    if pe is None:
        pe = positional_table(d)
    if speech is None:
        speech = speech_memory(sd, cfg, speech_encoder(sd, wav))
    step = step_encoder(sd, t, d)[None]
    memory = th.cat([step, speech], dim=0)
    x = x_t.permute(2, 0, 1)
    if cfg["type"] == "inpaint":  # x = x + proj(x_inp)  (model.py:164)
        x = x + inpaint_projection(sd, inpaint_pose, inpaint_mask)
    if cfg["decoder"] == "oneway_cross_attention":
        y = oneway_decoder(sd, x, memory, cfg["heads"], cfg["n_layers"], pe)
    elif cfg["decoder"] == "cross_attention":
        y = twoway_decoder(sd, x, memory, cfg["heads"], cfg["n_layers"], pe)
    else:
        raise ValueError(f"Unsupported decoder type {cfg['decoder']}")
    return y.permute(1, 2, 0)


class OracleModel:
    """Callable with the reference model protocol eps = model(x_t, t, wav=...) (model.py:12-15)."""

    def __init__(self, sd, cfg, cache_speech=False):
        self.sd = {k: v.detach().float() if v.is_floating_point() else v for k, v in sd.items()}
        self.cfg = cfg
        self.pe = positional_table(cfg["d_model"])
        self.cache_speech = cache_speech
        self._cache = None

    @th.no_grad()
    def __call__(self, x_t, t, wav=None, speech=None, inpaint_pose=None, inpaint_mask=None):
        if speech is None and self.cache_speech:
            if self._cache is None or self._cache[0] is not wav:
                self._cache = (wav, speech_memory(self.sd, self.cfg, speech_encoder(self.sd, wav)))
            speech = self._cache[1]
        return denoise(self.sd, self.cfg, x_t, t, wav=wav, speech=speech, pe=self.pe, inpaint_pose=inpaint_pose,
                       inpaint_mask=inpaint_mask)
