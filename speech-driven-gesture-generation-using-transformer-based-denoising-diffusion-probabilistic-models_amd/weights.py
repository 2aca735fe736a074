"""Synthetic weights in the reference's ``state_dict`` layout.

There is no network for checkpoints, so benchmarks and tests use seeded
random-init weights of the reference architecture, under the exact key names
``Speech2GestureModel*.state_dict()`` produces (a real checkpoint's
``model_state_dict`` loads through the same path, main.py:113-115).

Init follows the reference:
  * decoder layers: xavier-uniform for every >1-D parameter (models/nn.py:86-88,150-152)
  * SE-ResNet convs: kaiming-normal, fan_out, relu; BN weight 1 / bias 0
    (ha2g/model/ResNetSE34V2.py:89-94)
  * everything else: torch defaults (Linear/Conv: U(+-1/sqrt(fan_in)); LayerNorm 1/0)
"""
import math

import torch as th

from .config import JsonConfig


def _arch(model_params, d_pose):
    mp = model_params
    return {
        "type": mp["type"], "d_model": int(mp["d_model"]), "decoder": mp["Decoder"]["type"],
        "heads": int(mp["Decoder"]["heads"]), "n_layers": int(mp["Decoder"]["n_layers"]),
        "d_pose": int(d_pose),
    }


def arch_from_config(model_params, d_pose):
    """Architecture dict (type, d_model, decoder, heads, n_layers, d_pose) from Model params."""
    if isinstance(model_params, JsonConfig):
        model_params = model_params.to_dict()
    return _arch(model_params, d_pose)


def parameter_shapes(arch):
    """Ordered {name: (shape, init)} of every parameter and buffer of the reference model."""
    d, C, H = arch["d_model"], arch["d_pose"], arch["heads"]
    dk = d // H
    S = {}

    def lin(name, n_out, n_in, init="default"):
        S[name + ".weight"] = ((n_out, n_in), init)
        S[name + ".bias"] = ((n_out,), "bias:%d" % n_in)

    def ln(name, n):
        S[name + ".weight"] = ((n,), "ones")
        S[name + ".bias"] = ((n,), "zeros")

    def bn(name, n):
        S[name + ".weight"] = ((n,), "ones")
        S[name + ".bias"] = ((n,), "zeros")
        S[name + ".running_mean"] = ((n,), "zeros")
        S[name + ".running_var"] = ((n,), "ones")
        S[name + ".num_batches_tracked"] = ((), "int0")

    def conv2d(name, co, ci, k, bias):
        S[name + ".weight"] = ((co, ci, k, k), "kaiming_out")
        if bias:
            S[name + ".bias"] = ((co,), "bias:%d" % (ci * k * k))

    # step encoder (models/nn.py:38-46)
    lin("diffusion_step_encoder.proj.0", d, d)
    lin("diffusion_step_encoder.proj.2", d, d)

    # speech encoder (ha2g/speech_encoder.py:18-34, ResNetSE34V2.py:27-49, ResNetBlocks.py:10-17,81-90)
    p = "speech_encoder."
    S[p + "wav2spec.0.flipped_filter"] = ((1, 1, 2), "preemph")
    S[p + "wav2spec.1.spectrogram.window"] = ((1024,), "hann")
    S[p + "wav2spec.1.mel_scale.fb"] = ((513, 128), "melfb")
    r = p + "wav_encoder.feat_extractor."
    conv2d(r + "conv1", 32, 1, 3, True)
    bn(r + "bn1", 32)
    conv2d(r + "conv_low", 64, 64, 2, True)
    bn(r + "bn_low", 64)
    lin(r + "fc_low", 32, 63 * 64)
    conv2d(r + "conv_mid", 32, 32, 3, True)
    bn(r + "bn_mid", 32)
    lin(r + "fc_mid", 32, 62 * 32)
    conv2d(r + "conv_high", 16, 16, 3, True)
    bn(r + "bn_high", 16)
    lin(r + "fc_high", 32, 62 * 16)
    inplanes = 32
    for li, (planes, nblk, stride) in enumerate(zip((32, 64, 128, 256), (3, 4, 6, 3), (1, 2, 2, 2))):
        for bi in range(nblk):
            q = r + f"layer{li + 1}.{bi}."
            conv2d(q + "conv1", planes, inplanes, 3, False)
            bn(q + "bn1", planes)
            conv2d(q + "conv2", planes, planes, 3, False)
            bn(q + "bn2", planes)
            lin(q + "se.fc.0", planes // 8, planes)
            lin(q + "se.fc.2", planes, planes // 8)
            if bi == 0 and (stride != 1 or inplanes != planes):
                conv2d(q + "downsample.0", planes, inplanes, 1, False)
                bn(q + "downsample.1", planes)
            inplanes = planes
    lin(p + "wav_proj_layer", d, 32)

    # decoder (models/nn.py:177-214 oneway, 381-426 two-way; transformer.py:47-154)
    P = "pose_decoder."
    lin(P + "emb_x", d, C)
    lin(P + "emb_mem", d, d)

    def mdha(name):
        for w in ("query", "key", "value"):
            lin(name + f".{w}.0.linear", d, d, "xavier")
            S[name + f".{w}.1.conv.weight"] = ((dk, 1, 3), "xavier")
            S[name + f".{w}.1.conv.bias"] = ((dk,), "bias:3")
        lin(name + ".output", d, d, "xavier")

    def ffn(name):
        lin(name + ".layer1", 4 * d, d, "xavier")
        lin(name + ".layer2", d, 4 * d, "xavier")

    L = arch["n_layers"]
    for i in range(L):
        q = P + f"layers.{i}."
        if arch["decoder"] == "oneway_cross_attention":
            ln(q + "norm_self_attn", d)
            mdha(q + "self_attn")
            ln(q + "norm_cross_attn", d)
            mdha(q + "cross_attn")
            ln(q + "norm_ff", d)
            ffn(q + "feed_forward")
        elif arch["decoder"] == "cross_attention":
            ln(q + "norm_self_attn", d)
            mdha(q + "self_attn")
            ln(q + "norm_self_attn_mem", d)
            mdha(q + "self_attn_mem")
            ln(q + "norm_cross_attn", d)
            mdha(q + "cross_attn")
            ln(q + "norm_ff", d)
            ffn(q + "feed_forward")
            if i < L - 1:
                ffn(q + "feed_forward_mem")
                ln(q + "norm_ff_mem", d)
        else:
            raise ValueError(f"Unsupported decoder type {arch['decoder']}.")
    ln(P + "out_layers.0", d)
    lin(P + "out_layers.1", C, d)
    if arch["type"] == "s2g_v2":
        lin("blend_layer", d, 3 * d)
    elif arch["type"] == "inpaint":  # models/model.py:135-145: zero-initialised as in GLIDE
        for name, n_out, n_in in (("proj.0", d, C + 1), ("proj.2", d, d), ("proj.4", C, d)):
            S[name + ".weight"] = ((n_out, n_in), "zeros")
            S[name + ".bias"] = ((n_out,), "zeros")
    elif arch["type"] != "default":
        raise ValueError(f"Unsupported model_type {arch['type']}")
    return S


def _hann(n):
    """torchaudio Spectrogram's window buffer: torch.hann_window(n) (periodic)."""
    return th.hann_window(n)


def _mel_fb(n_freqs=513, n_mels=128, sr=16000):
    """HTK mel filterbank, norm=None (torchaudio melscale_fbanks semantics)."""
    all_f = th.linspace(0, sr // 2, n_freqs)
    m_max = 2595.0 * math.log10(1.0 + (sr / 2) / 700.0)
    m = th.linspace(0.0, m_max, n_mels + 2)
    f = 700.0 * (10.0 ** (m / 2595.0) - 1.0)
    fd = f[1:] - f[:-1]
    sl = f[None, :] - all_f[:, None]
    down = (-1.0 * sl[:, :-2]) / fd[:-1]
    up = sl[:, 2:] / fd[1:]
    return th.clamp(th.min(down, up), min=0.0)


def init_state_dict(arch, seed=0, perturb=False, bounded=False, speech=False):
    """Seeded synthetic state_dict.  ``perturb`` randomises LN affines and BN statistics
    (non-trivial values for parity tests; the benchmark uses the reference init).

    ``bounded`` gives the denoiser a pose skip path so that a 1000-step trajectory stays O(1)
    (parity tests at full length; see bounded_skip).  ``speech`` (implies ``bounded``) makes the
    output depend on the speech at O(0.1) (see speech_driven)."""
    g = th.Generator().manual_seed(seed)
    sd = {}
    for name, (shape, init) in parameter_shapes(arch).items():
        if init == "default":
            bound = 1.0 / math.sqrt(shape[1])
            t = (th.rand(shape, generator=g) * 2 - 1) * bound
        elif init.startswith("bias:"):
            bound = 1.0 / math.sqrt(int(init[5:]))
            t = (th.rand(shape, generator=g) * 2 - 1) * bound
        elif init == "xavier":
            if len(shape) == 2:
                fan_in, fan_out = shape[1], shape[0]
            else:
                rf = int(th.tensor(shape[2:]).prod())
                fan_in, fan_out = shape[1] * rf, shape[0] * rf
            bound = math.sqrt(6.0 / (fan_in + fan_out))
            t = (th.rand(shape, generator=g) * 2 - 1) * bound
        elif init == "kaiming_out":
            fan_out = shape[0] * shape[2] * shape[3]
            t = th.randn(shape, generator=g) * math.sqrt(2.0 / fan_out)
        elif init == "ones":
            t = th.ones(shape)
            if perturb:
                t = t + 0.1 * th.randn(shape, generator=g)
        elif init == "zeros":
            t = th.zeros(shape)
            if perturb:
                t = t + 0.1 * th.randn(shape, generator=g)
        elif init == "int0":
            t = th.zeros((), dtype=th.long)
        elif init == "preemph":
            t = th.tensor([[[-0.97, 1.0]]])
        elif init == "hann":
            t = _hann(shape[0])
        elif init == "melfb":
            t = _mel_fb(shape[0], shape[1])
        else:
            raise ValueError(init)
        if perturb and name.endswith("running_var"):
            t = 0.5 + th.rand(shape, generator=g)
        sd[name] = t.contiguous()
    if speech:
        bounded_skip(sd, arch, seed, emb_scale=3.0)
        speech_driven(sd, arch)
    elif bounded:
        bounded_skip(sd, arch, seed)
    return sd


def speech_driven(sd, arch, mem_gain=30.0, ca_out_gain=3.0, ca_qk_gain=4.0):
    """Scale the memory embedding and the cross-attention so that the speech visibly drives the
    output (parity tests that must see the cross-attention / encoder path).

    With reference-init weights the memory tokens are dominated by the positional table (the
    speech part of emb_mem's input is ~0.27 rms against PE's ~0.7) and attention over them is
    near uniform, so two different wavs change eps by only ~0.2 % (oracle, seed 0) and a
    1000-step trajectory by less: a parity test with those weights is blind to the speech path.
    Here emb_mem x mem_gain makes the memory speech-dominated, cross-attention query / key
    weights x ca_qk_gain make its attention content-dependent, and its output projections x
    ca_out_gain give it weight in the residual stream.  Measured with the oracle (2 clips, two
    N(0, 0.1^2) wavs): eps differs by 14.7 % rel-RMS between the wavs, the final x of a T = 1000
    DDPM run by 16 % (rms(x) 3.0: still bounded with bounded_skip(emb_scale=3))."""
    sd["pose_decoder.emb_mem.weight"] = (sd["pose_decoder.emb_mem.weight"] * mem_gain).contiguous()
    for i in range(arch["n_layers"]):
        p = f"pose_decoder.layers.{i}.cross_attn."
        sd[p + "output.weight"] = (sd[p + "output.weight"] * ca_out_gain).contiguous()
        for w in ("query", "key"):
            k = p + w + ".0.linear.weight"
            sd[k] = (sd[k] * ca_qk_gain).contiguous()
    return sd


def bounded_skip(sd, arch, seed=0, emb_scale=4.0, out_gain=3.0):
    """Make eps ~ out_gain * x / rms(x) along a random orthonormal pose subspace.

    With reference-init random weights the decoder's output does not depend on x_t (emb_x is
    swamped by the positional table and the final LayerNorm caps |eps| at ~0.6), so
    x0 = sqrt(1/abar) x - sqrt(1/abar - 1) eps amplifies x and a 1000-step DDPM trajectory
    grows to |x| ~ 1e3 (measured: rms 276 after T = 1000).  Here emb_x = emb_scale * Q and
    out_layers.1 = out_gain * sqrt(C/d) * Q^T for a seeded Q (d x C, orthonormal columns): the
    pose reaches the output through the residual stream and the final LayerNorm, so eps is a
    scaled copy of x plus the other paths' contributions.  The reverse update then contracts
    x whenever |eps| exceeds the posterior's growth (out_gain > 1): rms(x) stays within
    0.4-1.0 over the whole T = 1000 DDPM loop (oracle, 2 clips).  Every other parameter keeps
    the reference init, so all kernels see non-trivial operands.
    """
    d, C = arch["d_model"], arch["d_pose"]
    g = th.Generator().manual_seed(1000 + seed)
    q, _ = th.linalg.qr(th.randn(d, C, generator=g))
    sd["pose_decoder.emb_x.weight"] = (q * emb_scale).contiguous()
    sd["pose_decoder.out_layers.1.weight"] = (q.t() * (out_gain * math.sqrt(C / d))).contiguous()
    sd["pose_decoder.out_layers.1.bias"] = th.zeros(C)
    return sd


def count_parameters(sd, prefix=""):
    """Learnable parameter count (excludes BN statistics and torchaudio/pre-emphasis buffers)."""
    skip = ("running_mean", "running_var", "num_batches_tracked", "flipped_filter",
            "spectrogram.window", "mel_scale.fb")
    return sum(v.numel() for k, v in sd.items() if k.startswith(prefix) and not k.endswith(skip))
