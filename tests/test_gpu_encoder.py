"""GPU parity of the HIP speech encoder (csrc/ggd_encoder.hip, ggd_enc_* C ABI) against the CPU oracle
(oracle/ref_denoiser.py:speech_encoder, restating ha2g/speech_encoder.py:37-61).

Tolerances: f32 contexts (every product in f32, sums in another order than the CPU's)
max|diff| <= 2e-4 x max(1, max|z|); bf16 contexts (convolution operands rounded to bf16,
f32 accumulation) rel-RMS <= 3e-2 per token set.
"""
import pytest
import torch as th

from oracle import ref_denoiser

pytestmark = pytest.mark.gpu


def rel_rms(a, b):
    return (((a - b) ** 2).mean().sqrt() / (b ** 2).mean().sqrt()).item()


@pytest.fixture(scope="module")
def sd(pkg, beat_cfg):
    arch = pkg.arch_from_config(beat_cfg.Model, 123)
    return pkg.init_state_dict(arch, seed=0, perturb=True)


def encoder(pkg, sd, dtype):
    enc = __import__(pkg.__name__ + ".encoder", fromlist=["x"])
    return enc.SpeechEncoder(sd, "cuda:0", dtype=dtype)


def wavs(n, wav_len=32000, seed=5):
    g = th.Generator().manual_seed(seed)
    return th.randn(n, wav_len, generator=g) * 0.1


@pytest.mark.parametrize("wav_len", [32000, 128000])
def test_encoder_f32_matches_oracle(pkg, sd, wav_len):
    wav = wavs(2, wav_len)
    want = ref_denoiser.speech_encoder(sd, wav)
    got = [z.cpu() for z in encoder(pkg, sd, "f32")(wav.cuda())]
    for a, b in zip(got, want):
        assert a.shape == b.shape, (a.shape, b.shape)
        err = (a - b).abs().max().item()
        assert err <= 2e-4 * max(1.0, b.abs().max().item()), err


@pytest.mark.parametrize("wav_len", [32000, 80000, 128000])
def test_encoder_bf16_matches_oracle(pkg, sd, wav_len):
    """bf16 tower (compile-time-geometry NHWC convs at these widths: 63 / 157 / 250 frames)."""
    wav = wavs(3, wav_len)
    want = ref_denoiser.speech_encoder(sd, wav)
    got = [z.cpu() for z in encoder(pkg, sd, "bf16")(wav.cuda())]
    for a, b in zip(got, want):
        assert a.shape == b.shape
        r = rel_rms(a, b)
        print(f"bf16 encoder tokens {tuple(a.shape)}: rel-RMS {r:.3e}")
        assert r <= 3e-2, r


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_encoder_batch_invariant(pkg, sd, dtype):
    """A clip's tokens are bit-identical whatever batch (or chunk) it is encoded in."""
    enc = encoder(pkg, sd, dtype)
    wav = wavs(5).cuda()
    full = enc(wav)
    part = enc(wav[2:4].contiguous())
    for a, b in zip(full, part):
        assert th.equal(a[2:4], b)


@pytest.mark.parametrize("wav_len", [32000, 128000])
def test_encoder_frontend_matches_scipy_mel(pkg, sd, wav_len):
    """The HIP front end (pre-emphasis, STFT power, HTK mel, +1e-6, InstanceNorm1d;
    speech_encoder.py:18-34,53-58) against the scipy / float64 pipeline of tests/test_mel_pin.py,
    which shares no code with the oracle or the kernels.  Bound: max|diff| <= 1e-3 on the
    normalised image (O(1) values)."""
    import numpy as np
    from tests.test_mel_pin import htk_filterbank_f64, scipy_power_f64
    wav = wavs(2, wav_len, seed=9)
    got = encoder(pkg, sd, "f32").frontend(wav.cuda()).cpu().double().numpy()
    fb = htk_filterbank_f64()
    for i in range(wav.shape[0]):
        x = wav[i].double().numpy()
        y = np.empty_like(x)
        y[0] = x[0] - 0.97 * x[1]
        y[1:] = x[1:] - 0.97 * x[:-1]
        mel = fb.T @ scipy_power_f64(y) + 1e-6
        want = (mel - mel.mean(axis=1, keepdims=True)) / np.sqrt(mel.var(axis=1, keepdims=True) + 1e-5)
        assert got[i].shape == want.shape
        err = np.abs(got[i] - want).max()
        print(f"frontend {wav_len}: max|diff| {err:.3e}")
        assert err <= 1e-3, err


@pytest.mark.parametrize("wav_len", [32000, 128000])
@pytest.mark.parametrize("model_type", ["s2g_v2", "default"])
def test_encoder_writes_the_memory_layout(pkg, sd, wav_len, model_type):
    """ggd_enc_run_memory: the head kernels write the decoder's speech memory in place -- s2g_v2's
    left-zero-padded levels side by side (model.py:97-104, unequal lengths 31/30/30 and 125/124/126)
    and the default / inpaint time concat (model.py:55-68) -- bit-equal to the three tensors padded
    and concatenated by torch (encoder.speech_tokens)."""
    enc_mod = __import__(pkg.__name__ + ".encoder", fromlist=["x"])
    enc = encoder(pkg, sd, "bf16")
    wav = wavs(3, wav_len).cuda()
    want = enc_mod.speech_tokens(model_type, enc(wav))
    got = enc.memory(wav, model_type)
    assert got.shape == want.shape, (got.shape, want.shape)
    assert th.equal(got, want)
