"""Pins the oracle's restatement of torchaudio's MelSpectrogram (ha2g/speech_encoder.py:18-26:
MelSpectrogram(16000, n_fft=1024, hop_length=512, n_mels=128), torchaudio absent from this image)
against implementations that share no code with it:

* the power spectrogram against ``scipy.signal.stft`` (periodic Hann window, frames centred by a
  reflect pad of n_fft / 2 on each side, one-sided, unnormalised: scipy's ``scaling='spectrum'``
  divides by sum(window), undone here), in float64;
* the mel filterbank against the HTK triangular filters written out from their definition
  (mel(f) = 2595 log10(1 + f / 700), n_mels + 2 equally spaced mel points from 0 to 8 kHz,
  norm=None), evaluated in float64 by a per-filter loop;
* PreEmphasis (ha2g/model/utils.py:22-38: reflect pad, y[n] = x[n] - 0.97 x[n - 1]) against the
  formula.

Bounds (written here): filterbank 1e-12 when the restatement runs in float64, 3e-5 absolute in
float32 (torchaudio's precision); power and mel spectrum max|diff| <= 1e-5 x max|reference|;
pre-emphasis 1e-6 absolute.  This pins the third-party arithmetic the oracle
restates from documentation; the model as a whole stays "parity unpinned" (DESIGN.md 0).
"""
import math

import numpy as np
import pytest
import scipy.signal
import torch as th

from oracle import ref_denoiser

SR, N_FFT, HOP, N_MELS = 16000, 1024, 512, 128


def htk_filterbank_f64(n_freqs=N_FFT // 2 + 1, f_min=0.0, f_max=SR / 2, n_mels=N_MELS):
    mel = lambda f: 2595.0 * math.log10(1.0 + f / 700.0)
    hz = lambda m: 700.0 * (10.0 ** (m / 2595.0) - 1.0)
    lo, hi = mel(f_min), mel(f_max)
    pts = [hz(lo + (hi - lo) * i / (n_mels + 1)) for i in range(n_mels + 2)]
    freqs = [SR / 2 * k / (n_freqs - 1) for k in range(n_freqs)]
    fb = np.zeros((n_freqs, n_mels))
    for m in range(n_mels):
        fl, fc, fr = pts[m], pts[m + 1], pts[m + 2]
        for k, f in enumerate(freqs):
            fb[k, m] = max(0.0, min((f - fl) / (fc - fl), (fr - f) / (fr - fc)))
    return fb


def scipy_power_f64(wav):
    """|STFT|^2 (n_freqs, frames) of one clip, centred frames, torch.stft's unnormalised scale."""
    x = np.pad(np.asarray(wav, np.float64), N_FFT // 2, mode="reflect")
    win = scipy.signal.get_window("hann", N_FFT, fftbins=True)   # periodic, as torch.hann_window
    _, _, z = scipy.signal.stft(x, nperseg=N_FFT, noverlap=N_FFT - HOP, window=win, boundary=None,
                                padded=False, return_onesided=True, detrend=False, scaling="spectrum")
    return np.abs(z * win.sum()) ** 2


def test_mel_filterbank_matches_htk_definition():
    want = htk_filterbank_f64()
    # the restatement's formula, evaluated in float64: equal to the definition to rounding
    old = th.get_default_dtype()
    th.set_default_dtype(th.float64)
    try:
        got64 = ref_denoiser.mel_filterbank().numpy()
    finally:
        th.set_default_dtype(old)
    assert got64.shape == want.shape == (N_FFT // 2 + 1, N_MELS)
    assert np.abs(got64 - want).max() <= 1e-12
    # as torchaudio runs it, in float32: the Hz-domain differences (f - f_l, ~40 Hz apart at ~5 kHz)
    # carry f32 rounding, |diff| <= 3e-5 on weights <= 1
    got32 = ref_denoiser.mel_filterbank().double().numpy()
    assert np.abs(got32 - want).max() <= 3e-5
    assert (want > 0).sum(axis=0).min() >= 1   # every filter covers at least one bin


@pytest.mark.parametrize("n_wav", [32000, 36266, 128000])
def test_power_and_mel_spectrogram_match_scipy(n_wav):
    g = th.Generator().manual_seed(11)
    wav = th.randn(2, n_wav, generator=g) * 0.1
    window = th.hann_window(N_FFT)
    fb32 = ref_denoiser.mel_filterbank()
    got_mel = ref_denoiser.mel_power_spectrogram(wav, window, fb32).double().numpy()
    spec = th.stft(wav, n_fft=N_FFT, hop_length=HOP, win_length=N_FFT, window=window, center=True,
                   pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    got_pow = spec.abs().pow(2.0).double().numpy()
    fb = htk_filterbank_f64()
    for i in range(wav.shape[0]):
        want_pow = scipy_power_f64(wav[i].double().numpy())
        assert got_pow[i].shape == want_pow.shape == (N_FFT // 2 + 1, 1 + n_wav // HOP)
        assert np.abs(got_pow[i] - want_pow).max() <= 1e-5 * want_pow.max()
        want_mel = fb.T @ want_pow
        assert got_mel[i].shape == want_mel.shape
        assert np.abs(got_mel[i] - want_mel).max() <= 1e-5 * want_mel.max()


def test_pre_emphasis_formula():
    x = th.randn(3, 1000, generator=th.Generator().manual_seed(12))
    y = ref_denoiser.pre_emphasis(x).numpy()
    xn = x.numpy()
    want = np.empty_like(xn)
    want[:, 0] = xn[:, 0] - 0.97 * xn[:, 1]          # reflect pad: x[-1] = x[1]
    want[:, 1:] = xn[:, 1:] - 0.97 * xn[:, :-1]
    assert np.abs(y - want).max() <= 1e-6
