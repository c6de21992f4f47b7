"""1D front-end on the GPU: torchaudio ``MelSpectrogram`` + ``AmplitudeToDB`` defaults, batched.

The reference computes it per waveform on the CPU (``lib/wam_1D.py:194-219``). Here it is one
batched ``torch.stft`` + mel matmul + dB on the device, differentiable by autograd (the adjoint
into the waverec output). Algorithm (torchaudio's documented defaults; parity unpinned offline,
see DESIGN.md): periodic hann(n_fft), hop n_fft//2, center + reflect pad, power 2, onesided,
htk mel filterbank without normalisation over [0, sr//2], 10*log10(clamp(x, 1e-10)).
"""
import math

import torch

_FB = {}


def _hz_to_mel(f):
    return 2595.0 * math.log10(1.0 + (f / 700.0))


def mel_filterbank(n_fft, n_mels, sample_rate, device):
    key = (n_fft, n_mels, sample_rate, torch.device(device))
    if key not in _FB:
        n_freqs = n_fft // 2 + 1
        all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
        m_pts = torch.linspace(_hz_to_mel(0.0), _hz_to_mel(float(sample_rate // 2)), n_mels + 2)
        f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
        f_diff = f_pts[1:] - f_pts[:-1]
        slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
        down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
        up = slopes[:, 2:] / f_diff[1:]
        fb = torch.max(torch.zeros(1), torch.min(down, up))
        _FB[key] = (fb.to(device), torch.hann_window(n_fft).to(device))
    return _FB[key]


def melspec_db(wave, n_fft, sample_rate, n_mels):
    """wave [B, T] -> [B, 1, frames, n_mels] (the reference's stacked ``.T`` layout)."""
    fb, win = mel_filterbank(n_fft, n_mels, sample_rate, wave.device)
    spec = torch.stft(wave, n_fft=n_fft, hop_length=n_fft // 2, win_length=n_fft, window=win, center=True,
                      pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    power = spec.abs().pow(2.0)                       # [B, freqs, frames]
    mel = torch.matmul(power.transpose(-1, -2), fb)   # [B, frames, n_mels]
    db = 10.0 * torch.log10(torch.clamp(mel, min=1e-10))
    return db.unsqueeze(1)


def melspec_power(wave, n_fft, sample_rate, n_mels):
    """torchaudio MelSpectrogram (power, no dB) of [B, T] -> [B, n_mels, frames]."""
    fb, win = mel_filterbank(n_fft, n_mels, sample_rate, wave.device)
    spec = torch.stft(wave, n_fft=n_fft, hop_length=n_fft // 2, win_length=n_fft, window=win, center=True,
                      pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    return torch.matmul(spec.abs().pow(2.0).transpose(-1, -2), fb).transpose(-1, -2)
