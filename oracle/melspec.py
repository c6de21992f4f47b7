"""Restatement of torchaudio's MelSpectrogram + AmplitudeToDB defaults (TEST INFRASTRUCTURE).

The reference's 1D front-end is ``lib/wam_1D.py:194-219`` (``compute_melspec``):
``MelSpectrogram(sample_rate, n_fft, n_mels)`` then ``AmplitudeToDB()``, per waveform, ``.T``.
torchaudio is absent offline, so this follows torchaudio's documented algorithm and defaults:
hann(n_fft) periodic window, hop = n_fft // 2, center=True, reflect padding, power 2, onesided,
htk mel scale, no filter normalisation, f_min = 0, f_max = sample_rate // 2;
AmplitudeToDB(stype='power'): 10 * log10(clamp(x, 1e-10)), no top_db.
PARITY UNPINNED (no torchaudio / librosa fixtures exist in either interpreter here).
"""
import math

import torch


def hz_to_mel(f):
    return 2595.0 * math.log10(1.0 + (f / 700.0))


def mel_to_hz(m):
    return 700.0 * (10.0 ** (m / 2595.0) - 1.0)


def melscale_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate):
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_pts = torch.linspace(hz_to_mel(f_min), hz_to_mel(f_max), n_mels + 2)
    f_pts = mel_to_hz(m_pts)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.max(torch.zeros(1), torch.min(down, up))


class MelSpectrogram(torch.nn.Module):
    def __init__(self, sample_rate=16000, n_fft=400, n_mels=128, **_):
        super().__init__()
        self.n_fft = n_fft
        self.hop = n_fft // 2
        self.register_buffer("window", torch.hann_window(n_fft))
        self.register_buffer("fb", melscale_fbanks(n_fft // 2 + 1, 0.0, float(sample_rate // 2),
                                                   n_mels, sample_rate))

    def forward(self, waveform):
        shape = waveform.shape
        w = waveform.reshape(-1, shape[-1])
        spec = torch.stft(w, n_fft=self.n_fft, hop_length=self.hop, win_length=self.n_fft,
                          window=self.window.to(w.device), center=True, pad_mode="reflect",
                          normalized=False, onesided=True, return_complex=True)
        spec = spec.reshape(shape[:-1] + spec.shape[-2:]).abs().pow(2.0)
        return torch.matmul(spec.transpose(-1, -2), self.fb.to(spec.device)).transpose(-1, -2)


class AmplitudeToDB(torch.nn.Module):
    def __init__(self, stype="power", top_db=None):
        super().__init__()
        self.multiplier = 10.0 if stype == "power" else 20.0
        self.amin = 1e-10
        self.db_multiplier = math.log10(max(self.amin, 1.0))

    def forward(self, x):
        x_db = self.multiplier * torch.log10(torch.clamp(x, min=self.amin))
        return x_db - self.multiplier * self.db_multiplier
