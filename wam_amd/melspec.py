"""1D front-end on the GPU: torchaudio ``MelSpectrogram`` + ``AmplitudeToDB`` defaults, batched.

The reference computes it per waveform on the CPU (``lib/wam_1D.py:194-219``). Here one HIP
kernel does the whole front-end of a batch of waveforms (``k_mel_fwd`` in csrc/melspec.hip:
reflect-padded periodic-Hann frames, a packed real FFT in LDS, the band-sparse HTK mel sum, dB)
and one does its adjoint into the waveform (``k_mel_adj``: the frame recomputed, the chain rule
through dB / mel / power, an inverse packed FFT and the reflect-folded overlap-add).
Algorithm (torchaudio's documented defaults; parity unpinned offline): periodic
hann(n_fft), hop n_fft//2, center + reflect pad, power 2, onesided, HTK mel filterbank without
normalisation over [0, sr//2], 10*log10(clamp(x, 1e-10)).

The kernels take n_fft a power of two in [64, 2048] and n_mels <= 256; other sizes (the
reference accepts any) run the same definition through torch.stft on the device
(``_torch_melspec``).
"""
import math

import numpy as np
import torch

from ._lib import check, lib, ptr, require_cuda, stream_of

_FB = {}
_TABLES = {}


def _hz_to_mel(f):
    return 2595.0 * math.log10(1.0 + (f / 700.0))


def mel_filterbank(n_fft, n_mels, sample_rate, device):
    """torchaudio.functional.melscale_fbanks(n_fft//2+1, 0, sr//2, n_mels, sr, norm=None, 'htk')
    (float32, as torchaudio builds it) and the periodic Hann window."""
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


def kernel_supported(n_fft, n_mels=128):
    return 64 <= n_fft <= 2048 and n_fft & (n_fft - 1) == 0 and n_mels <= 256


class MelTables:
    """The device tables wam_melspec / wam_melspec_adjoint read (include/wam_hip.h): window,
    twiddles (float64 -> float32), and the filterbank's nonzeros in CSR form by band and by bin."""

    def __init__(self, n_fft, n_mels, sample_rate, device):
        fb, win = mel_filterbank(n_fft, n_mels, sample_rate, "cpu")
        fbn = fb.numpy()
        nz_bin, nz_band = np.nonzero(fbn)                      # row-major: by bin, bands ascending
        by_band = np.lexsort((nz_bin, nz_band))               # by band, bins ascending
        band_ptr = np.searchsorted(nz_band[by_band], np.arange(n_mels + 1))
        bin_ptr = np.searchsorted(nz_bin, np.arange(n_fft // 2 + 2))
        tw = np.exp(-2j * np.pi * np.arange(n_fft) / n_fft)
        tables = np.concatenate([win.numpy().astype(np.float32),
                                 np.stack([tw.real, tw.imag], 1).reshape(-1).astype(np.float32),
                                 fbn[nz_bin[by_band], nz_band[by_band]], fbn[nz_bin, nz_band]]).astype(np.float32)
        index = np.concatenate([band_ptr, nz_bin[by_band], bin_ptr, nz_band]).astype(np.int32)
        self.n_fft, self.n_mels, self.nnz = n_fft, n_mels, int(len(nz_bin))
        self.tables = torch.tensor(tables, device=device)
        self.index = torch.tensor(index, device=device)

    @staticmethod
    def get(n_fft, n_mels, sample_rate, device):
        key = (n_fft, n_mels, sample_rate, torch.device(device))
        if key not in _TABLES:
            _TABLES[key] = MelTables(n_fft, n_mels, sample_rate, device)
        return _TABLES[key]


def _frames(samples, n_fft):
    if samples <= n_fft // 2:
        raise RuntimeError("melspec: reflect padding of %d needs more than %d samples, got %d"
                           % (n_fft // 2, n_fft // 2, samples))
    return samples // (n_fft // 2) + 1


def mel_forward(wave, n_fft, sample_rate, n_mels, to_db=True):
    """wave [B, T] float32 (device) -> [B, frames, n_mels] (dB when to_db) on the kernel."""
    require_cuda(wave, "waveform")
    wave = wave.contiguous()
    b, t = wave.shape
    tb = MelTables.get(n_fft, n_mels, sample_rate, wave.device)
    out = torch.empty((b, _frames(t, n_fft), n_mels), dtype=torch.float32, device=wave.device)
    check(lib.wam_melspec(b, t, n_fft, n_mels, tb.nnz, int(to_db), ptr(wave), ptr(tb.tables), ptr(tb.index), ptr(out),
                          stream_of(wave.device)))
    return out


def mel_adjoint(wave, grad_out, n_fft, sample_rate, n_mels, to_db=True):
    """d/dwave of <grad_out, mel_forward(wave)>: grad_out [B, frames, n_mels] -> [B, T]."""
    require_cuda(wave, "waveform")
    wave = wave.contiguous()
    b, t = wave.shape
    g = grad_out.reshape(b, _frames(t, n_fft), n_mels).to(torch.float32).contiguous()
    tb = MelTables.get(n_fft, n_mels, sample_rate, wave.device)
    out = torch.empty_like(wave)
    check(lib.wam_melspec_adjoint(b, t, n_fft, n_mels, tb.nnz, int(to_db), ptr(wave), ptr(g), ptr(tb.tables),
                                  ptr(tb.index), ptr(out), stream_of(wave.device)))
    return out


class _MelFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, wave, n_fft, sample_rate, n_mels, to_db):
        ctx.save_for_backward(wave)
        ctx.args = (n_fft, sample_rate, n_mels, to_db)
        return mel_forward(wave, n_fft, sample_rate, n_mels, to_db)

    @staticmethod
    def backward(ctx, g):
        (wave,) = ctx.saved_tensors
        return mel_adjoint(wave, g, *ctx.args), None, None, None, None


def _torch_melspec(wave, n_fft, sample_rate, n_mels, to_db):
    fb, win = mel_filterbank(n_fft, n_mels, sample_rate, wave.device)
    spec = torch.stft(wave, n_fft=n_fft, hop_length=n_fft // 2, win_length=n_fft, window=win, center=True,
                      pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    mel = torch.matmul(spec.abs().pow(2.0).transpose(-1, -2), fb)   # [B, frames, n_mels]
    return 10.0 * torch.log10(torch.clamp(mel, min=1e-10)) if to_db else mel


def melspec_db(wave, n_fft, sample_rate, n_mels):
    """wave [B, T] -> [B, 1, frames, n_mels] (the reference's stacked ``.T`` layout), differentiable."""
    if kernel_supported(n_fft, n_mels):
        return _MelFn.apply(wave, n_fft, sample_rate, n_mels, True).unsqueeze(1)
    return _torch_melspec(wave, n_fft, sample_rate, n_mels, True).unsqueeze(1)


def melspec_power(wave, n_fft, sample_rate, n_mels):
    """torchaudio MelSpectrogram (power, no dB) of [B, T] -> [B, n_mels, frames]."""
    if kernel_supported(n_fft, n_mels):
        return _MelFn.apply(wave, n_fft, sample_rate, n_mels, False).transpose(-1, -2)
    return _torch_melspec(wave, n_fft, sample_rate, n_mels, False).transpose(-1, -2)
