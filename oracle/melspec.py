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


# ---------------------------------------------------------------------------- librosa mel inversion
def slaney_mel_basis(sr, n_fft, n_mels):
    """librosa.filters.mel(sr=sr, n_fft=n_fft, n_mels=n_mels, dtype=float32) with its defaults
    (htk=False: Slaney scale, linear below 1 kHz at 200/3 Hz per mel, logarithmic above with step
    ln(6.4)/27; fmin 0, fmax sr/2; norm='slaney'), element by element in librosa's rounding order:
    bin frequencies j * (1 / (n_fft * (1 / sr))) (np.fft.rfftfreq), mel points by np.linspace, each
    triangle value rounded to float32, then multiplied by the float64 area norm 2 / (f[i+2] - f[i])
    and rounded again."""
    import numpy as np

    def hz2mel(f):
        return f / (200.0 / 3) if f < 1000.0 else 1000.0 / (200.0 / 3) + math.log(f / 1000.0) / (math.log(6.4) / 27.0)

    def mel2hz(m):
        return (200.0 / 3) * m if m < 1000.0 / (200.0 / 3) else 1000.0 * math.exp((math.log(6.4) / 27.0) * (m - 1000.0 / (200.0 / 3)))

    n_f = 1 + n_fft // 2
    step = 1.0 / (n_fft * (1.0 / sr))
    freqs = [j * step for j in range(n_f)]
    pts = [mel2hz(float(m)) for m in np.linspace(hz2mel(0.0), hz2mel(float(sr) / 2), n_mels + 2)]
    w = np.zeros((n_mels, n_f), dtype=np.float32)
    for i in range(n_mels):
        norm = 2.0 / (pts[i + 2] - pts[i])
        for j, f in enumerate(freqs):
            lower = -(pts[i] - f) / (pts[i + 1] - pts[i])
            upper = (pts[i + 2] - f) / (pts[i + 2] - pts[i + 1])
            w[i, j] = np.float32(float(np.float32(max(0.0, min(lower, upper)))) * norm)
    return w


MAX_MEM_BLOCK = 2 ** 8 * 2 ** 10  # librosa.util.MAX_MEM_BLOCK


def _nnls_obj(x, shape, A, B):
    """librosa.util._nnls._nnls_obj: float64 objective / gradient of a float32 basis and data."""
    import numpy as np
    x = x.reshape(shape)
    diff = A.astype(np.float64) @ x - B
    return (1 / B.size) * 0.5 * np.sum(diff ** 2), ((1 / B.size) * (A.astype(np.float64).T @ diff)).ravel()


def _nnls_lbfgs_block(A, B, x_init):
    import scipy.optimize
    shape = x_init.shape
    x, _, _ = scipy.optimize.fmin_l_bfgs_b(_nnls_obj, x_init, args=(shape, A, B), bounds=[(0, None)] * x_init.size,
                                           m=A.shape[1])
    return x.reshape(shape)


def nnls(A, B):
    """librosa.util.nnls(A, B) for a 2D float32 B [M, T]: x_init = clip(pinv(A) @ B, 0) in float32;
    scipy L-BFGS-B (bounds x >= 0, history m = A.shape[1], scipy's default tolerances) on
    0.5 / B.size * ||A x - B||^2 over all columns if they fit MAX_MEM_BLOCK bytes, else per block of
    columns (each block from its own columns of x_init); result in A's dtype."""
    import numpy as np
    n_columns = max(int(MAX_MEM_BLOCK // (B.shape[0] * A.itemsize)), 1)
    x_init = np.linalg.pinv(A) @ B
    np.clip(x_init, 0, None, out=x_init)
    if B.shape[-1] <= n_columns:
        return _nnls_lbfgs_block(A, B, x_init).astype(A.dtype)
    x = x_init.copy()
    for s in range(0, B.shape[-1], n_columns):
        t = min(s + n_columns, B.shape[-1])
        x[:, s:t] = _nnls_lbfgs_block(A, B[:, s:t], x_init[:, s:t])
    return x


def mel_to_stft(M, sr, n_fft, power=2.0):
    """librosa.feature.inverse.mel_to_stft (librosa's published algorithm; librosa is absent
    offline): A = the float32 mel basis of M's dtype, nnls(A, M), then x ** (1 / power) in float32.
    M [n_mels, T] float32."""
    import numpy as np
    B = np.asarray(M, dtype=np.float32)
    A = slaney_mel_basis(sr, n_fft, B.shape[0])
    x = nnls(A, B)
    return np.power(x, 1.0 / power, out=x), A


def process_in_chunks(melspec, chunk_size, sr, n_fft):
    """lib/wam_1D.py:442-448: mel_to_stft per chunk of chunk_size frames, hstacked."""
    import numpy as np
    return np.hstack([mel_to_stft(melspec[:, i:i + chunk_size], sr, n_fft)[0]
                      for i in range(0, melspec.shape[1], chunk_size)])


def nnls_exact(A, B):
    """Column-wise exact NNLS in float64: bounded-variable least squares (scipy.optimize.lsq_linear
    method='bvls', an active-set method that terminates at the optimum). scipy 1.15's nnls was
    seen returning non-optimal points on these underdetermined bases, so it is not used."""
    import numpy as np
    import scipy.optimize
    A = np.asarray(A, dtype=np.float64)
    B = np.asarray(B, dtype=np.float64)
    return np.stack([scipy.optimize.lsq_linear(A, B[:, j], bounds=(0, np.inf), method="bvls", tol=1e-14,
                                               max_iter=20 * A.shape[1]).x for j in range(B.shape[1])], 1)
