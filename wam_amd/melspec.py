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


# ------------------------------------------------------------------------------ mel inversion (f2)
_MELINV = {}


def _slaney_hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep, f / f_sp)


def _slaney_mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def slaney_mel_basis(sample_rate, n_fft, n_mels):
    """librosa.filters.mel(sr, n_fft, n_mels, dtype=float32) defaults (the basis
    librosa.feature.inverse.mel_to_stft inverts, lib/wam_1D.py:446): Slaney mel scale (htk=False),
    fmin 0, fmax sr / 2, triangles over the rfft bin frequencies (np.fft.rfftfreq), each triangle
    rounded to float32 and then scaled by the 'slaney' area norm 2 / (f[i+2] - f[i]) in float64 and
    rounded again -- librosa's own rounding sequence. [n_mels, 1 + n_fft // 2] float32.
    Published algorithm of librosa (absent offline: parity unpinned)."""
    fftfreqs = np.arange(0, 1 + n_fft // 2) * (1.0 / (n_fft * (1.0 / sample_rate)))
    mel_f = _slaney_mel_to_hz(np.linspace(_slaney_hz_to_mel(0.0), _slaney_hz_to_mel(float(sample_rate) / 2),
                                          n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    w = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, np.newaxis]
    return w


class MelInverse:
    """Device data of the NNLS mel inversion for one (sr, n_fft, n_mels): the float32 basis A [M, F]
    and A^T; the basis widened to float64 (A64, A64^T: librosa's objective multiplies the float32
    basis into float64 iterates); pinv(A) [F, M] computed as librosa does (np.linalg.pinv of the
    float32 basis, i.e. a float32 SVD: librosa's initial point); for the exact solver the Gram
    matrix A^T A and the Lipschitz constant ||A||_2^2 (float64 on the host)."""

    def __init__(self, sample_rate, n_fft, n_mels, device):
        A = slaney_mel_basis(sample_rate, n_fft, n_mels)
        A64 = A.astype(np.float64)
        self.n_mels = n_mels
        self.lip = float(np.linalg.norm(A64, 2) ** 2)
        self.A = torch.tensor(A, device=device)
        self.At = self.A.t().contiguous()
        self.A64 = torch.tensor(A64, device=device)
        self.A64t = self.A64.t().contiguous()
        self.G = torch.tensor((A64.T @ A64).astype(np.float32), device=device)
        self.pinv = torch.tensor(np.linalg.pinv(A), device=device)

    @staticmethod
    def get(sample_rate, n_fft, n_mels, device):
        key = (sample_rate, n_fft, n_mels, torch.device(device))
        if key not in _MELINV:
            _MELINV[key] = MelInverse(sample_rate, n_fft, n_mels, device)
        return _MELINV[key]


# librosa.util.MAX_MEM_BLOCK: librosa's nnls solves at most this many bytes of columns per L-BFGS-B run
MAX_MEM_BLOCK = 2 ** 8 * 2 ** 10


def lbfgsb_columns(n_mels, itemsize=4):
    """Columns per L-BFGS-B block in librosa.util.nnls for a [n_mels, T] float32 right-hand side."""
    return max(1, int(MAX_MEM_BLOCK // (n_mels * itemsize)))


def nnls_lbfgsb_block(evaluate, x0, m):
    """One librosa ``_nnls_lbfgs_block``: scipy.optimize.fmin_l_bfgs_b with bounds x >= 0 and history
    m = A.shape[1] from x0 (float32 [F, T], already clipped), scipy's default tolerances (factr 1e7,
    pgtol 1e-5, 15,000 iterations / evaluations). evaluate(x float64 flat) -> (value, gradient flat)
    is the objective 0.5 / B.size * ||A x - B||^2. Host logic only; returns float64 [F, T]."""
    import scipy.optimize
    shape = tuple(x0.shape)
    xi = np.asarray(x0)
    x, _, _ = scipy.optimize.fmin_l_bfgs_b(evaluate, xi, bounds=[(0, None)] * xi.size, m=m)
    return x.reshape(shape)


def device_objective(inv, B):
    """librosa's ``_nnls_obj`` for one block on the device in float64: diff = A x - B (the float32
    basis and right-hand side widened, as numpy's einsum widens them against the float64 iterate),
    value = (1 / B.size) * 0.5 * sum(diff^2), gradient = (1 / B.size) * A^T diff. The iterate goes
    host -> device and (value, gradient) device -> host once per evaluation through pinned buffers
    (scipy's L-BFGS-B drives the iteration on the host, as in the reference)."""
    F, T = inv.A.shape[1], B.shape[1]
    dev = B.device
    B64 = B.to(torch.float64)
    scale = 1.0 / B.numel()
    xh = torch.empty(F * T, dtype=torch.float64, pin_memory=True)
    oh = torch.empty(F * T + 1, dtype=torch.float64, pin_memory=True)
    xd = torch.empty((F, T), dtype=torch.float64, device=dev)
    od = torch.empty(F * T + 1, dtype=torch.float64, device=dev)
    xh_np, oh_np = xh.numpy(), oh.numpy()

    def evaluate(x):
        xh_np[:] = x
        xd.view(-1).copy_(xh, non_blocking=True)
        diff = torch.mm(inv.A64, xd).sub_(B64)                              # A x - B
        od[:1].copy_(torch.sum(diff * diff).view(1)).mul_(scale * 0.5)
        torch.mm(inv.A64t, diff, out=od[1:].view(F, T))
        od[1:].mul_(scale)
        oh.copy_(od, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        return float(oh_np[0]), oh_np[1:].copy()
    return evaluate


def nnls_lbfgsb(inv, B):
    """librosa.util.nnls(A, B) for a [M, T] float32 device block, the algorithm lib/wam_1D.py:446
    runs: x_init = clip(pinv(A) @ B, 0) (float32, on the device); if the T columns fit
    MAX_MEM_BLOCK one L-BFGS-B run over all of them, else one per block of lbfgsb_columns(M)
    columns, each from its own columns of x_init; the float64 result rounded to float32.
    -> [F, T] float32 on B's device."""
    M, T = B.shape
    x_init = torch.clamp(inv.pinv @ B, min=0.0)
    n_col = lbfgsb_columns(M)
    m = int(inv.A.shape[1])
    if T <= n_col:
        x = nnls_lbfgsb_block(device_objective(inv, B), x_init.cpu().numpy(), m)
        return torch.from_numpy(x.astype(np.float32)).to(B.device)
    x = x_init.clone()
    for s0 in range(0, T, n_col):
        s1 = min(s0 + n_col, T)
        blk = nnls_lbfgsb_block(device_objective(inv, B[:, s0:s1].contiguous()), x_init[:, s0:s1].cpu().numpy(), m)
        x[:, s0:s1] = torch.from_numpy(blk).to(B.device)
    return x


def nnls_mel(inv, B, max_iter=3000, tol=1e-6):
    """min_x 0.5 ||A x - B||^2 s.t. x >= 0, column by column, B [..., M, T] (device) -> x [..., F, T].
    The exact minimiser (``nnls="exact"``; the default follows librosa: nnls_lbfgsb).

    librosa's nnls (the algorithm lib/wam_1D.py:446 runs) starts from the clipped minimum-norm
    least-squares solution and runs scipy's L-BFGS-B. Here every column of the batch runs FISTA
    (accelerated projected gradient, step 1 / ||A||^2, gradient-restarted momentum) from the same
    initial point; each iteration is one GEMM with the Gram matrix (hipBLASLt) plus elementwise
    updates. The mel basis has more bins than bands, so the minimiser x is not unique, but its
    re-projection A x is (the objective is strictly convex in A x): that is what the tests compare.
    Stops when the KKT residual max |min(x, grad)| of every column is <= tol * max |A^T B| or
    after max_iter iterations. librosa's L-BFGS-B stops at an absolute projected-gradient tolerance
    (pgtol 1e-5 on an objective scaled by 1 / B.size), i.e. earlier and data-scale dependent: its
    objective is never below the NNLS optimum this converges to (tests/test_gpu_visual1d.py)."""
    shape = B.shape
    M, T = shape[-2], shape[-1]
    Bc = B.reshape(-1, M, T).permute(1, 0, 2).reshape(M, -1).to(torch.float32)   # [M, cols]
    AtB = inv.At @ Bc                                                              # [F, cols]
    x = torch.clamp(inv.pinv @ Bc, min=0.0)
    y = x.clone()
    t = torch.ones(x.shape[1], dtype=torch.float32, device=x.device)   # momentum per column
    step = 1.0 / inv.lip
    scale = float(AtB.abs().max()) if AtB.numel() else 0.0  # the gradient's scale at x = 0
    stop = tol * max(scale, 1e-30)
    for it in range(max_iter):
        grad = inv.G @ y - AtB
        x_new = torch.clamp(y - step * grad, min=0.0)
        if it % 25 == 24:  # the only host synchronisation: the KKT residual every 25 iterations
            kkt = torch.minimum(x_new, inv.G @ x_new - AtB).abs().max()
            if float(kkt) <= stop:
                x = x_new
                break
        # gradient restart per column (O'Donoghue & Candes): momentum dropped where it points uphill
        d = x_new - x
        restart = (grad * d).sum(0) > 0
        t_new = 0.5 * (1.0 + torch.sqrt(1.0 + 4.0 * t * t))
        beta = torch.where(restart, torch.zeros_like(t), (t - 1.0) / t_new)
        t = torch.where(restart, torch.ones_like(t), t_new)
        y = x_new + beta * d
        x = x_new
    F = x.shape[0]
    return x.reshape(F, -1, T).permute(1, 0, 2).reshape(shape[:-2] + (F, T))


NNLS_METHODS = ("lbfgsb", "exact")


def mel_to_stft(M, sample_rate, n_fft, power=2.0, nnls="lbfgsb"):
    """librosa.feature.inverse.mel_to_stft(M, sr, n_fft) (power 2): NNLS of the Slaney mel basis,
    then x ** (1 / power) in float32. M [n_mels, T] (or [..., n_mels, T] with nnls="exact") on the
    device. nnls="lbfgsb" (default) is librosa's solver (nnls_lbfgsb: the reference's result);
    nnls="exact" returns the exact minimiser of the same problem (nnls_mel, batched FISTA)."""
    require_cuda(M, "mel spectrogram")
    if nnls not in NNLS_METHODS:
        raise ValueError("nnls must be one of %s, got %r" % (NNLS_METHODS, nnls))
    inv = MelInverse.get(sample_rate, n_fft, M.shape[-2], M.device)
    if nnls == "exact":
        return nnls_mel(inv, M).pow(1.0 / power)
    if M.dim() != 2:
        raise ValueError("librosa's nnls takes one [n_mels, T] spectrogram per call, got %s" % (tuple(M.shape),))
    return nnls_lbfgsb(inv, M.to(torch.float32).contiguous()).pow(1.0 / power)
