"""Row f2 front-end on the GPU: k_mel_fwd / k_mel_adj (wam_amd/melspec.py) vs the torchaudio
MelSpectrogram + AmplitudeToDB restatement (oracle/melspec.py filterbank, torch.stft) evaluated in
float64 on the CPU, and its autograd gradient. Parity unpinned offline (no torchaudio fixtures).
The kernels take n_fft a power of two in [64, 2048] and n_mels <= 256 (torch.stft beyond). The bar
is fp32 FFT rounding: power within 2e-5 of each waveform's peak band, dB within 2e-3 dB on bands
above 1e-6 of the peak, gradients within 1e-4 of their max."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = {  # name: (n_fft, samples, n_mels, sample_rate)
    "c3_1024": (1024, 80000, 128, 16000),
    "sr44k_1024": (1024, 8000, 128, 44100),
    "n256_ragged": (256, 1001, 40, 8000),
    "n64_min_T": (64, 33, 8, 16000),
    "n2048_T_multiple_of_hop": (2048, 4096, 128, 44100),
    "n2048_256mels": (2048, 10000, 256, 44100),
    "n512_two_frames": (512, 300, 64, 22050),
}


@pytest.fixture(scope="module")
def M():
    from wam_amd import melspec
    return melspec


def _reference(x, n_fft, n_mels, sr, to_db):
    """float64 CPU autograd chain of torchaudio's definition (oracle filterbank and window)."""
    from oracle import melspec as om
    fb = om.melscale_fbanks(n_fft // 2 + 1, 0.0, float(sr // 2), n_mels, sr).double()
    win = torch.hann_window(n_fft).double()
    spec = torch.stft(x, n_fft=n_fft, hop_length=n_fft // 2, win_length=n_fft, window=win, center=True,
                      pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    mel = torch.matmul(spec.abs().pow(2.0).transpose(-1, -2), fb)
    return 10.0 * torch.log10(torch.clamp(mel, min=1e-10)) if to_db else mel


def _signal(b, t, seed):
    rs = np.random.RandomState(seed)
    tt = np.arange(t) / 16000.0
    x = 0.1 * rs.standard_normal((b, t))
    for i in range(b):
        for f in rs.uniform(50, 4000, size=3):
            x[i] += np.sin(2 * np.pi * f * tt)
    return x.astype(np.float32)


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("to_db", [True, False])
def test_forward(M, name, to_db):
    n_fft, t, n_mels, sr = CASES[name]
    x = _signal(2, t, 5)
    got = M.mel_forward(torch.tensor(x).cuda(), n_fft, sr, n_mels, to_db).cpu().double()
    ref = _reference(torch.tensor(x).double(), n_fft, n_mels, sr, to_db)
    assert got.shape == ref.shape
    if to_db:
        lin = _reference(torch.tensor(x).double(), n_fft, n_mels, sr, False)
        live = lin > 1e-6 * lin.amax(dim=(1, 2), keepdim=True)
        err = (got - ref).abs()[live].max().item()
        assert err <= 2e-3, err
        # empty bands: 10 log10(float32(1e-10)) = -100 (to float32 rounding)
        assert (got[lin == 0] + 100).abs().max().item() <= 1e-4 if (lin == 0).any() else True
    else:
        err = ((got - ref).abs() / ref.amax(dim=(1, 2), keepdim=True)).max().item()
        assert err <= 2e-5, err


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("to_db", [True, False])
def test_adjoint_vs_autograd(M, name, to_db):
    n_fft, t, n_mels, sr = CASES[name]
    x = _signal(2, t, 6)
    xd = torch.tensor(x).double().requires_grad_(True)
    ref = _reference(xd, n_fft, n_mels, sr, to_db)
    g = torch.tensor(np.random.RandomState(7).standard_normal(tuple(ref.shape)))
    (ref_grad,) = torch.autograd.grad(ref, xd, grad_outputs=g)
    got = M.mel_adjoint(torch.tensor(x).cuda(), g.float().cuda(), n_fft, sr, n_mels, to_db).cpu().double()
    err = ((got - ref_grad).abs().max() / ref_grad.abs().max()).item()
    assert err <= 1e-4, err


def test_autograd_function_and_layout(M):
    """melspec_db: [B, 1, F, n_mels] and differentiable through k_mel_adj."""
    x = torch.tensor(_signal(3, 8000, 8)).cuda().requires_grad_(True)
    db = M.melspec_db(x, 1024, 16000, 128)
    assert db.shape == (3, 1, 8000 // 512 + 1, 128)
    g = torch.randn_like(db)
    (gx,) = torch.autograd.grad(db, x, grad_outputs=g)
    assert torch.equal(gx, M.mel_adjoint(x.detach(), g, 1024, 16000, 128))
    power = M.melspec_power(x.detach(), 1024, 16000, 128)
    assert power.shape == (3, 128, 8000 // 512 + 1)


def test_deterministic(M):
    x = torch.tensor(_signal(4, 20000, 9)).cuda()
    g = torch.randn(4, 20000 // 512 + 1, 128, device="cuda")
    a = M.mel_adjoint(x, g, 1024, 16000, 128)
    b = M.mel_adjoint(x, g, 1024, 16000, 128)
    assert torch.equal(a, b)
    assert torch.equal(M.mel_forward(x, 1024, 16000, 128), M.mel_forward(x, 1024, 16000, 128))


def test_errors(M):
    from wam_amd._lib import WamError
    x = torch.zeros(1, 512, device="cuda")
    with pytest.raises(RuntimeError):
        M.mel_forward(x, 1024, 16000, 128)  # reflect pad of 512 needs more than 512 samples
    with pytest.raises(WamError):
        M.mel_forward(torch.zeros(1, 5000, device="cuda"), 4096, 16000, 128)  # beyond the kernel's n_fft
    with pytest.raises(WamError):
        M.mel_forward(torch.zeros(1, 5000, device="cuda"), 1024, 16000, 300)  # beyond the kernel's n_mels
    # non-power-of-two n_fft: the same definition through torch.stft on the device
    y = torch.tensor(_signal(1, 4000, 3)).cuda()
    ref = _reference(y.cpu().double(), 400, 64, 16000, True)
    got = M.melspec_db(y, 400, 16000, 64)[:, 0].cpu().double()
    lin = _reference(y.cpu().double(), 400, 64, 16000, False)
    live = lin > 1e-6 * lin.max()
    assert (got - ref).abs()[live].max() <= 2e-3
