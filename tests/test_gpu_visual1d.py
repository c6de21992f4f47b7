"""Row f2 (VisualizerWAM1D and BaseWAM1D.filter) on the GPU vs the reference's own outputs made with
the real PyWavelets 1.1.1 (tests/golden/f2_goldens.npz, make_f2_goldens.py). The coefficients fed
in here come from the oracle DWT (pinned to pywt at float32 rounding), so the bar is 1e-5 of the
signal's scale."""
import numpy as np
import pytest
import torch

import testmodels
from tests.golden.make_f2_goldens import CASES, inputs
from tests.helpers import npz

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def W():
    import wam_amd
    return wam_amd


def _close(a, b):
    return np.abs(a - b).max() <= 1e-5 * max(1.0, np.abs(b).max())


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("method", ["ht", "st", "modulation"])
def test_filter_from_wavelet_coefficients(W, name, method):
    wav, J, shape, seed = CASES[name]
    _, coeffs, grads = inputs(wav, J, shape, seed)
    v = W.VisualizerWAM1D(testmodels.TinyAudio().cuda(), np.zeros(shape, np.float32), wavelet=wav, J=J)
    got = v.filter_from_wavelet_coefficients(coeffs, grads, filtering_method=method, EPS=0.2)
    ref = npz("f2_goldens.npz")["%s_%s" % (name, method)]
    assert got.shape == ref.shape and _close(got, ref), np.abs(got - ref).max()


@pytest.mark.parametrize("name", list(CASES))
def test_basewam1d_filter(W, name):
    from wam_amd.plan import get_plan
    wav, J, shape, seed = CASES[name]
    _, coeffs, grads = inputs(wav, J, shape, seed)
    b = W.BaseWAM1D(testmodels.TinyAudio().cuda(), wavelet=wav, J=J, mode="reflect")
    p = get_plan(1, (shape[1],), J, wav, "reflect", "cuda")
    flat = lambda bands: torch.cat([torch.tensor(c).reshape(-1) for c in bands]).cuda()  # noqa: E731
    n = shape[0]
    b._record(p, flat(coeffs), n, 0, flat(grads), n, 0, n)
    got = b.filter(0.3)
    ref = npz("f2_goldens.npz")["%s_filter" % name]
    assert got.shape == ref.shape and _close(got, ref), np.abs(got - ref).max()


def test_melspec_filters_and_spectrogram(W):
    """filter_melspec ('ht' / 'modulation') vs numpy on the same arrays; the power mel spectrogram
    vs the torch restatement of torchaudio (oracle/melspec.py; parity unpinned offline)."""
    from oracle import melspec as om
    rs = np.random.RandomState(3)
    x = rs.standard_normal((2, 8000)).astype(np.float32)
    v = W.VisualizerWAM1D(testmodels.TinyAudio().cuda(), x, wavelet="haar", J=2, sample_rate=16000)
    mel = v.compute_melspec(x)
    ref = om.MelSpectrogram(sample_rate=16000, n_fft=1024, n_mels=128)(torch.tensor(x)).numpy()
    assert mel.shape == ref.shape and np.abs(mel - ref).max() <= 1e-4 * np.abs(ref).max()
    g = rs.standard_normal((2, mel.shape[2], mel.shape[1])).astype(np.float32)
    gt = np.transpose(g, (0, 2, 1))
    ht = v.filter_melspec(mel, g, "ht", EPS=0.2)
    gn = (gt - gt.min()) / (gt.max() - gt.min())
    assert np.allclose(ht, mel * (gn > 0.2), rtol=1e-6, atol=0)
    assert np.allclose(v.filter_melspec(mel, g, "modulation"), mel * np.abs(gt), rtol=1e-6, atol=0)
    spec = v.spectrogram_from_waveform(x)
    assert spec.shape == (2, 513, 8000 // 256 + 1)


def _record_gap(rec):
    """The compute_spectrogram gap to the oracle's librosa restatement, appended as one JSON line to
    $WAM_TEST_RECORD_DIR (default gpurun_out/, merged back from the GPU box) so that the measured
    agreement is on record (profiles/r06*_compute_spectrogram_gap.jsonl)."""
    import json
    import os
    d = os.environ.get("WAM_TEST_RECORD_DIR", os.path.join(os.path.dirname(os.path.dirname(__file__)), "gpurun_out"))
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "compute_spectrogram_gap.jsonl"), "a") as f:
        f.write(json.dumps(rec) + "\n")


def _nnls_obj(A, x, B):
    return 0.5 * float(np.sum((A.astype(np.float64) @ x.astype(np.float64) - B) ** 2))


# magnitudes vs the oracle's librosa restatement: the device evaluates the same float64 objective
# in another summation order and starts from its own fp32 GEMM pinv(A) @ B. L-BFGS-B carries a
# one-ulp change of that start into up to ~7e-4 rel-L2 / 1e-2 of max of its result (one iteration
# more or less before the projected-gradient stop; measured on the reference algorithm itself,
# tests/test_oracle.py::test_librosa_lbfgsb_start_sensitivity), i.e. librosa's own result moves by
# that much with the BLAS it runs on; typical cases agree to 1e-7
SPEC_REL_L2 = 2e-3
SPEC_MAX_OVER_MAX = 2e-2


@pytest.mark.parametrize("sr,n_fft,n_mels,T", [(16000, 256, 32, 24), (16000, 1024, 128, 40), (44100, 512, 64, 17)])
def test_compute_spectrogram_matches_librosa_lbfgsb(W, sr, n_fft, n_mels, T):
    """compute_spectrogram / process_in_chunks (lib/wam_1D.py:442-448,478-488: librosa mel_to_stft
    per chunk = clipped pinv start + scipy L-BFGS-B on 0.5 / B.size ||A x - B||^2, then sqrt) with the
    objective evaluated on the device, vs the oracle's restatement of librosa's algorithm
    (oracle/melspec.py process_in_chunks) on the same mel spectrograms and chunks: rel-L2 <=
    SPEC_REL_L2 and max |diff| <= SPEC_MAX_OVER_MAX of max |ref| per waveform, on all six recorded
    (shape, waveform) cases. Parity unpinned (librosa absent): the basis and the solver are
    restatements of librosa's published algorithm. nnls="exact" (build-only keyword) returns the exact
    minimiser: its re-projection A x agrees with scipy's active-set NNLS to 1e-4 of max |B|, and its
    objective is never above the L-BFGS-B one."""
    from oracle import melspec as om
    rs = np.random.RandomState(n_fft)
    x = rs.standard_normal((2, (T - 1) * (n_fft // 2))).astype(np.float32)
    v = W.VisualizerWAM1D(testmodels.TinyAudio().cuda(), x, wavelet="haar", J=2, sample_rate=sr, n_fft=n_fft,
                          n_mels=n_mels)
    mel = v.compute_melspec(x)                        # torchaudio HTK power mel [2, n_mels, T]
    assert mel.shape == (2, n_mels, T)
    spec = v.compute_spectrogram(mel, chunk_size=7)
    assert spec.shape == (2, n_fft // 2 + 1, T) and spec.dtype == np.float32 and (spec >= 0).all()
    exact = v.compute_spectrogram(mel, chunk_size=7, nnls="exact")
    A = om.slaney_mel_basis(sr, n_fft, n_mels)
    for i in range(2):
        ref = om.process_in_chunks(mel[i], 7, sr, n_fft)
        l2 = float(np.linalg.norm(spec[i] - ref) / max(1e-30, np.linalg.norm(ref)))
        mx = float(np.abs(spec[i] - ref).max() / max(1e-30, np.abs(ref).max()))
        B = mel[i].astype(np.float64)
        xe = om.nnls_exact(A, B)
        xg = exact[i].astype(np.float64) ** 2
        err = np.abs(A @ xg - A @ xe).max() / np.abs(B).max()
        fo, fe, fl = _nnls_obj(A, xg, B), _nnls_obj(A, xe, B), _nnls_obj(A, ref.astype(np.float64) ** 2, B)
        _record_gap({"sr": sr, "n_fft": n_fft, "n_mels": n_mels, "frames": T, "chunk": 7, "waveform": i,
                     "lbfgsb_rel_l2": l2, "lbfgsb_max_over_max": mx,
                     "exact_reprojection_gap_over_max_B": float(err), "objective_exact_device": fo,
                     "objective_exact_nnls": fe, "objective_lbfgsb_oracle": fl})
        assert l2 <= SPEC_REL_L2 and mx <= SPEC_MAX_OVER_MAX, (i, l2, mx)
        assert err <= 1e-4 and fo <= fe * (1 + 1e-5) + 1e-12 * np.sum(B ** 2), (i, err, fo, fe)
        assert fo <= fl * (1 + 1e-6)
    # process_in_chunks (module function, lib/wam_1D.py:442-448) at another chunking
    from wam_amd.wam_1D import process_in_chunks
    pc = process_in_chunks(mel[1], 5, sr, n_fft)
    ref = om.process_in_chunks(mel[1], 5, sr, n_fft)
    assert pc.shape == ref.shape and pc.dtype == np.float32 and (pc >= 0).all()
    assert np.linalg.norm(pc - ref) <= SPEC_REL_L2 * np.linalg.norm(ref)
    assert np.abs(pc - ref).max() <= SPEC_MAX_OVER_MAX * np.abs(ref).max()
    with pytest.raises(ValueError):
        process_in_chunks(mel[1], 0, sr, n_fft)
    with pytest.raises(ValueError):
        v.compute_spectrogram(mel, nnls="fista")


def test_filtered_spectrogram_from_melspec(W):
    """lib/wam_1D.py:619-643 end to end: the source spectrogram is the inversion of the waveform's mel
    spectrogram, the filtered one the inversion of filter_melspec's output."""
    rs = np.random.RandomState(5)
    x = rs.standard_normal((2, 4096)).astype(np.float32)
    v = W.VisualizerWAM1D(testmodels.TinyAudio().cuda(), x, wavelet="haar", J=2, sample_rate=16000, n_fft=256,
                          n_mels=32)
    mel = v.compute_melspec(x)
    g = rs.standard_normal((2, mel.shape[2], mel.shape[1])).astype(np.float32)
    src, filt = v.filtered_spectrogram_from_melspec(g, "ht", EPS=0.3, chunk_size=10)
    assert src.shape == filt.shape == (2, 129, mel.shape[2])
    assert np.array_equal(src, v.source_spectrograms)
    assert np.abs(src - v.compute_spectrogram(mel, chunk_size=10)).max() <= 1e-6 * np.abs(src).max()
    want = v.compute_spectrogram(v.filter_melspec(mel, g, "ht", EPS=0.3), chunk_size=10)
    assert np.abs(filt - want).max() <= 1e-6 * max(1e-30, np.abs(want).max())
