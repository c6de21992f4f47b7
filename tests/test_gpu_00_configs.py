"""GPU parity at the five BASELINE configurations (c1-c5), class level, against the oracle
(oracle/wam_ref.py, the reference glue restated on the CPU) on this box's CPU. This module sorts
first in the suite so that an early -x stop cannot hide the configuration tests.

* c1  -- haar J=3 SmoothGrad n=25, random-init ResNet-18, the elephant crop, numpy noise
         (statistical ReLU-network bar);
* c2  -- db4 J=3 SmoothGrad n=25 at 224^2, ResNet-50 fp32, numpy noise (statistical bar), and the
         bench's Philox path on a kink-free model against the oracle fed the same noise;
* c3  -- db6 J=5 SmoothGrad on 80,000-sample clips at 16 kHz through the HIP mel front-end and
         the persistent 1D tiles, numpy and Philox noise (bar 1e-4 relative);
* c4  -- sym8 J=5 Integrated Gradients at 512x512 (native frame E2, the per-level sym8 kernels
         with the IG alpha fused into the synthesis load);
* c5  -- haar J=2 SmoothGrad (symmetric) on 128^3 volumes, numpy and Philox noise, legacy
         in-loop averaging (bar 1e-4 relative);
* a8  -- BaseWAM2D.scales (disentangle_scales on the GPU) vs the reference's own outputs.
"""
import numpy as np
import pytest
import torch

import testmodels
from tests.golden.glue_cases import BASE_CASES, make_inputs, make_model
from tests.helpers import npz

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def W():
    import wam_amd
    return wam_amd


def _top_iou(a, b, frac=0.10):
    """IoU of the top-`frac` pixels of two maps (per image, averaged)."""
    out = []
    for x, y in zip(a.reshape(a.shape[0], -1), b.reshape(b.shape[0], -1)):
        k = max(1, int(frac * x.size))
        sa, sb = set(np.argsort(-x)[:k].tolist()), set(np.argsort(-y)[:k].tolist())
        out.append(len(sa & sb) / len(sa | sb))
    return float(np.mean(out))


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(1e-30, np.abs(b).max()))


def _philox_noise(x, spread, S, item_len, shape):
    """The fused kernels' Philox values sigma_i * z for samples 0..S-1 (wam_noise_add's stream,
    which the fused noisy analyses reproduce bit for bit), as float32 [S, *shape] on the host."""
    from wam_amd import plan as P
    xd = x.reshape(x.shape[0], -1).cuda()
    n = xd.shape[0]
    sigma = P.item_sigma(xd, xd.shape[1], item_len, spread)
    z = P.noise_add(torch.zeros(n, item_len, device="cuda"), sigma, S, n, item_len, item_len, seed=42,
                    sample_base=0)
    return z.view((S,) + tuple(shape)).cpu().numpy()


# ------------------------------------------------------------------------------------------ c1
def test_c1_resnet18_elephant_statistical(W):
    """Config c1 (haar J=3 SmoothGrad n=25, random-init ResNet-18, 1 image, numpy noise) vs the
    oracle on this box's CPU. ReLU kinks make the map sensitive to fp32 rounding (a
    4e-6 input change moved it by 9.3e-3 max-abs), so the bar is statistical:
    relative L2 <= 2e-2 and max-abs <= 5e-2. lib/wam_2D.py:379-415."""
    from oracle import wam_ref
    crop = npz("elephant_224.npz")["crop"].astype(np.float32) / 255.0
    mean = np.array([0.485, 0.456, 0.406], dtype=np.float32)[:, None, None]
    std = np.array([0.229, 0.224, 0.225], dtype=np.float32)[:, None, None]
    x = torch.tensor(((crop.transpose(2, 0, 1) - mean) / std)[None])
    cpu_model = testmodels.resnet18(seed=0)
    y = int(cpu_model(x).argmax().item())
    ref = wam_ref.smooth_2d(cpu_model, x, y, wavelet="haar", J=3, mode="reflect", n_samples=25)
    ex = W.WaveletAttribution2D(testmodels.resnet18(seed=0).cuda(), wavelet="haar", J=3, method="smooth",
                                mode="reflect")
    out = ex(x, y)
    rel_l2 = np.linalg.norm(out - ref) / np.linalg.norm(ref)
    print("c1 resnet18: rel L2 %.3e, max abs %.3e" % (rel_l2, np.abs(out - ref).max()))
    assert rel_l2 <= 2e-2 and np.abs(out - ref).max() <= 5e-2


# ------------------------------------------------------------------------------------------ c3
C3_KW = dict(wavelet="db6", J=5, mode="reflect", sample_rate=16000)


def test_c3_db6_j5_80k_numpy(W):
    """Config c3's geometry: WaveletAttribution1D(db6, J=5, reflect, sample_rate=16000) on 2 clips x
    80,000 samples (the bench's clip generator), TinyAudio on the [N, 1, 157, 128] dB mel input,
    n_samples=2, numpy legacy noise, vs oracle.wam_ref.smooth_1d (lib/wam_1D.py:294-343). Runs the
    HIP mel front-end (k_mel_fwd / k_mel_adj) and the persistent tile kernels. Bar: 1e-4 of the
    max, per output (melspec gradients and every level's coefficient gradients)."""
    from oracle import wam_ref
    x = testmodels.audio_clips(2)
    y = [3, 7]
    ref_mel, ref_c = wam_ref.smooth_1d(testmodels.TinyAudio(), x, y, n_samples=2, **C3_KW)
    ex = W.WaveletAttribution1D(testmodels.TinyAudio().cuda(), n_samples=2, **C3_KW)
    mel, cs = ex(x, y)
    assert mel.shape == ref_mel.shape == (2, 157, 128)
    assert [c.shape for c in cs] == [c.shape for c in ref_c]
    assert [c.shape[1] for c in cs] == [2510, 2510, 5010, 10009, 20008, 40005]
    errs = [_rel(mel, ref_mel)] + [_rel(c, r) for c, r in zip(cs, ref_c)]
    print("c3 numpy: rel errors mel %.2e, bands %s" % (errs[0], ["%.2e" % e for e in errs[1:]]))
    assert max(errs) < 1e-4, errs


def test_c3_db6_j5_80k_philox(W):
    """The bench's c3 perf path: Philox noise fused into the 1D tile analyses (interior and
    boundary tiles), vs the oracle fed the same noise values (wam_noise_add's stream)."""
    from oracle import wam_ref
    x = testmodels.audio_clips(2)
    y = [3, 7]
    S = 2
    noise = _philox_noise(x, 0.001, S, 80000, (2, 80000))
    ref_mel, ref_c = wam_ref.smooth_1d(testmodels.TinyAudio(), x, y, n_samples=S, noise=noise, **C3_KW)
    ex = W.WaveletAttribution1D(testmodels.TinyAudio().cuda(), n_samples=S, noise="philox", **C3_KW)
    mel, cs = ex(x, y)
    errs = [_rel(mel, ref_mel)] + [_rel(c, r) for c, r in zip(cs, ref_c)]
    print("c3 philox: rel errors mel %.2e, bands %s" % (errs[0], ["%.2e" % e for e in errs[1:]]))
    assert max(errs) < 1e-4, errs


# ------------------------------------------------------------------------------------------ c5
C5_KW = dict(wavelet="haar", J=2, mode="symmetric")


def test_c5_haar_j2_128_numpy(W):
    """Config c5's geometry: WaveletAttribution3D(haar, J=2, symmetric) on 1 x 1 x 128^3 volumes
    (the bench's volume generator), TinyVoxel, n_samples=2, numpy legacy noise (channel 0,
    spread 1e-4), legacy in-loop averaging, vs oracle.wam_ref.smooth_3d (lib/wam_3D.py:550-591).
    Bar: 1e-4 of the max."""
    from oracle import wam_ref
    x = testmodels.voxel_volumes(1)
    y = [3]
    ref = wam_ref.smooth_3d(testmodels.TinyVoxel(), x, y, n_samples=2, **C5_KW)
    ex = W.WaveletAttribution3D(testmodels.TinyVoxel().cuda(), n_samples=2, **C5_KW)
    out = ex(x, y)
    assert out.shape == ref.shape == (1, 128, 128, 128) and out.dtype == np.float32
    err = _rel(out, ref)
    print("c5 numpy: rel error %.2e" % err)
    assert err < 1e-4


def test_c5_haar_j2_128_philox(W):
    """The bench's c5 perf path: Philox noise fused into the Haar block analysis (k_haar3_ana<noise>)
    vs the oracle fed the same noise values on channel 0."""
    from oracle import wam_ref
    x = testmodels.voxel_volumes(2)
    y = [3, 5]
    S = 3
    noise = _philox_noise(x, 1e-4, S, 128 ** 3, (2, 128, 128, 128))
    ref = wam_ref.smooth_3d(testmodels.TinyVoxel(), x, y, n_samples=S, noise=noise, **C5_KW)
    ex = W.WaveletAttribution3D(testmodels.TinyVoxel().cuda(), n_samples=S, noise="philox", sample_batch=2,
                                **C5_KW)
    out = ex(x, y)
    err = _rel(out, ref)
    print("c5 philox: rel error %.2e" % err)
    assert err < 1e-4


# ------------------------------------------------------------------------------------------ c4
def test_c4_ig_sym8_j5_512_native(W):
    """Config c4's estimator: IG, sym8, J=5, reflect, native frame at 512^2 (tiny kink-free model,
    3 path steps, 2 images) vs oracle.wam_ref.ig_2d; bar 1e-4 * max|ref|."""
    from oracle import wam_ref
    rs = np.random.RandomState(4)
    x = torch.tensor(rs.standard_normal((2, 3, 512, 512)).astype(np.float32))
    y = [3, 8]
    ref = wam_ref.ig_2d(testmodels.TinySmooth2D(), x, y, wavelet="sym8", J=5, mode="reflect", n_samples=3,
                        frame="native")
    ex = W.WaveletAttribution2D(testmodels.TinySmooth2D().cuda(), wavelet="sym8", J=5, mode="reflect",
                                method="integratedgrad", n_samples=3, frame="native")
    out = ex(x, y)
    assert out.shape == ref.shape == (2, 512, 512)
    err = np.abs(out - ref).max()
    print("c4 ig sym8 J5 512: max abs %.3e (max |ref| %.3e)" % (err, np.abs(ref).max()))
    assert err <= 1e-4 * max(1.0, np.abs(ref).max())


def _force_passes(monkeypatch, W, steps_per_pass):
    """Cap the samples / IG steps per WAM transform pass (engine.wam_group, as the classes call it)
    so a call runs several passes."""
    monkeypatch.setattr(W.wam_2D, "wam_group", lambda mg, total, per, budget=None: max(1, min(total, steps_per_pass)))


def test_c4_ig_sym8_j5_512_multipass(W, monkeypatch):
    """The c4 path as the bench times it: IG sym8 J=5 reflect, native frame, 512^2, with the path
    steps split into several transform passes (25 steps, 10 per pass: passes 10 / 10 / 5) so the
    trapezoid carries `prev` across passes (k_frame_trapz with k0 > 0) and each pass's synthesis
    runs its alphas in per-launch groups of 8 with a partial last group (8 + 2, 8 + 2, 5) -- vs
    oracle.wam_ref.ig_2d (lib/wam_2D.py:437-459); bar 1e-4 * max|ref|."""
    from oracle import wam_ref
    _force_passes(monkeypatch, W, 10)
    rs = np.random.RandomState(41)
    x = torch.tensor(rs.standard_normal((2, 3, 512, 512)).astype(np.float32))
    y = [3, 8]
    n = 25
    ref = wam_ref.ig_2d(testmodels.TinySmooth2D(), x, y, wavelet="sym8", J=5, mode="reflect", n_samples=n,
                        frame="native")
    ex = W.WaveletAttribution2D(testmodels.TinySmooth2D().cuda(), wavelet="sym8", J=5, mode="reflect",
                                method="integratedgrad", n_samples=n, frame="native", sample_batch=2)
    out = ex(x, y)
    assert out.shape == ref.shape == (2, 512, 512)
    err = np.abs(out - ref).max()
    print("c4 ig multipass: max abs %.3e (max |ref| %.3e)" % (err, np.abs(ref).max()))
    assert err <= 1e-4 * max(1.0, np.abs(ref).max())
    # the same call in one pass agrees to fp32 summation order
    monkeypatch.undo()
    one = W.WaveletAttribution2D(testmodels.TinySmooth2D().cuda(), wavelet="sym8", J=5, mode="reflect",
                                 method="integratedgrad", n_samples=n, frame="native", sample_batch=2)(x, y)
    assert np.abs(one - out).max() <= 1e-5 * max(1.0, np.abs(ref).max())


def test_c2_ig_db4_plane_multipass(W, monkeypatch):
    """IG on the plane-resident synthesis (db4 J=3 at 224^2, all alphas of a pass in one launch)
    over several passes (10 steps, 4 per pass) vs oracle.wam_ref.ig_2d."""
    from oracle import wam_ref
    _force_passes(monkeypatch, W, 4)
    rs = np.random.RandomState(42)
    x = torch.tensor(rs.standard_normal((2, 3, 224, 224)).astype(np.float32))
    y = [1, 4]
    ref = wam_ref.ig_2d(testmodels.TinySmooth2D(), x, y, wavelet="db4", J=3, mode="reflect", n_samples=10,
                        frame="native")
    out = W.WaveletAttribution2D(testmodels.TinySmooth2D().cuda(), wavelet="db4", J=3, mode="reflect",
                                 method="integratedgrad", n_samples=10, frame="native", sample_batch=2)(x, y)
    err = np.abs(out - ref).max()
    print("c2-geometry ig multipass: max abs %.3e (max |ref| %.3e)" % (err, np.abs(ref).max()))
    assert err <= 1e-4 * max(1.0, np.abs(ref).max())


def test_c2_philox_smooth_multipass(W, monkeypatch):
    """The c2 perf path (Philox noise fused into k_plane_ana<noise>) over several transform passes
    (7 samples, 2 per pass: sample_base 0, 2, 4, 6) vs the oracle fed noise_add's values."""
    from oracle import wam_ref
    from wam_amd import plan as P
    _force_passes(monkeypatch, W, 2)
    rs = np.random.RandomState(43)
    N, C, H, S = 2, 3, 224, 7
    x = torch.tensor(rs.standard_normal((N, C, H, H)).astype(np.float32))
    y = [5, 2]
    xd = x.cuda()
    item = C * H * H
    sigma = P.item_sigma(xd, item, item, 0.25)
    noise = P.noise_add(torch.zeros_like(xd), sigma, S, N, item, item, seed=42, sample_base=0)
    noise = noise.view(S, N, C, H, H).cpu().numpy()
    ref = wam_ref.smooth_2d(testmodels.TinySmooth2D(), x, y, wavelet="db4", J=3, n_samples=S, frame="native",
                            noise=noise)
    out = W.WaveletAttribution2D(testmodels.TinySmooth2D().cuda(), wavelet="db4", J=3, n_samples=S,
                                 noise="philox", frame="native", sample_batch=1)(x, y)
    err = np.abs(out - ref).max()
    print("c2 philox multipass: max abs %.3e" % err)
    assert err < 1e-4


def test_alpha_fused_waverec_sym8_512_j5():
    """The per-level sym8 synthesis with the IG alpha fused on the coefficient load equals the
    synthesis of the pre-scaled coefficients fp32(alpha) * c, bit for bit (c4 geometry)."""
    from wam_amd import plan as P
    p = P.get_plan(2, (512, 512), 5, "sym8", "reflect", "cuda")  # 16 taps: per-level kernels
    torch.manual_seed(12)
    B = 6
    c = torch.randn(B * p.coeff_numel, device="cuda")
    alphas = np.linspace(0, 1, 7)
    out = p.waverec(c, B, alphas=alphas)
    assert out.shape == (7, B, 512, 512)
    for i, a in enumerate(alphas):
        assert torch.equal(out[i], p.waverec(c * float(np.float32(a)), B)[0]), i


# ------------------------------------------------------------------------------------------ c2
def test_c2_resnet50_fp32_statistical(W):
    """Config c2 with an fp32 model: random-init ResNet-50, db4 J=3 reflect SmoothGrad n=25 at
    224^2 (native frame E1), numpy noise, 2 images, vs the oracle glue on the CPU. ReLU kinks make
    the map sensitive to fp32 rounding, so the bar is the statistical one of c1: relative L2 <=
    2e-2, max-abs <= 5e-2, and the top-10 % pixels agree (IoU >= 0.9)."""
    from oracle import wam_ref
    torch.set_num_threads(16)
    x = torch.tensor(np.random.RandomState(1).standard_normal((2, 3, 224, 224)).astype(np.float32))
    y = [int(v) for v in np.random.RandomState(2).randint(0, 1000, 2)]
    ref = wam_ref.smooth_2d(testmodels.resnet50(seed=0), x, y, wavelet="db4", J=3, mode="reflect", n_samples=25,
                            frame="native")
    ex = W.WaveletAttribution2D(testmodels.resnet50(seed=0).cuda(), wavelet="db4", J=3, method="smooth",
                                mode="reflect", n_samples=25, frame="native")
    out = ex(x, y)
    rel_l2 = np.linalg.norm(out - ref) / np.linalg.norm(ref)
    mx = np.abs(out - ref).max()
    iou = _top_iou(out, ref)
    print("c2 resnet50 fp32: rel L2 %.3e, max abs %.3e, top-10%% IoU %.4f" % (rel_l2, mx, iou))
    assert rel_l2 <= 2e-2 and mx <= 5e-2 and iou >= 0.9


def test_c2_philox_fused_db4_vs_oracle(W):
    """The bench's perf path (Philox noise fused into the plane-resident analysis, native frame,
    db4, several model chunks in one WAM group) vs the reference glue fed the same noise values."""
    from oracle import wam_ref
    from wam_amd import plan as P
    rs = np.random.RandomState(21)
    N, C, H = 2, 3, 224
    S = 5
    x = torch.tensor(rs.standard_normal((N, C, H, H)).astype(np.float32))
    y = [3, 7]
    xd = x.cuda()
    item = C * H * H
    sigma = P.item_sigma(xd, item, item, 0.25)
    noise = P.noise_add(torch.zeros_like(xd), sigma, S, N, item, item, seed=42, sample_base=0)
    noise = noise.view(S, N, C, H, H).cpu().numpy()
    ref = wam_ref.smooth_2d(testmodels.TinySmooth2D(), x, y, wavelet="db4", J=3, n_samples=S, frame="native",
                            noise=noise)
    ex = W.WaveletAttribution2D(testmodels.TinySmooth2D().cuda(), wavelet="db4", J=3, n_samples=S,
                                noise="philox", frame="native", sample_batch=2)
    out = ex(x, y)
    assert out.shape == ref.shape
    assert np.abs(out - ref).max() < 1e-4, np.abs(out - ref).max()


@pytest.mark.parametrize("name", list(BASE_CASES))
def test_basewam2d_scales_vs_reference_goldens(W, name):
    """Row a8: BaseWAM2D's map and its .scales side attribute (disentangle_scales as the
    k_disentangle kernel, incl. the reference's stale approximation index) vs the reference's own
    outputs (tests/golden/base_goldens.npz). cv2 is restated as half-pixel bilinear (unpinned)."""
    case = BASE_CASES[name]
    g = npz("base_goldens.npz")
    x, y = make_inputs(case)
    b = W.BaseWAM2D(make_model(case).cuda(), **case["kw"])
    out = b(x, y)
    assert out.shape == g[name].shape and np.abs(out - g[name]).max() < 1e-4
    sc = b.scales
    ref = g[name + "_scales"]
    assert sc.shape == ref.shape and sc.dtype == np.float64
    assert np.abs(sc - ref).max() < 1e-4 * max(1.0, np.abs(ref).max()), np.abs(sc - ref).max()
    # host restatement on the GPU's own gradients: tight (only the bilinear rounding differs)
    from oracle import wam_ref
    host = wam_ref.disentangle_scales_2d(b.gradient_coeffs, case["kw"]["J"], case["kw"]["approx_coeffs"])
    assert np.abs(sc - host).max() < 1e-5, np.abs(sc - host).max()
