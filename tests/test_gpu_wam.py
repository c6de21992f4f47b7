"""GPU parity of the drop-in WAM classes against the reference glue.

Two anchors:
* tests/golden/glue_goldens.npz -- outputs of the REFERENCE's own lib/wam_{1,2,3}D.py run in the
  survey container (tests/golden/make_glue_goldens.py) on kink-free tiny models, numpy noise;
* oracle/wam_ref.py run on this box's CPU on the same inputs (for cases beyond the goldens).
Tolerances: normalised 2D maps 1e-4 abs (fp32 GPU conv vs CPU conv on a smooth model; the
mosaic values are in [0, 1]); raw 1D / 3D gradients 1e-4 relative to the max.
"""
import numpy as np
import pytest
import torch

import testmodels
from tests.golden.glue_cases import CASES, make_inputs, make_model
from tests.helpers import npz

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def W():
    import wam_amd
    return wam_amd


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(1e-30, np.abs(b).max()))


@pytest.mark.parametrize("name", [k for k in CASES])
def test_glue_goldens(W, name):
    case = CASES[name]
    g = npz("glue_goldens.npz")
    x, y = make_inputs(case)
    model = make_model(case).cuda()
    kw = dict(case["kw"])
    if case["dim"] == 2:
        ex = W.WaveletAttribution2D(model, **kw)
        out = ex(x, y)
        ref = g[name]
        assert out.shape == ref.shape and out.dtype == ref.dtype
        assert np.abs(out - ref).max() < 1e-4, np.abs(out - ref).max()
        if case.get("scales"):
            sc = ex.scales
            assert sc.shape == g[name + "_scales"].shape
            assert np.abs(sc - g[name + "_scales"]).max() < 1e-4
    elif case["dim"] == 1:
        ex = W.WaveletAttribution1D(model, **kw)
        mel, cs = ex(x, y)
        assert mel.shape == g[name + "_mel"].shape
        assert _rel(mel, g[name + "_mel"]) < 1e-4
        for j, c in enumerate(cs):
            assert c.shape == g[name + "_c%d" % j].shape
            assert _rel(c, g[name + "_c%d" % j]) < 1e-4, (j, _rel(c, g[name + "_c%d" % j]))
    else:
        ex = W.WaveletAttribution3D(model, **kw)
        out = ex(x, y)
        ref = g[name]
        assert out.shape == ref.shape and out.dtype == ref.dtype
        assert _rel(out, ref) < 1e-4


@pytest.mark.parametrize("wavelet,J,mode,method,y", [
    ("db4", 3, "reflect", "smooth", [2, 5]), ("sym8", 2, "symmetric", "smooth", 4),
    ("db6", 3, "zero", "integratedgrad", [1, 2]), ("haar", 3, "reflect", "integratedgrad", 3)])
def test_native_frame_vs_oracle(W, wavelet, J, mode, method, y):
    """E1/E2 native frame (non-haar SmoothGrad at 224; IG at a non-224 size) vs the oracle."""
    from oracle import wam_ref
    rs = np.random.RandomState(7)
    size = 224 if method == "smooth" else 96
    x = torch.tensor(rs.standard_normal((2, 3, size, size)).astype(np.float32))
    m = testmodels.TinySmooth2D()
    fn = wam_ref.smooth_2d if method == "smooth" else wam_ref.ig_2d
    ref = fn(m, x, y, wavelet=wavelet, J=J, mode=mode, n_samples=3, frame="native")
    ex = W.WaveletAttribution2D(testmodels.TinySmooth2D().cuda(), wavelet=wavelet, J=J, mode=mode, method=method,
                                n_samples=3, frame="native")
    out = ex(x, y)
    assert out.shape == ref.shape
    assert np.abs(out - ref).max() < 1e-4 * max(1.0, np.abs(ref).max())


def test_legacy_errors_match_reference(W):
    """The reference crashes on non-haar SmoothGrad at 224 and on IG at sizes != 224 (A.13)."""
    x = torch.zeros(1, 3, 224, 224)
    ex = W.WaveletAttribution2D(testmodels.TinySmooth2D().cuda(), wavelet="db4", method="smooth", n_samples=1)
    with pytest.raises(ValueError):
        ex(x, 0)
    ex = W.WaveletAttribution2D(testmodels.TinySmooth2D().cuda(), wavelet="haar", method="integratedgrad",
                                n_samples=2)
    with pytest.raises(ValueError):
        ex(torch.zeros(1, 3, 128, 128), 0)


def test_basewam2d_attributes(W):
    from oracle import wam_ref
    rs = np.random.RandomState(9)
    x = torch.tensor(rs.standard_normal((2, 3, 224, 224)).astype(np.float32))
    m = testmodels.TinySmooth2D()
    c_ref, g_ref = wam_ref.single_pass_2d(m, x.clone(), [1, 2], "haar", 3, "reflect")
    canvas = wam_ref.mosaic_2d(g_ref, True, (224, 224), (224, 224))
    b = W.BaseWAM2D(testmodels.TinySmooth2D().cuda(), wavelet="haar", J=3)
    out = b(x, [1, 2])
    assert np.abs(out - canvas).max() < 1e-4
    for got, ref in zip([b.wavelet_coeffs[0]] + [t for lv in b.wavelet_coeffs[1:] for t in lv],
                        [c_ref[0]] + [t for lv in c_ref[1:] for t in lv]):
        assert got.shape == ref.shape and np.abs(got - ref).max() < 1e-5
    for got, ref in zip([b.gradient_coeffs[0]] + [t for lv in b.gradient_coeffs[1:] for t in lv],
                        [g_ref[0]] + [t for lv in g_ref[1:] for t in lv]):
        assert got.shape == ref.shape and _rel(got, ref) < 1e-4
    assert b.scales.shape == (2, 3, 224, 224)


def test_philox_noise_statistics(W):
    """Philox mode: zero-mean unit-variance noise scaled by sigma_i; deterministic per seed;
    independent of how samples are batched."""
    from wam_amd import plan as P
    x = torch.zeros(3, 1000, device="cuda")
    x[1, 0] = 4.0
    sigma = P.item_sigma(x, 1000, 1000, 0.25)
    assert torch.allclose(sigma.cpu(), torch.tensor([0.0, 1.0, 0.0]))
    xx = torch.zeros(2, 200000, device="cuda")
    xx[:, 0] = 1.0
    s = P.item_sigma(xx, 200000, 200000, 1.0)
    a = P.noise_add(xx, s, 4, 2, 200000, 200000, seed=42).view(4, 2, 200000)
    b = torch.cat([P.noise_add(xx, s, 2, 2, 200000, 200000, seed=42, sample_base=0),
                   P.noise_add(xx, s, 2, 2, 200000, 200000, seed=42, sample_base=2)]).view(4, 2, 200000)
    assert torch.equal(a, b)
    z = (a[..., 1:]).double()
    assert abs(z.mean().item()) < 5e-3 and abs(z.std().item() - 1.0) < 5e-3
    assert not torch.equal(a[0], a[1])


def test_philox_noise_distribution_1e8(W):
    """The 'philox' noise stream over 1.0e8 draws (4 samples x 5 items x 5e6 elements, the
    counters the fused kernels use): moments of N(0, 1) (mean, variance, skewness, excess
    kurtosis within ~6 standard errors), a Kolmogorov-Smirnov bound against the normal CDF
    (D_n * sqrt(n) < 1.95, p ~ 0.001), tail frequencies beyond 3 and 4 sigma, and no lag-1
    correlation between neighbouring elements, items or samples."""
    from wam_amd import plan as P
    S, I, n = 4, 5, 5_000_000
    x = torch.zeros(I, n, device="cuda")
    z = P.noise_add(x, torch.ones(I, device="cuda"), S, I, n, n, seed=0x5EED_0001).view(S, I, n)
    N = z.numel()
    assert N >= 100_000_000
    zd = z.double()
    m = zd.mean().item()
    c = zd - m
    var = (c * c).mean().item()
    skew = (c ** 3).mean().item() / var ** 1.5
    kurt = (c ** 4).mean().item() / var ** 2 - 3.0
    se = 1.0 / N ** 0.5
    print("philox 1e8: mean %.2e var-1 %.2e skew %.2e kurt %.2e" % (m, var - 1, skew, kurt))
    assert abs(m) < 6 * se and abs(var - 1) < 6 * 2 ** 0.5 * se
    assert abs(skew) < 6 * 6 ** 0.5 * se and abs(kurt) < 6 * 24 ** 0.5 * se
    del c, zd
    srt = torch.sort(z.reshape(-1))[0].double()
    cdf = torch.special.ndtr(srt)
    k = torch.arange(1, N + 1, device="cuda", dtype=torch.float64) / N
    d = torch.maximum((k - cdf).max(), (cdf - (k - 1.0 / N)).max()).item()
    print("philox 1e8: KS D*sqrt(n) = %.3f" % (d * N ** 0.5))
    assert d * N ** 0.5 < 1.95
    del srt, cdf, k
    for t, p in ((3.0, 2.6997960632601e-3), (4.0, 6.334248366623e-5)):
        f = (z.abs() > t).double().mean().item()
        assert abs(f - p) < 6 * (p * (1 - p) / N) ** 0.5, (t, f, p)
    zf = z.float()
    for a, b in ((zf[..., 1:], zf[..., :-1]), (zf[:, 1:], zf[:, :-1]), (zf[1:], zf[:-1])):
        r = (a.double() * b.double()).mean().item()
        assert abs(r) < 6 / a.numel() ** 0.5, r


def test_philox_stream_matches_host_restatement(W):
    """The GPU noise stream is Philox4x32-10 (pinned by the Random123 known answers on the host
    restatement, tests/test_host_logic.py) + Box-Muller on the hardware transcendentals: compare
    every drawn value with the float64 host restatement (|err| <= 2e-5 * (1 + |z|))."""
    from wam_amd import plan as P
    from tests.helpers import philox_normals
    n, items, samples, base, seed = 4099, 3, 2, 5, 0x1234_5678_9ABC
    x = torch.zeros(items, n, device="cuda")
    sigma = torch.ones(items, device="cuda")
    z = P.noise_add(x, sigma, samples, items, n, n, seed=seed, sample_base=base).view(samples, items, n).cpu().numpy()
    for s in range(samples):
        for i in range(items):
            ref = philox_normals(n, i, base + s, seed)
            assert np.all(np.abs(z[s, i] - ref) <= 2e-5 * (1 + np.abs(ref))), (s, i)


def test_wam3d_y_none_and_ig_native(W):
    from oracle import wam_ref
    rs = np.random.RandomState(3)
    x = torch.tensor((rs.standard_normal((2, 1, 16, 16, 16)) > 0).astype(np.float32))
    m = testmodels.TinyVoxel()
    ref = wam_ref.smooth_3d(m, x, [1, 2], wavelet="haar", J=2, n_samples=3, stdev_spread=0.05)
    ex = W.WaveletAttribution3D(testmodels.TinyVoxel().cuda(), wavelet="haar", J=2, n_samples=3,
                                stdev_spread=0.05)
    out = ex(x, [1, 2])
    assert _rel(out, ref) < 1e-4
    # IG at 32^3: legacy raises (inner refactor size 16), native runs and matches the oracle
    x32 = torch.tensor((rs.standard_normal((1, 1, 32, 32, 32)) > 0).astype(np.float32))
    ex = W.WaveletAttribution3D(testmodels.TinyVoxel().cuda(), wavelet="haar", J=2, method="integratedgrad",
                                n_samples=3)
    with pytest.raises(ValueError):
        ex(x32, 1)
    ex = W.WaveletAttribution3D(testmodels.TinyVoxel().cuda(), wavelet="haar", J=2, method="integratedgrad",
                                n_samples=3, frame="native")
    out = ex(x32, 1)
    ref = wam_ref.ig_3d(testmodels.TinyVoxel(), x32, 1, wavelet="haar", J=2, n_samples=3, inner_size=32)
    assert _rel(out, ref) < 1e-4


def test_sample_batching_invariance(W):
    """Stacking noise samples into one model batch gives the per-sample reference result."""
    rs = np.random.RandomState(11)
    x = torch.tensor(rs.standard_normal((3, 3, 224, 224)).astype(np.float32))
    outs = []
    for sb in (1, 2, 5):
        ex = W.WaveletAttribution2D(testmodels.TinySmooth2D().cuda(), wavelet="haar", n_samples=5, sample_batch=sb)
        outs.append(ex(x, [0, 1, 2]))
    assert np.abs(outs[0] - outs[1]).max() < 1e-5 and np.abs(outs[0] - outs[2]).max() < 1e-5


def test_wam_group_size_invariance(W, monkeypatch):
    """Transform launches over the whole sample range vs one model group at a time: same map."""
    import wam_amd.wam_2D as m2
    rs = np.random.RandomState(22)
    x = torch.tensor(rs.standard_normal((3, 3, 224, 224)).astype(np.float32))
    kw = dict(wavelet="db4", J=3, n_samples=7, noise="philox", frame="native", sample_batch=2)
    full = W.WaveletAttribution2D(testmodels.TinySmooth2D().cuda(), **kw)(x, [0, 1, 2])
    monkeypatch.setattr(m2, "wam_group", lambda model_group, total, per_sample, budget=None: model_group)
    small = W.WaveletAttribution2D(testmodels.TinySmooth2D().cuda(), **kw)(x, [0, 1, 2])
    assert np.abs(full - small).max() < 1e-6
