"""The credited kernels at the bench's exact launch sizes (BASELINE.json configs c2, c3, c5), not
only at the small shapes of the other GPU tests: thousands of workgroups through the XCD swizzle,
several rounds of resident workgroups, the sample-fastest order of the noisy analyses, a sample base
> 0 (the second transform pass of a call) -- reference semantics lib/wam_2D.py:385-406 (noise +
wavedec2), :113-116 (waverec2 -> model -> backward), lib/wam_1D.py:305-322, lib/wam_3D.py:565-582.

Each fused noisy analysis must equal wam_noise_add (the same Philox stream, materialised) followed by
the clean analysis, bit for bit, over the WHOLE launch (compared on the device). The maps pass at
1,600 items must equal the same kernel launched per model group (scheduling cannot change a value)
and the adjoint + wam_subband_maps path to fp32 rounding of the reordered channel mean.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wam():
    from wam_amd import plan
    assert torch.cuda.is_available()
    return plan


def _timed_names(P, fn):
    P.timing_drain()
    P.timing_enable(True)
    out = fn()
    torch.cuda.synchronize()
    P.timing_enable(False)
    return out, {r[0] for r in P.timing_drain()}


@pytest.mark.parametrize("sample_base", [0, 25])
def test_c2_noisy_plane_analysis_full_launch(wam, sample_base):
    """k_plane_ana<noise> at c2: 64 images x 3 channels x 224^2, 25 samples = 4,800 planes."""
    P = wam
    p = P.get_plan(2, (224, 224), 3, "db4", "reflect", "cuda")
    torch.manual_seed(40)
    N, C, S, H = 64, 3, 25, 224
    x = torch.randn(N, C, H, H, device="cuda")
    sigma = P.item_sigma(x, C * H * H, C * H * H, 0.25)
    fused, names = _timed_names(P, lambda: p.wavedec_noisy(x, sigma, S, N, C, seed=42, sample_base=sample_base))
    assert "k_plane_ana<noise>" in names, names
    noisy = P.noise_add(x, sigma, S, N, C * H * H, C * H * H, seed=42, sample_base=sample_base)
    ref = p.wavedec(noisy.view(S * N * C, H, H))
    del noisy
    assert fused.shape == ref.shape and torch.equal(fused, ref)


def test_c2_plane_synthesis_full_launch(wam):
    """k_plane_syn at c2 (4,800 planes): one launch equals launches over planes subsets (a plane's
    reconstruction does not depend on where it is scheduled) and the bf16 NHWC output equals the
    fp32 one cast."""
    P = wam
    p = P.get_plan(2, (224, 224), 3, "db4", "reflect", "cuda")
    torch.manual_seed(41)
    B = 4800
    cf = p.wavedec(torch.randn(B, 224, 224, device="cuda"))
    whole = p.waverec(cf, B)[0]
    views = p.split(cf, B)
    for lo, hi in [(0, 1600), (1600, 3203), (3203, 4800)]:
        sub = torch.cat([v[lo:hi].reshape(-1) for v in views])
        assert torch.equal(p.waverec(sub, hi - lo)[0], whole[lo:hi])
    if p.caps & P.CAP_BF16_NHWC:
        bf = p.waverec_bf16_nhwc(cf, B, 3)
        assert torch.equal(bf, whole.view(B // 3, 3, 224, 224).to(torch.bfloat16)
                           .contiguous(memory_format=torch.channels_last))


def test_c2_maps_full_launch(wam):
    """k_plane_maps at c2: 25 samples x 64 images (1,600 items on 512 resident workgroups, a partial
    fourth round) vs the same kernel per model group (13 + 12 samples) and vs adjoint + subband maps."""
    P = wam
    p = P.get_plan(2, (224, 224), 3, "db4", "reflect", "cuda")
    torch.manual_seed(43)
    G, N, C = 25, 64, 3
    g = torch.randn((G * N * C, 224, 224), device="cuda") * 1e-3
    (maps, bmax, _), names = _timed_names(P, lambda: p.adjoint_maps(g, G, N, C))
    assert "k_plane_maps" in names, names
    K = p.coeff_numel
    m2 = torch.empty_like(maps)
    b2 = torch.zeros_like(bmax)
    for g0, gc in [(0, 13), (13, 12)]:
        p.adjoint_maps(g[g0 * N * C:(g0 + gc) * N * C], gc, N, C, maps=m2[g0 * N * K:(g0 + gc) * N * K],
                       band_max=b2[g0:g0 + gc])
    assert torch.equal(maps, m2) and torch.equal(bmax, b2)
    # the fused pass averages the channels before the (linear) adjoint; subband_maps after it
    rmaps, rbmax = P.subband_maps(p, p.adjoint(g), G, N, C)
    tol = 2e-6 * float(rbmax.max())
    assert float((maps - rmaps).abs().max()) <= tol and float((bmax - rbmax).abs().max()) <= tol


@pytest.mark.parametrize("sample_base", [0, 7])
def test_c3_noisy_dwt1_full_launch(wam, sample_base):
    """k_dwt1_ana_int<noise> at c3: 256 clips x 80,000 samples, 25 noise samples (6,400 signals)."""
    P = wam
    n, N, S = 80000, 256, 25
    p = P.get_plan(1, (n,), 5, "db6", "reflect", "cuda")
    torch.manual_seed(44)
    x = torch.randn(N, n, device="cuda")
    sigma = P.item_sigma(x, n, n, 0.001)
    fused, names = _timed_names(P, lambda: p.wavedec_noisy(x, sigma, S, N, 1, seed=42, sample_base=sample_base))
    assert any(k.startswith("k_dwt1_ana") and "noise" in k for k in names), names
    noisy = P.noise_add(x, sigma, S, N, n, n, seed=42, sample_base=sample_base)
    ref = p.wavedec(noisy.view(S * N, n))
    del noisy
    assert torch.equal(fused, ref)


def test_c5_noisy_haar3_full_launch(wam):
    """k_haar3_ana<noise> at c5: 16 volumes of 128^3, 25 noise samples (400 volumes)."""
    P = wam
    D, N, S = 128, 16, 25
    p = P.get_plan(3, (D, D, D), 2, "haar", "symmetric", "cuda")
    torch.manual_seed(45)
    vol = D ** 3
    x = torch.randn((N, 1, D, D, D), device="cuda")
    sigma = P.item_sigma(x, vol, vol, 0.25)
    fused, names = _timed_names(P, lambda: p.wavedec_noisy(x, sigma, S, N, 1, seed=42, sample_base=3))
    assert any(k.startswith("k_haar3_ana") for k in names), names
    noisy = P.noise_add(x, sigma, S, N, vol, vol, seed=42, sample_base=3)
    ref = p.wavedec(noisy.view((S * N, D, D, D)))
    del noisy
    assert torch.equal(fused, ref)
