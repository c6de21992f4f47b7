"""The WAM <-> model hand-off in the explained model's own dtype and layout (bf16 NHWC), the
boundary of lib/wam_2D.py:113-116 (waverec2 -> model -> loss.backward() through waverec2).

* wam_waverec_bf16_nhwc must equal the fp32 synthesis followed by torch's cast to bf16 and its
  channels_last copy, bit for bit (same synthesis arithmetic, RNE rounding as torch);
* wam_waverec_adjoint_maps_bf16_nhwc must equal the fp32 maps pass over the widened gradient, bit for
  bit (bf16 -> fp32 is exact, the channel mean and the adjoint run in the same order);
both at the c2 bench geometry (db4 J=3 224^2, 3 channels, one model group of 13 samples x 64 images)
and on ragged shapes; end to end, WaveletAttribution2D with a bf16 channels_last folded model gives
the fp32 hand-off's maps (bf16_handoff=False) up to the model backward's own run-to-run spread.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wam():
    from wam_amd import plan
    assert torch.cuda.is_available()
    return plan


CASES = [("db4", (224, 224), 3, "reflect", 3, 13 * 64), ("haar", (224, 224), 3, "reflect", 3, 40),
         ("db3", (100, 84), 2, "zero", 3, 17), ("sym4", (36, 252), 3, "constant", 1, 9),
         ("db2", (64, 96), 4, "symmetric", 1, 33), ("db4", (37, 52), 2, "reflect", 3, 5)]


@pytest.mark.parametrize("wav,shape,J,mode,C,N", CASES)
def test_waverec_bf16_nhwc_equals_cast(wam, wav, shape, J, mode, C, N):
    p = wam.get_plan(2, shape, J, wav, mode, "cuda")
    if not p.caps & wam.CAP_BF16_NHWC:
        pytest.skip("no plane-resident synthesis / COOP maps for this geometry")
    torch.manual_seed(31)
    x = torch.randn((N * C,) + shape, device="cuda") * 3.0
    cf = p.wavedec(x)
    ref = p.waverec(cf, N * C)[0].view((N, C) + p.rec_shape)
    got = p.waverec_bf16_nhwc(cf, N * C, C)
    assert got.dtype == torch.bfloat16 and got.shape == (N, C) + p.rec_shape
    assert got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(got, ref.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
    # with the IG path scaling (alphas fused on the load)
    al = [0.0, 0.3, 1.0]
    ref = p.waverec(cf, N * C, alphas=al).view((len(al) * N, C) + p.rec_shape)
    got = p.waverec_bf16_nhwc(cf, N * C, C, alphas=al)
    assert torch.equal(got, ref.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))


def test_waverec_bf16_rounding_edges(wam):
    """RNE ties, overflow to inf, NaN -> 0x7FC0 and signed zeros through the synthesis: a Haar J=1
    plane whose only nonzero coefficient is the approximation reproduces it scaled by 1/2 exactly."""
    p = wam.get_plan(2, (2, 8), 1, "haar", "reflect", "cuda")
    if not p.caps & wam.CAP_BF16_NHWC:
        pytest.skip("no plane-resident synthesis")
    vals = torch.tensor([1.0 + 2 ** -8, 1.0 + 3 * 2 ** -8, -(1.0 + 2 ** -8), 3.4e38 * 2, float("nan"), -0.0, 2 ** -130,
                         65504.0], dtype=torch.float32)
    cf = torch.zeros(p.coeff_numel, device="cuda")
    cf[:4] = vals[:4].cuda() * 2.0   # A of a 1 x 4 approximation band: out = a / 2 per 2 x 2 block
    ref = p.waverec(cf, 1)[0].view(1, 1, 2, 8)
    got = p.waverec_bf16_nhwc(cf, 1, 1)
    assert torch.equal(got.float(), ref.to(torch.bfloat16).float())
    cf[:4] = vals[4:].cuda() * 2.0
    ref = p.waverec(cf, 1)[0].view(1, 1, 2, 8)
    got = p.waverec_bf16_nhwc(cf, 1, 1)
    a, b = got.view(torch.int16).flatten(), ref.to(torch.bfloat16).view(torch.int16).flatten()
    assert torch.equal(a, b), (a, b)


@pytest.mark.parametrize("wav,shape,J,mode,C,N", CASES)
def test_adjoint_maps_bf16_equals_fp32(wam, wav, shape, J, mode, C, N):
    p = wam.get_plan(2, shape, J, wav, mode, "cuda")
    if not p.caps & wam.CAP_BF16_NHWC:
        pytest.skip("no plane-resident synthesis / COOP maps for this geometry")
    torch.manual_seed(32)
    G = 13 if N % 13 == 0 else 1
    n = N // G
    g = (torch.randn((N, C) + p.rec_shape, device="cuda") * 1e-3).to(torch.bfloat16)
    g = g.contiguous(memory_format=torch.channels_last)
    maps, bmax, full = p.adjoint_maps(g, G, n, C)
    assert full is None
    rmaps, rbmax, _ = p.adjoint_maps(g.float().contiguous().view((N * C,) + p.rec_shape), G, n, C)
    assert torch.equal(maps, rmaps) and torch.equal(bmax, rbmax)
    # into caller-owned rows of a larger buffer (the hand-off writes each model group's rows)
    K = p.coeff_numel
    big = torch.full((2 * N * K,), -1.0, device="cuda")
    bm = torch.zeros((2 * G, p.nbands), device="cuda")
    p.adjoint_maps(g, G, n, C, maps=big[N * K:], band_max=bm[G:])
    assert torch.equal(big[N * K:], rmaps) and bool((big[:N * K] == -1.0).all())
    assert torch.equal(bm[G:], rbmax) and bool((bm[:G] == 0).all())
    # the same gradient in planar NCHW order (what a model whose first backward op is planar returns)
    m3, b3, _ = p.adjoint_maps(g.contiguous(), G, n, C)
    assert torch.equal(m3, rmaps) and torch.equal(b3, rbmax)
    with pytest.raises(ValueError):
        p.adjoint_maps(g, G, n, C, full=True)  # no per-channel coefficient gradients from bf16


def test_handoff_end_to_end_matches_fp32_handoff():
    """WaveletAttribution2D SmoothGrad with a bf16 channels_last folded model: the bf16 hand-off
    (synthesis writes the model input, maps read the model gradient, per model group) against the
    fp32 hand-off of the same call (same Philox noise, same model). The model's bf16 backward is not
    bit-reproducible from call to call on the GPU (MIOpen solvers), so the bar is its spread; the
    hand-off kernels themselves are bit-checked above."""
    import torch.nn as nn
    from wam_amd import plan as P
    from wam_amd.wam_2D import WaveletAttribution2D

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = nn.Conv2d(3, 8, 3, padding=1)
            self.bn = nn.BatchNorm2d(8)
            self.fc = nn.Linear(8 * 16, 5)

        def forward(self, x):
            h = torch.tanh(self.bn(self.conv(x)))
            return self.fc(torch.flatten(nn.functional.adaptive_avg_pool2d(h, 4), 1))

    torch.manual_seed(0)
    m = Net().eval().cuda()
    x = torch.tensor(np.random.RandomState(1).standard_normal((4, 3, 64, 64)).astype(np.float32))
    kw = dict(wavelet="db4", J=3, method="smooth", n_samples=6, noise="philox", frame="native", sample_batch=4,
              optimize_model=True, autocast_dtype=torch.bfloat16, channels_last=True)
    P.timing_drain()
    P.timing_enable(True)
    ex = WaveletAttribution2D(m, **kw)
    a = ex(x, [1, 3, 0, 2])
    torch.cuda.synchronize()
    P.timing_enable(False)
    names = {r[0] for r in P.timing_drain()}
    assert any(k.startswith("k_plane_maps<bf16") for k in names), names
    b = WaveletAttribution2D(m, bf16_handoff=False, **kw)(x, [1, 3, 0, 2])
    assert a.shape == b.shape == (4, 64, 64)
    rel = np.linalg.norm(a - b) / np.linalg.norm(b)
    assert rel <= 2e-2, rel
    # side attributes of the last pass from the bf16 gradient (widened on access)
    gc = ex.wam.gradient_coeffs
    assert len(gc) == 4 and gc[0].shape[:2] == (4, 3)
