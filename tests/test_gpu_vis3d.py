"""Row f4 on the GPU: WaveletAttribution3D.visualize (k_vis3d_* kernels) vs the reference's own
outputs (tests/golden/f4_goldens.npz), filter_voxels vs its restatement on the same pass, the
point-cloud pass (evaluate_point_clouds) vs the oracle's torch-CPU ptwt restatement, and the
disabled point-cloud entry of __call__ (prints, returns None, as the reference)."""
import numpy as np
import pytest
import torch

import testmodels
from tests.helpers import npz

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def W():
    import wam_amd
    return wam_amd


@pytest.mark.parametrize("name", ["vis_s32_j2", "vis_s16_j1", "vis_s64_j3"])
def test_visualize_vs_reference_goldens(W, name):
    """scipy zoom(order=1) restated term by term in double, cast to float32: values in [0, 1]
    agree to 1 ulp-ish (<= 1e-6)."""
    from tests.golden.make_f4_goldens import VIS_CASES, cube
    n, S, J, seed = VIS_CASES[name]
    ex = W.WaveletAttribution3D(testmodels.TinyVoxel().cuda(), wavelet="haar", J=J)
    ex.grads = cube(n, S, seed)
    ex.input_size = S
    got = ex.visualize()
    ref = npz("f4_goldens.npz")[name]
    assert got.shape == ref.shape and got.dtype == np.float32
    assert np.abs(got - ref).max() <= 1e-6, np.abs(got - ref).max()


def test_visualize_after_smooth(W):
    """visualize() on the device cube a smooth call left behind == on its host copy."""
    from oracle import wam_ref
    x = torch.tensor((np.random.RandomState(9).standard_normal((2, 1, 32, 32, 32)) > 0).astype(np.float32))
    ex = W.WaveletAttribution3D(testmodels.TinyVoxel().cuda(), wavelet="haar", J=2, n_samples=3, stdev_spread=0.05)
    cube = ex(x, [1, 2])
    got = ex.visualize()
    ref = wam_ref.visualize_3d(cube, 2, 32)
    assert np.abs(got - ref).max() <= 1e-6


@pytest.mark.parametrize("wav,J", [("haar", 2), ("haar", 1)])
def test_filter_voxels_vs_restatement(W, wav, J):
    """(BaseWAM3D's cube, hence the pass filter_voxels reads, exists for Haar only: other filters
    give non-dyadic coefficient blocks the reference's refactor cannot place)"""
    from oracle import wam_ref
    x = torch.tensor((np.random.RandomState(10).standard_normal((2, 1, 16, 16, 16)) > 0).astype(np.float32))
    b = W.BaseWAM3D(testmodels.TinyVoxel().cuda(), wavelet=wav, J=J, EPS=0.3)
    b(x, [1, 2])
    got = b.filter_voxels()
    ref = wam_ref.filter_voxels_3d(b.grads, b.coeffs, 0.3, wav)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())
    with pytest.raises(AttributeError):  # the |grad| cube of a smooth call has no per-band dicts
        ex = W.WaveletAttribution3D(testmodels.TinyVoxel().cuda(), wavelet="haar", J=2, n_samples=1)
        ex(x, [1, 2])
        ex.coeffs = b.coeffs
        ex.filter_voxels()


class _TinyPoints(torch.nn.Module):
    """PointNet-shaped stand-in: [B, 3, N] -> (logits, aux, aux)."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(3)
        self.conv = torch.nn.Conv1d(3, 8, 1)
        self.fc = torch.nn.Linear(8, 5)

    def forward(self, x):
        h = torch.tanh(self.conv(x)).mean(-1)
        return self.fc(h), None, None


def test_point_clouds(W, capsys):
    from oracle import ptwt_torch as ptwt
    x = torch.tensor(np.random.RandomState(11).standard_normal((2, 64, 3)).astype(np.float32))
    b = W.BaseWAM3D(_TinyPoints().cuda(), wavelet="db2", J=2, instance="point_clouds")
    assert b(x, [1, 2]) is None and "Not implemented yet" in capsys.readouterr().out
    coeffs, same = b.evaluate_point_clouds(x, [1, 2], (0, 2, 1))
    assert coeffs is same
    # oracle: the reference's pass on torch-CPU ptwt
    cs = ptwt.wavedec(x.reshape(2, -1).double(), "db2", level=2)
    leaves = [c.requires_grad_() for c in cs]
    rec = ptwt.waverec(leaves, "db2").view(2, 64, 3)
    m = _TinyPoints().double()
    out = m(rec.permute(0, 2, 1))[0]
    torch.diag(out[:, [1, 2]]).mean().backward()
    for a, c in zip(coeffs, cs):
        assert a.shape == tuple(c.shape) and np.abs(a - c.detach().numpy()).max() < 1e-5
    for a, c in zip(b.point_grads, leaves):
        assert np.abs(a - c.grad.numpy()).max() < 1e-5 * max(1.0, float(c.grad.abs().max()))
