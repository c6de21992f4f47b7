"""Row f3 on the GPU: wavelet-domain insertion / deletion / mu-fidelity (wam_amd.evaluation.Eval2DWAM)
vs the reference helpers' own outputs (tests/golden/eval_goldens.npz, real PyWavelets 1.1.1) and
the oracle restatement of Eval2DWAM (oracle/evaluation_ref.py) on the same inputs.

Tolerances: model inputs come from a uint8 quantisation of an fp32 (GPU) vs float32-analysis /
float64-synthesis (pywt) reconstruction, so a pixel may sit one grey level apart (<= 1e-3 of the
pixels); probabilities / AUCs then agree to 1e-4; mu-fidelity is a rank correlation over
sample_size values, compared to 0.05."""
import random

import numpy as np
import pytest
import torch

import testmodels
from tests.golden.make_eval_goldens import inputs
from tests.helpers import npz

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def W():
    import wam_amd
    return wam_amd


def _expected_inputs(u8):
    from oracle import evaluation_ref as E
    return torch.stack([E.to_input(im) for im in u8])


def _level_diff(got, ref):
    """fraction of input values more than rounding apart, and the max difference in grey levels"""
    std = torch.tensor([0.229, 0.224, 0.225])[:, None, None]
    lv = ((got.cpu() - ref) * std * 255).abs()
    return float((lv > 1e-3).float().mean()), float(lv.max())


@pytest.mark.parametrize("wav", ["haar", "db2"])
def test_altered_inputs_vs_reference_helpers(W, wav):
    g = npz("eval_goldens.npz")
    img, wam, masks_db2, _ = inputs()
    ev = W.Eval2DWAM(testmodels.TinySmooth2D().cuda(), wavelet=wav, J=3)
    x = torch.tensor(np.moveaxis(img, 2, 0)[None])
    if wav == "haar":
        from oracle import evaluation_ref as E
        masks = E.generate_masks(8, wam)[0][[0, 2, 5, 8]]
        # the GPU ranking masks equal the reference's (no ties in this map)
        got_masks = ev._rank_masks(wam, 8, False).cpu().numpy()
        assert np.array_equal(got_masks.astype(np.uint8), g["ins"])
        assert np.array_equal(ev._rank_masks(wam, 8, True).cpu().numpy().astype(np.uint8), g["del"])
    else:
        masks = masks_db2
    got = ev._altered_inputs(ev._images(x)[0], torch.tensor(masks, dtype=torch.float32).cuda())
    frac, mx = _level_diff(got, _expected_inputs(g["rec_" + wav]))
    assert mx <= 1.0 + 1e-3 and frac < 1e-3, (frac, mx)


def test_mask_shape_must_match_coefficient_array(W):
    """db4 at 224: pywt's coeffs_to_array is 244 x 244, a 224 x 224 WAM mask cannot multiply it
    (the reference raises numpy's broadcast ValueError)."""
    ev = W.Eval2DWAM(testmodels.TinySmooth2D().cuda(), wavelet="db4", J=3)
    x = torch.rand(1, 3, 224, 224)
    with pytest.raises(ValueError):
        ev._altered_inputs(ev._images(x)[0], torch.ones(2, 224, 224, device="cuda"))


@pytest.mark.parametrize("mode", ["insertion", "deletion"])
def test_insertion_deletion_vs_oracle(W, mode):
    """End to end on a WAM map (haar J=3, 3 images, n_iter=16): the GPU class vs the oracle's
    Eval2DWAM restatement on the same map (numpy tie order on both sides)."""
    from oracle import evaluation_ref as E
    rs = np.random.RandomState(41)
    x = torch.tensor(rs.standard_normal((3, 3, 224, 224)).astype(np.float32))
    y = [1, 5, 7]
    ev = W.Eval2DWAM(testmodels.TinySmooth2D().cuda(), wavelet="haar", J=3, n_samples=3, tie_order="numpy",
                     eval_batch=40)
    scores = getattr(ev, mode)(x, y, n_iter=16)
    curves = ev.insertion_curves if mode == "insertion" else ev.deletion_curves
    ref_scores, ref_curves = E.evaluate_auc(testmodels.TinySmooth2D(), ev.grad_wams, x, y, mode, 3, "haar", n_iter=16)
    assert len(scores) == 3 and len(curves) == 3
    assert np.abs(np.array(scores) - np.array(ref_scores)).max() < 1e-4
    for a, b in zip(curves, ref_curves):
        assert a.shape == (17,) and np.abs(a - b).max() < 1e-4


def test_mu_fidelity_vs_oracle(W):
    from oracle import evaluation_ref as E
    rs = np.random.RandomState(42)
    x = torch.tensor(rs.uniform(size=(2, 3, 224, 224)).astype(np.float32))
    y = [2, 3]
    ev = W.Eval2DWAM(testmodels.TinySmooth2D().cuda(), wavelet="haar", J=3, n_samples=2, batch_size=16)
    wams = ev.smooted_grad_wam(x, y)
    ev.grad_wams = wams
    random.seed(3)
    got = ev.mu_fidelity(x, y, grid_size=28, sample_size=16, subset_size=100)
    random.seed(3)
    ref = E.mu_fidelity(testmodels.TinySmooth2D(), wams, x, y, 3, "haar", grid_size=28, sample_size=16,
                        subset_size=100, batch_size=16)
    print("mu-fidelity gpu %s oracle %s" % (got, ref))
    assert len(got) == 2 and np.abs(np.array(got) - np.array(ref)).max() < 0.05


def test_gaussian_and_masked_sums_vs_scipy(W):
    """wam_gaussian_filter2d == scipy.ndimage.gaussian_filter(sigma=2) (same accumulation order)
    and wam_masked_sums == sum_importance (golden), through the C-ABI."""
    import ctypes
    from scipy.ndimage import gaussian_filter
    from wam_amd import evaluation as ev_mod
    from wam_amd._lib import check, lib, ptr, stream_of
    g = npz("eval_goldens.npz")
    _, wam, _, _ = inputs()
    w, r = ev_mod.gaussian_weights(2)
    src = torch.tensor(wam, device="cuda")
    out, tmp = torch.empty_like(src), torch.empty_like(src)
    check(lib.wam_gaussian_filter2d(1, 224, 224, w.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), r, ptr(src),
                                    ptr(tmp), ptr(out), stream_of(src.device)))
    ref = gaussian_filter(wam, sigma=2)
    assert np.abs(out.cpu().numpy() - ref).max() <= 1e-15 * np.abs(ref).max()
    sub = np.zeros((16, 28, 28), dtype=np.float32)
    for j, s in enumerate(g["subsets"]):
        sub[j, s[:, 0], s[:, 1]] = 1
    cell = torch.tensor(ev_mod.zoom_cell_map(28, (224, 224)).astype(np.int32), device="cuda").reshape(-1)
    sums = torch.empty(16, dtype=torch.float64, device="cuda")
    check(lib.wam_masked_sums(16, 224 * 224, ptr(src), 28 * 28, ptr(torch.tensor(sub).cuda()), ptr(cell), ptr(sums),
                              stream_of(src.device)))
    assert np.allclose(sums.cpu().numpy(), g["importances"], rtol=1e-12, atol=0)
