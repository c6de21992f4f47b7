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


def test_quantize_constant_image_nan_pinned_to_zero(W):
    """Insertion step 0 masks every coefficient: the reconstruction is all zero and the reference's
    normalize_data computes 0 / 0 = NaN, which numpy's uint8 cast maps to 0 on x86. The fused
    k_quantize_normalize pins NaN -> 0 explicitly: the model input is (0 - mean) / std everywhere;
    a constant non-zero image behaves the same; a regular image is unaffected."""
    from wam_amd._lib import c_f32, check, lib, ptr, stream_of
    from wam_amd.evaluation import IMAGENET_MEAN, IMAGENET_STD
    C, HW = 3, 224 * 224
    rec = torch.zeros(3, C, HW, device="cuda")
    rec[1] = 0.37                                       # constant, non-zero
    rec[2] = torch.rand(C, HW, device="cuda")           # regular
    out = torch.empty_like(rec)
    mean, std = (c_f32 * C)(*IMAGENET_MEAN), (c_f32 * C)(*IMAGENET_STD)
    check(lib.wam_quantize_normalize(3, C, HW, ptr(rec), mean, std, ptr(out), stream_of(rec.device)))
    want = ((0.0 - torch.tensor(IMAGENET_MEAN)) / torch.tensor(IMAGENET_STD))[:, None].float()
    for i in (0, 1):
        assert torch.equal(out[i].cpu(), want.expand(C, HW)), i
    from oracle import evaluation_ref as E
    d = np.moveaxis(rec[2].view(C, 224, 224).cpu().numpy(), 0, 2)
    u8 = (E.normalize_data(d) * 255).astype(np.uint8)
    ref = E.to_input(u8)
    assert torch.equal(out[2].view(C, 224, 224).cpu(), ref)


@pytest.mark.parametrize("hw", [(256, 256), (230, 230), (112, 112), (300, 200), (224, 257)])
def test_default_transform_non224_matches_pillow(W, hw):
    """Eval2DWAM's default transform on a reconstruction that is not 224 x 224 (the reference's
    Resize((224, 224)) on a PIL image, src/evaluators.py:593-598): the device quantisation + Pillow
    BILINEAR resample + ToTensor / Normalize equals the real Pillow pipeline bit for bit."""
    from oracle import evaluation_ref as E
    from wam_amd._lib import c_f32
    from wam_amd.evaluation import IMAGENET_MEAN, IMAGENET_STD
    H, Wd = hw
    rs = np.random.RandomState(H + Wd)
    rec = torch.tensor(rs.standard_normal((3, 3, H, Wd)).astype(np.float32)).cuda()
    rec[1] = 0.25  # a constant reconstruction (insertion step 0): NaN -> 0 bytes
    ev = W.Eval2DWAM(testmodels.TinySmooth2D().cuda(), wavelet="haar", J=3)
    got = ev._resize_default(rec, 3, 3, H, Wd, (c_f32 * 3)(*IMAGENET_MEAN), (c_f32 * 3)(*IMAGENET_STD))
    assert got.shape == (3, 3, 224, 224)
    for i in range(3):
        d = np.moveaxis(rec[i].cpu().numpy(), 0, 2)
        with np.errstate(invalid="ignore"):
            u8 = (E.normalize_data(d) * 255).astype(np.uint8)
        assert torch.equal(got[i].cpu(), E.to_input(u8)), i


def test_insertion_non224_default_transform_vs_oracle(W):
    """haar J=3 at 256 x 256 (coefficient array 256 x 256): insertion end to end through the default
    transform's resize path vs the oracle Eval2DWAM with the real Pillow resize."""
    from oracle import evaluation_ref as E
    rs = np.random.RandomState(43)
    x = torch.tensor(rs.standard_normal((2, 3, 256, 256)).astype(np.float32))
    y = [1, 5]
    ev = W.Eval2DWAM(testmodels.TinySmooth2D().cuda(), wavelet="haar", J=3, n_samples=2, tie_order="numpy",
                     eval_batch=40)
    scores = ev.insertion(x, y, n_iter=8)
    ref_scores, ref_curves = E.evaluate_auc(testmodels.TinySmooth2D(), ev.grad_wams, x, y, "insertion", 3, "haar",
                                            n_iter=8)
    assert np.abs(np.array(scores) - np.array(ref_scores)).max() < 1e-4
    for a, b in zip(ev.insertion_curves, ref_curves):
        assert np.abs(a - b).max() < 1e-4


def test_user_transform_receives_pil_image(W):
    """A user transform gets the reference's PIL image (Image.fromarray of the uint8 HWC array)."""
    seen = []

    def tf(im):
        seen.append((type(im).__name__, im.size, im.mode))
        return torch.tensor(np.asarray(im, dtype=np.float32)).permute(2, 0, 1) / 255.0

    ev = W.Eval2DWAM(testmodels.TinySmooth2D().cuda(), wavelet="haar", J=3, transform=tf)
    x = torch.rand(1, 3, 224, 224)
    out = ev._altered_inputs(ev._images(x)[0], torch.ones(2, 224, 224, device="cuda"))
    assert out.shape == (2, 3, 224, 224) and seen and seen[0] == ("Image", (224, 224), "RGB")
