"""Row f3's oracle (oracle/evaluation_ref.py) pinned to the reference's own evaluation helpers run
with the REAL PyWavelets 1.1.1 (tests/golden/eval_goldens.npz, make_eval_goldens.py), and the
host-side geometry of the GPU path (coeffs_to_array positions, zoom cell map) checked against them."""
import random

import numpy as np
import pytest
import torch

from oracle import dwt, evaluation_ref as E
from tests.golden.make_eval_goldens import inputs
from tests.helpers import npz


@pytest.fixture(scope="module")
def G():
    return npz("eval_goldens.npz")


def test_generate_masks(G):
    _, wam, _, _ = inputs()
    ins, dele = E.generate_masks(8, wam)
    assert np.array_equal(ins.astype(np.uint8), G["ins"]) and np.array_equal(dele.astype(np.uint8), G["del"])


@pytest.mark.parametrize("wav", ["haar", "db2"])
def test_reconstruct_images(G, wav):
    """uint8 reconstructions: pywt analyses the float32 channel in float32, the oracle in float64,
    so a handful of pixels may land one level apart after the uint8 truncation."""
    img, wam, masks_db2, _ = inputs()
    masks = E.generate_masks(8, wam)[0][[0, 2, 5, 8]] if wav == "haar" else masks_db2
    got = np.stack(E.reconstruct_images(img, 3, masks, wav))
    ref = G["rec_" + wav]
    assert got.shape == ref.shape
    d = np.abs(got.astype(int) - ref.astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 1e-3, (d.max(), (d > 0).mean())


def test_auc_subsets_importances(G):
    _, wam, _, probs = inputs()
    assert np.float32(E.compute_auc(probs)) == G["auc"]
    random.seed(7)
    idx = E.generate_subsets(28, 157, 16)
    assert np.array_equal(np.array(idx), G["subsets"])
    imp = E.sum_importance(wam, idx, 28, 16, batch_size=5)
    assert np.allclose(imp, G["importances"], rtol=1e-13, atol=0)


def test_zoom_map_and_gaussian(G):
    from scipy.ndimage import gaussian_filter
    from wam_amd.evaluation import zoom_cell_map
    _, wam, _, _ = inputs()
    assert np.array_equal(zoom_cell_map(28, (224, 224)), G["zoom_map"].astype(np.int64))
    assert np.allclose(gaussian_filter(wam, sigma=2), G["gauss"], rtol=1e-14, atol=1e-15)


@pytest.mark.parametrize("wav,size,J", [("haar", 224, 3), ("db2", 224, 3), ("db4", 96, 2), ("sym4", 64, 1)])
def test_coeff_array_positions(wav, size, J):
    """The GPU path's per-coefficient positions reproduce pywt.coeffs_to_array (via the oracle)."""
    from wam_amd.evaluation import coeff_array_layout

    class P:  # band layout of a plan without a device
        pass
    x = np.random.RandomState(5).standard_normal((size, size))
    c = dwt.wavedec2(x, wav, J, mode="symmetric")
    bands = [c[0]] + [t for lv in c[1:] for t in lv]
    p = P()
    p.band_shapes = [b.shape for b in bands]
    p.levels = J
    arr, _ = E.coeffs_to_array(c)
    pos, shape = coeff_array_layout(p)
    assert shape == arr.shape
    flat = np.concatenate([b.reshape(-1) for b in bands])
    placed = np.zeros(arr.size)
    placed[pos] = flat
    assert np.array_equal(placed.reshape(shape), arr)
