"""Restatement of the reference's wavelet-domain evaluation (TEST INFRASTRUCTURE only).

Follows ``src/evaluation_helpers.py`` (``generate_masks`` 455-505, ``reconstruct_images`` 507-541,
``generate_images`` 560-578, ``generate_subsets`` 580-594, ``sum_importance`` 361-393,
``evaluate`` 395-431, ``normalize_data`` 433-435, ``compute_auc`` 437-453) and the ``Eval2DWAM``
methods of ``src/evaluators.py`` (``evaluate_auc`` 605-648, ``insertion`` / ``deletion``
650-665, ``mu_fidelity`` 667-767, ``compute_baseline_state`` 769-801), with:
* pywt.wavedec2 / waverec2 (default mode 'symmetric') -> ``oracle.dwt`` (float64, pinned to
  PyWavelets 1.1.1 by tests/golden/pywt_dwt.npz) and ``coeffs_to_array`` / ``array_to_coeffs``
  restated below (pywt 1.1.1 ``_multilevel.py`` layout: 'da' = cH bottom-left, 'ad' = cV
  top-right);
* PIL ``Image.fromarray`` + torchvision ``Resize((224, 224))`` (a no-op at 224: PIL returns a
  copy for an unchanged size) + ``ToTensor`` + ``Normalize`` -> the same float32 arithmetic on
  the uint8 array;
* scipy (zoom, gaussian_filter, spearmanr) and Python's ``random`` used as the reference uses them.
The model runs where its parameters live. Structure mirrors the reference's per-image loops.
"""
import random

import numpy as np
import torch
from scipy.ndimage import gaussian_filter, zoom
from scipy.stats import spearmanr

from . import dwt

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def show(img):
    """src/helpers.py:421-448 (plot=False): CHW tensor -> HWC float32, min-max normalised if
    outside [0, 1]."""
    img = np.array(img, dtype=np.float32)
    if img.shape[0] == 1:
        img = img[0]
    elif img.shape[0] == 3:
        img = np.moveaxis(img, 0, 2)
    if img.shape[-1] == 1:
        img = img[:, :, 0]
    if img.max() > 1 or img.min() < 0:
        img -= img.min()
        img /= img.max()
    return img


def generate_masks(n_iter, wam):
    flat = np.argsort(wam, axis=None)[::-1]
    rows, cols = np.unravel_index(flat, wam.shape)
    n_components = int(len(flat) / n_iter)
    ins = np.zeros((n_iter + 1,) + wam.shape)
    dele = np.ones((n_iter + 1,) + wam.shape)
    for i in range(n_iter):
        k = min((i + 1) * n_components, len(flat))
        ins[i + 1, rows[:k], cols[:k]] = 1
        dele[i + 1, rows[:k], cols[:k]] = 0
    ins[-1] = 1
    dele[-1] = 0
    return ins, dele


def coeffs_to_array(coeffs):
    """pywt.coeffs_to_array for wavedec2 output (padding 0)."""
    a = coeffs[0]
    ah, aw = a.shape
    H = ah + sum(lv[0].shape[0] for lv in coeffs[1:])
    W = aw + sum(lv[0].shape[1] for lv in coeffs[1:])
    arr = np.zeros((H, W), dtype=a.dtype)
    arr[:ah, :aw] = a
    slices = [(slice(0, ah), slice(0, aw))]
    for ch, cv, cd in coeffs[1:]:
        dh, dw = cd.shape
        s = {"da": (slice(ah, ah + ch.shape[0]), slice(0, ch.shape[1])),
             "ad": (slice(0, cv.shape[0]), slice(aw, aw + cv.shape[1])),
             "dd": (slice(ah, ah + dh), slice(aw, aw + dw))}
        arr[s["da"]], arr[s["ad"]], arr[s["dd"]] = ch, cv, cd
        slices.append(s)
        ah, aw = ah + dh, aw + dw
    return arr, slices


def array_to_coeffs(arr, slices):
    out = [arr[slices[0]]]
    for s in slices[1:]:
        out.append((arr[s["da"]], arr[s["ad"]], arr[s["dd"]]))
    return out


def normalize_data(data):
    data = data.astype(np.float32)
    return (data - np.min(data)) / (np.max(data) - np.min(data)).astype(np.float32)


def reconstruct_images(img, J, masks, wavelet="haar"):
    """-> list of uint8 HWC arrays (the reference's PIL images)."""
    out = []
    for i in range(masks.shape[0]):
        chans = []
        for j in range(3):
            coeffs = dwt.wavedec2(img[:, :, j].astype(np.float64), wavelet, J, mode="symmetric")
            arr, sl = coeffs_to_array(coeffs)
            pert = arr * masks[i, :, :]
            chans.append(dwt.waverec2(array_to_coeffs(pert, sl), wavelet))
        out.append((normalize_data(np.stack(chans, axis=2)) * 255).astype(np.uint8))
    return out


def to_input(u8, device=None):
    """Resize((224, 224)) + ToTensor + Normalize(ImageNet) of one uint8 HWC image, as torchvision does
    it to the reference's PIL image (src/evaluators.py:593-598): Resize on a PIL image is Pillow's
    Image.resize((224, 224), BILINEAR) (the identity at 224 x 224) -- run with the real Pillow."""
    if u8.shape[:2] != (224, 224):
        from PIL import Image
        u8 = np.asarray(Image.fromarray(np.ascontiguousarray(u8)).resize((224, 224), Image.BILINEAR))
    t = torch.from_numpy(np.ascontiguousarray(u8)).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    mean = torch.tensor(IMAGENET_MEAN, dtype=torch.float32)[:, None, None]
    std = torch.tensor(IMAGENET_STD, dtype=torch.float32)[:, None, None]
    t = t.sub(mean).div(std)
    return t if device is None else t.to(device)


def softmax_np(preds):
    return np.exp(preds) / np.sum(np.exp(preds), axis=1, keepdims=True)


def compute_auc(probs):
    return sum(probs) / (np.max(probs) * len(probs))


def generate_subsets(grid_size, subset_size, sample_size):
    return [[(i // grid_size, i % grid_size) for i in random.sample(range(grid_size * grid_size), subset_size)]
            for _ in range(sample_size)]


def sum_importance(wam, indices, grid_size, n_samples, batch_size=None):
    if batch_size is None:
        batch_size = n_samples
    masks = np.zeros((n_samples, grid_size, grid_size), dtype=np.uint8)
    for i, index_set in enumerate(indices):
        x, y = zip(*index_set)
        masks[i, x, y] = 1
    zf = (1, wam.shape[0] / grid_size, wam.shape[1] / grid_size)
    imp = np.empty(n_samples)
    for b in range(int(np.ceil(n_samples / batch_size))):
        s, e = b * batch_size, min(n_samples, (b + 1) * batch_size)
        imp[s:e] = np.sum(wam * zoom(masks[s:e], zf, order=0), axis=(1, 2))
    return imp


def evaluate(x, y, model, batch_size):
    device = next(model.parameters()).device
    out = np.empty(len(x), dtype=np.float32)
    with torch.no_grad():
        for b in range(int(np.ceil(len(x) / batch_size))):
            s, e = b * batch_size, min(len(x), (b + 1) * batch_size)
            preds = model(x[s:e].to(device)).cpu().numpy()
            out[s:e] = softmax_np(preds)[:, y]
    return out


# ------------------------------------------------------------------ Eval2DWAM (src/evaluators.py)
def evaluate_auc(model, grad_wams, x, y, mode, J, wavelet, n_iter=64):
    images = [show(x[i]) for i in range(x.shape[0])]
    scores, curves = [], []
    dev = next(model.parameters()).device
    for s in range(grad_wams.shape[0]):
        ins, dele = generate_masks(n_iter, grad_wams[s])
        alt = reconstruct_images(images[s], J, ins if mode == "insertion" else dele, wavelet)
        x_t = torch.stack([to_input(im) for im in alt]).to(dev)
        with torch.no_grad():
            preds = model(x_t).cpu().numpy()
        p = softmax_np(preds)[:, y[s]]
        scores.append(compute_auc(p))
        curves.append(p)
    return scores, curves


def compute_baseline_state(model, image, label, J, wavelet, grid_size, batch_size, sample_size):
    src = np.random.uniform(size=(sample_size, grid_size, grid_size))
    masks = zoom(src, (1, image.shape[0] / grid_size, image.shape[1] / grid_size), order=0)
    alt = reconstruct_images(image, J, masks, wavelet)
    ys = []
    for b in range(int(np.ceil(len(alt)) / batch_size)):  # the reference's (sic) batch count
        s, e = b * batch_size, min(len(alt), (b + 1) * batch_size)
        ys.append(evaluate(torch.stack([to_input(im) for im in alt[s:e]]), label, model, batch_size).tolist())
    ys = np.array(sum(ys, []))
    return src[np.argmin(ys), :, :]


def mu_fidelity(model, grad_wams, x, y, J, wavelet, grid_size=28, sample_size=128, subset_size=157,
                batch_size=128, random_seed=42):
    np.random.seed(random_seed)
    dev = next(model.parameters()).device
    with torch.no_grad():
        base = softmax_np(model(x.to(dev)).cpu().numpy())
    base_probs = [base[i, y[i]] for i in range(len(y))]
    images = [show(x[i]) for i in range(x.shape[0])]
    out = []
    for i in range(len(grad_wams)):
        wam = gaussian_filter(grad_wams[i], sigma=2)
        indices = generate_subsets(grid_size, subset_size, sample_size)
        bmask = compute_baseline_state(model, images[i], y[i], J, wavelet, grid_size, batch_size, sample_size)
        masks = np.ones((sample_size, grid_size, grid_size))
        for j, index_set in enumerate(indices):
            cx, cy = zip(*index_set)
            masks[j, cx, cy] = bmask[cx, cy]
        up = zoom(masks, (1, x.shape[2] / grid_size, x.shape[3] / grid_size), order=0)
        alt = reconstruct_images(images[i], J, up, wavelet)
        preds = []
        for b in range(int(np.ceil(len(alt)) / batch_size)):  # (sic)
            s, e = b * batch_size, min(len(alt), (b + 1) * batch_size)
            preds.append(evaluate(torch.stack([to_input(im) for im in alt[s:e]]), y[i], model, batch_size).tolist())
        preds = base_probs[i] - np.array(sum(preds, []))
        attrs = sum_importance(wam, indices, grid_size, sample_size, batch_size=batch_size)
        out.append(np.nanmean(spearmanr(preds, attrs)))  # mean of (rho, p-value), as the reference
    return out
