"""Wavelet-domain insertion, deletion and mu-fidelity on MI355X.

Drop-in for the reference's ``Eval2DWAM`` (``src/evaluators.py:553-801``) and the helpers it
calls (``src/evaluation_helpers.py:361-594``): same class, constructor arguments, methods,
return values and debug attributes (``insertion_curves``, ``deletion_curves``, ``grad_wams``).
The reference reconstructs every altered image on the CPU, mask by mask and channel by channel
(pywt.wavedec2 -> coeffs_to_array -> arr * mask -> array_to_coeffs -> waverec2), round-trips it
through uint8 / PIL, and runs the model on the result. Here, per image:

  show()-normalised planes --wam_wavedec (pywt's default mode 'symmetric')--> coefficients
  --wam_coeff_masks (all masks x 3 channels, pywt coeffs_to_array positions)--> band-major
  --wam_waverec (one launch)--> reconstructions --wam_quantize_normalize (min-max, uint8
  truncation, ToTensor, ImageNet Normalize)--> model inputs on the device

and the model evaluates several images' masks per forward. Insertion / deletion masks come from
the importance ranking (wam_rank_masks); mu-fidelity's superpixel masks are upsampled through
scipy.ndimage.zoom's order-0 cell map (wam_upsample_masks), its Gaussian-smoothed importance and
subset sums are wam_gaussian_filter2d / wam_masked_sums. Host work left: the ranking's tie order
option, Python/numpy RNG draws (the reference's own streams), the softmax on [M, classes]
logits and spearmanr on sample_size values.

Semantics kept from the reference (pinned by tests/golden/eval_goldens.npz, made with the real
PyWavelets 1.1.1): the mask is applied in pywt's coeffs_to_array layout (cH bottom-left, cV
top-right -- transposed relative to the WAM mosaic), so the mask shape must equal the
coefficient array's (a ValueError as numpy's broadcast otherwise: haar at 224 is 224 x 224);
grad_wams are computed once and cached across calls; mu-fidelity seeds numpy with the INHERITED
random_seed (42) and averages spearmanr's (rho, p-value) pair; its batch count is
int(ceil(len) / batch_size) (sic). Tie order of equal importances: numpy's argsort is not
stable and differs across numpy builds; the default ranks ties stably (``tie_order='stable'``,
GPU), ``tie_order='numpy'`` ranks on the host with np.argsort like the reference.
Transform: the default (Resize((224, 224)) -- a no-op for 224 x 224 reconstructions --, ToTensor,
Normalize(ImageNet)) runs fused on the GPU; a user ``transform`` (a callable on HWC uint8 numpy
images) is applied on the host instead.
"""
import ctypes
import math
import random

import numpy as np
import torch
from scipy.ndimage import zoom
from scipy.stats import spearmanr

from ._lib import c_f32, check, lib, ptr, stream_of
from .plan import get_plan
from .wam_2D import WaveletAttribution2D

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
_LAYOUT = {}


# ------------------------------------------------------------------------------ host geometry
def coeff_array_layout(plan):
    """pywt.coeffs_to_array positions (row-major flat index) of a plan's band-major item and the
    array shape: A at [0:ah, 0:aw]; per level (coarsest first) 'da' (= cH, ptwt 'horizontal')
    rows [ah:ah+dh] x cols [0:dw], 'ad' (cV) rows [0:dh] x cols [aw:aw+dw], 'dd' at
    [ah:, aw:]; then (ah, aw) += (dh, dw)."""
    J = plan.levels
    ah, aw = plan.band_shapes[0]
    H = ah + sum(plan.band_shapes[1 + 3 * l][0] for l in range(J))
    W = aw + sum(plan.band_shapes[1 + 3 * l][1] for l in range(J))
    parts = [(np.arange(ah)[:, None] * W + np.arange(aw)[None, :]).reshape(-1)]
    for l in range(J):
        dh, dw = plan.band_shapes[1 + 3 * l + 2]
        for b, (r0, c0) in enumerate(((ah, 0), (0, aw), (ah, aw))):
            h, w = plan.band_shapes[1 + 3 * l + b]
            parts.append(((r0 + np.arange(h))[:, None] * W + (c0 + np.arange(w))[None, :]).reshape(-1))
        ah, aw = ah + dh, aw + dw
    return np.concatenate(parts), (H, W)


def zoom_cell_map(grid, hw):
    """scipy.ndimage.zoom(masks, (1, H / grid, W / grid), order=0) as a per-pixel grid-cell
    index map (zoom of the cell-index grid: nearest neighbour copies values exactly)."""
    idx = np.arange(grid * grid, dtype=np.float64).reshape(1, grid, grid)
    return zoom(idx, (1, hw[0] / grid, hw[1] / grid), order=0)[0].astype(np.int64)


def gaussian_weights(sigma, truncate=4.0):
    """scipy's _gaussian_kernel1d(sigma, 0, int(truncate * sigma + 0.5)): w[j] for |offset| j."""
    r = int(truncate * float(sigma) + 0.5)
    x = np.arange(-r, r + 1)
    phi = np.exp(-0.5 / (sigma * sigma) * x ** 2)
    phi = phi / phi.sum()
    return phi[r:], r


def _softmax(preds):
    return np.exp(preds) / np.sum(np.exp(preds), axis=1, keepdims=True)


def compute_auc(probs):
    """src/evaluation_helpers.py:437-453."""
    return sum(probs) / (np.max(probs) * len(probs))


def generate_subsets(grid_size, subset_size, sample_size):
    """src/evaluation_helpers.py:580-594 (Python's global random, as the reference)."""
    return [[(i // grid_size, i % grid_size) for i in random.sample(range(grid_size * grid_size), subset_size)]
            for _ in range(sample_size)]


def pil_bilinear_coeffs(in_size, out_size):
    """Pillow's resample tables for BILINEAR along one axis (libImaging/Resample.c precompute_coeffs
    with box (0, in_size), then normalize_coeffs_8bpc): (ksize, bounds [out, 2] = (first source
    index, count), 22-bit fixed-point weights [out, ksize] int64, C truncation of w * 2^22 +- 0.5)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale                      # the triangle filter's support is 1
    ksize = int(math.ceil(support)) * 2 + 1
    kk = np.zeros((out_size, ksize))
    bounds = np.zeros((out_size, 2), dtype=np.int64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        ww = 0.0
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w = 1.0 - t if t < 1.0 else 0.0
            kk[xx, x] = w
            ww += w
        if ww != 0.0:
            kk[xx, :xmax] /= ww
        bounds[xx] = (xmin, xmax)
    fixed = np.trunc(np.where(kk < 0, -0.5 + kk * (1 << 22), 0.5 + kk * (1 << 22))).astype(np.int64)
    return ksize, bounds, fixed


class Eval2DWAM(WaveletAttribution2D):
    """src/evaluators.py:553-801 -- insertion / deletion (Petsiuk et al.), mu-fidelity (Bhatt et al.)."""

    def __init__(self, model, wavelet="haar", J=3, device=None, mode="reflect", transform=None, approx_coeffs=False,
                 method="smooth", n_samples=25, batch_size=128, stdev_spread=0.25, random_seed=42, *,
                 tie_order="stable", eval_batch=520, **wam_kw):
        super().__init__(model, wavelet=wavelet, J=J, device=device, mode=mode, approx_coeffs=approx_coeffs)
        self.smooted_grad_wam = WaveletAttribution2D(model, wavelet=wavelet, J=J, mode=mode,
                                                     approx_coeffs=approx_coeffs, n_samples=n_samples,
                                                     stdev_spread=stdev_spread, random_seed=random_seed,
                                                     method=method, device=device, **wam_kw)
        self.batch_size = batch_size
        self.grad_wams = None
        self.transform = transform
        if tie_order not in ("stable", "numpy"):
            raise ValueError("tie_order must be 'stable' or 'numpy'")
        self.tie_order = tie_order
        self.eval_batch = eval_batch
        self.insertion_curves = []
        self.deletion_curves = []

    # -------------------------------------------------------------------- device pipeline
    def _images(self, x):
        """show(x[i]) (src/helpers.py:421-448) on the device: [N, 3, H, W] float32, min-max
        normalised per image when outside [0, 1] (numpy: img -= min; img /= max)."""
        xd = torch.as_tensor(x).detach().to(self._dev, torch.float32).contiguous()
        out = []
        for i in range(xd.shape[0]):
            img = xd[i]
            mn, mx = img.min(), img.max()
            if bool(mx > 1) or bool(mn < 0):
                img = img - mn
                img = img / img.max()
            out.append(img)
        return out

    def _layout(self, plan):
        key = (plan, self._dev)
        if key not in _LAYOUT:
            pos, shape = coeff_array_layout(plan)
            _LAYOUT[key] = (torch.as_tensor(pos.astype(np.int32)).to(self._dev), shape)
        return _LAYOUT[key]

    def _altered_inputs(self, img, masks):
        """masks [M, AH, AW] float32 device -> model inputs [M, 3, 224, 224] (or uint8 HWC numpy
        images when a host transform is set)."""
        dev = self._dev
        C, H, W = img.shape
        plan = get_plan(2, (H, W), self.J, self.wavelet, "symmetric", dev)  # pywt.wavedec2's default mode
        pos, shape = self._layout(plan)
        if tuple(masks.shape[1:]) != tuple(shape):
            raise ValueError("operands could not be broadcast together with shapes (%d,%d) (%d,%d)"
                             % (shape + tuple(masks.shape[1:])))
        M = masks.shape[0]
        coeffs = plan.wavedec(img.contiguous())
        masked = torch.empty(M * C * plan.coeff_numel, dtype=torch.float32, device=dev)
        check(lib.wam_coeff_masks(plan.handle, C, ptr(coeffs), ptr(pos), M, shape[0] * shape[1],
                                  ptr(masks.contiguous()), ptr(masked), stream_of(dev)))
        rec = plan.waverec(masked, M * C)[0]
        rh, rw = plan.rec_shape
        if self.transform is not None:
            return self._host_transform(rec.view(M, C, rh, rw))
        mean = (c_f32 * C)(*IMAGENET_MEAN[:C])
        std = (c_f32 * C)(*IMAGENET_STD[:C])
        if (rh, rw) == (224, 224):  # Resize((224, 224)) is the identity: one fused pass
            out = torch.empty((M, C, rh, rw), dtype=torch.float32, device=dev)
            check(lib.wam_quantize_normalize(M, C, rh * rw, ptr(rec), mean, std, ptr(out), stream_of(dev)))
            return out
        return self._resize_default(rec, M, C, rh, rw, mean, std)

    def _resize_default(self, rec, M, C, rh, rw, mean, std, size=(224, 224)):
        """The default transform on a reconstruction of another size: uint8 quantisation, Pillow's
        BILINEAR resample to 224 x 224 (what torchvision's Resize does to the reference's PIL image)
        and ToTensor + Normalize, on the device (wam_quantize_resize_normalize)."""
        dev = self._dev
        oh, ow = size
        th = tv = None
        if ow != rw:
            th = pil_bilinear_coeffs(rw, ow)
        if oh != rh:
            tv = pil_bilinear_coeffs(rh, oh)
        y0, tmp_h = 0, rh
        if th is not None and tv is not None:  # the horizontal pass covers the rows the vertical one reads
            b = tv[1]
            y0, tmp_h = int(b[0, 0]), int(b[-1, 0] + b[-1, 1] - b[0, 0])
            tv = (tv[0], b - np.array([y0, 0], dtype=b.dtype), tv[2])
        dv = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.int32)).to(dev)  # noqa: E731
        bh = kh = bv = kv = None
        if th is not None:
            bh, kh = dv(th[1]), dv(th[2])
        if tv is not None:
            bv, kv = dv(tv[1]), dv(tv[2])
        scratch = torch.empty(M * C * (rh * rw + (tmp_h * ow if th is not None else 0)) + 16, dtype=torch.uint8,
                              device=dev)
        out = torch.empty((M, C, oh, ow), dtype=torch.float32, device=dev)
        p_ = lambda t: None if t is None else ptr(t)  # noqa: E731
        check(lib.wam_quantize_resize_normalize(M, C, rh, rw, ptr(rec), oh, ow, th[0] if th else 0, p_(bh), p_(kh),
                                                tv[0] if tv else 0, p_(bv), p_(kv), y0, tmp_h, mean, std,
                                                ptr(scratch), ptr(out), stream_of(dev)))
        return out

    def _host_transform(self, rec):
        """The reference's PIL images (uint8 HWC -> PIL.Image.fromarray, src/evaluation_helpers.py
        reconstruct_images), then the user's transform (src/evaluators.py:631-633)."""
        from PIL import Image
        out = []
        for r in rec.double().cpu().numpy():
            d = np.moveaxis(r, 0, 2).astype(np.float32)
            u8 = (((d - d.min()) / (d.max() - d.min()).astype(np.float32)) * 255).astype(np.uint8)
            out.append(torch.as_tensor(np.asarray(self.transform(Image.fromarray(u8)))).float())
        return torch.stack(out).to(self._dev)

    def _probs(self, inputs, label):
        """Model forward (no grad) -> the reference's host softmax -> probabilities of `label`."""
        with torch.no_grad():
            preds = self.model(inputs).float().cpu().numpy()
        return _softmax(preds)[:, label]

    def _ranks(self, wam):
        """rank[p] = position of pixel p in the descending importance order."""
        flat = torch.as_tensor(np.ascontiguousarray(wam)).reshape(-1)
        if self.tie_order == "numpy":
            order = torch.as_tensor(np.argsort(flat.numpy(), axis=None)[::-1].copy()).to(self._dev)
        else:
            order = torch.argsort(flat.to(self._dev), stable=True).flip(0)
        rank = torch.empty_like(order)
        rank[order] = torch.arange(order.numel(), device=self._dev)
        return rank.to(torch.int32)

    def _rank_masks(self, wam, n_iter, deletion):
        hw = wam.shape[-2] * wam.shape[-1]
        masks = torch.empty((n_iter + 1, wam.shape[-2], wam.shape[-1]), dtype=torch.float32, device=self._dev)
        check(lib.wam_rank_masks(n_iter, int(hw / n_iter), hw, ptr(self._ranks(wam)), int(bool(deletion)),
                                 ptr(masks), stream_of(self._dev)))
        return masks

    def _upsample(self, grid_masks, grid_size, hw):
        key = (grid_size, tuple(hw), self._dev)
        if key not in _LAYOUT:
            _LAYOUT[key] = torch.as_tensor(zoom_cell_map(grid_size, hw).astype(np.int32)).to(self._dev).reshape(-1)
        cell = _LAYOUT[key]
        g = torch.as_tensor(np.ascontiguousarray(grid_masks), dtype=torch.float32).to(self._dev)
        out = torch.empty((g.shape[0],) + tuple(hw), dtype=torch.float32, device=self._dev)
        check(lib.wam_upsample_masks(g.shape[0], grid_size * grid_size, ptr(g), hw[0] * hw[1], ptr(cell), ptr(out),
                                     stream_of(self._dev)))
        return out, cell

    def _evaluate_batched(self, images, label, batch_size):
        """evaluate() calls of the reference with its batch count int(ceil(len) / batch_size)."""
        n = images.shape[0]
        out = []
        for b in range(int(np.ceil(n) / batch_size)):
            s, e = b * batch_size, min(n, (b + 1) * batch_size)
            out.append(self._probs(images[s:e], label).astype(np.float32))
        return np.concatenate(out) if out else np.empty(0, dtype=np.float32)

    # -------------------------------------------------------------------- reference API
    def evaluate_auc(self, x, y, mode, n_iter=64):
        """src/evaluators.py:605-648: AUC of the class probability along the insertion
        (deletion) path of the WAM ranking; several images' masks per model forward."""
        if self.grad_wams is None:
            self.grad_wams = self.smooted_grad_wam(x, y)
        n_samples = self.grad_wams.shape[0]
        images = self._images(x)
        scores, predicted_probs = [], []
        per_call = max(1, self.eval_batch // (n_iter + 1))
        for s0 in range(0, n_samples, per_call):
            batch = [self._altered_inputs(images[s], self._rank_masks(self.grad_wams[s], n_iter, mode == "deletion"))
                     for s in range(s0, min(n_samples, s0 + per_call))]
            with torch.no_grad():
                preds = self.model(torch.cat(batch)).float().cpu().numpy()
            for k, s in enumerate(range(s0, s0 + len(batch))):
                p = _softmax(preds[k * (n_iter + 1):(k + 1) * (n_iter + 1)])[:, y[s]]
                scores.append(compute_auc(p))
                predicted_probs.append(p)
        return scores, predicted_probs

    def insertion(self, x, y, n_iter=64):
        scores, predicted_probs = self.evaluate_auc(x, y, "insertion", n_iter=n_iter)
        self.insertion_curves = predicted_probs
        return scores

    def deletion(self, x, y, n_iter=64):
        scores, predicted_probs = self.evaluate_auc(x, y, "deletion", n_iter=n_iter)
        self.deletion_curves = predicted_probs
        return scores

    def mu_fidelity(self, x, y, grid_size=28, sample_size=128, subset_size=157):
        """src/evaluators.py:667-767."""
        if self.grad_wams is None:
            self.grad_wams = self.smooted_grad_wam(x, y)
        np.random.seed(self.random_seed)
        xd = torch.as_tensor(x).detach().to(self._dev, torch.float32)
        with torch.no_grad():
            base = _softmax(self.model(xd).float().cpu().numpy())
        base_probs = [base[i, y[i]] for i in range(len(y))]
        images = self._images(x)
        H, W = xd.shape[2], xd.shape[3]
        w, r = gaussian_weights(2)
        dev = self._dev
        mu = []
        for i in range(len(self.grad_wams)):
            g = torch.as_tensor(np.ascontiguousarray(self.grad_wams[i]), dtype=torch.float64).to(dev)
            wam = torch.empty_like(g)
            tmp = torch.empty_like(g)
            check(lib.wam_gaussian_filter2d(1, g.shape[0], g.shape[1], w.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                            r, ptr(g), ptr(tmp), ptr(wam), stream_of(dev)))
            indices = generate_subsets(grid_size, subset_size, sample_size)
            bmask = self.compute_baseline_state(images[i], y[i], grid_size, self.batch_size, sample_size)
            masks = np.ones((sample_size, grid_size, grid_size))
            for j, index_set in enumerate(indices):
                cx, cy = zip(*index_set)
                masks[j, cx, cy] = bmask[cx, cy]
            up, cell = self._upsample(masks, grid_size, (H, W))
            altered = self._evaluate_batched(self._altered_inputs(images[i], up), y[i], self.batch_size)
            preds = base_probs[i] - altered
            sub = np.zeros((sample_size, grid_size, grid_size), dtype=np.float32)
            for j, index_set in enumerate(indices):
                cx, cy = zip(*index_set)
                sub[j, cx, cy] = 1
            subd = torch.as_tensor(sub).to(dev)
            attrs = torch.empty(sample_size, dtype=torch.float64, device=dev)
            check(lib.wam_masked_sums(sample_size, wam.numel(), ptr(wam), grid_size * grid_size, ptr(subd), ptr(cell),
                                      ptr(attrs), stream_of(dev)))
            mu.append(np.nanmean(spearmanr(preds, attrs.cpu().numpy())))
        return mu

    def compute_baseline_state(self, image, label, grid_size, batch_size, sample_size):
        """src/evaluators.py:769-801: the uniform random superpixel mask whose reconstruction
        has the lowest class probability."""
        source_masks = np.random.uniform(size=(sample_size, grid_size, grid_size))
        up, _ = self._upsample(source_masks, grid_size, tuple(image.shape[1:]))
        ys = self._evaluate_batched(self._altered_inputs(image, up), label, batch_size)
        return source_masks[int(np.argmin(ys)), :, :]
