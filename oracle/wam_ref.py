"""Restatement of the reference WAM glue on the CPU (TEST INFRASTRUCTURE / CPU baseline).

Follows ``lib/wam_2D.py`` (``BaseWAM2D.__call__`` 79-131, ``visualize_grad_wam`` 200-264,
``_reproject_wam`` 268-341, ``smooth_gradcam`` 379-415, ``intergrated_wam`` 417-459,
``reproject_wam`` 488-536), ``lib/wam_1D.py`` (``BaseWAM1D.__call__`` 88-150, ``compute_melspec``
194-219, ``smooth_wam`` 294-343, ``integrated_wam`` 353-421) and ``lib/wam_3D.py``
(``refactor`` 127-166, ``evaluate_voxels`` 168-245, ``smooth`` 550-591, ``intergrated_wam``
614-643), with the DWT done by ``oracle.ptwt_torch`` (the ptwt algorithm on torch-CPU) and the
model run where its parameters live. Structure mirrors the reference on purpose (per-sample
loop, global numpy legacy RNG, numpy float64 mosaic) because ``bench.py`` times it as the CPU
baseline.

Frame modes (build policy): ``legacy`` reproduces the reference exactly,
including its hard-coded 224 frame and its crashes; ``native`` (extensions E1/E2) uses a canvas of
the input's own size with indices derived from it (identical to legacy whenever legacy runs).
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import ptwt_torch as ptwt
from .melspec import AmplitudeToDB, MelSpectrogram


# ---------------------------------------------------------------------------- shared pieces
def legacy_noise_stream(x, n_samples, spread, seed, item_slice=None):
    """Yields (s, noisy_x) exactly like lib/wam_2D.py:385-403 (global numpy RNG, float64 -> f32)."""
    np.random.seed(seed)
    for s in range(n_samples):
        noisy = torch.zeros(x.shape)
        for i in range(x.shape[0]):
            xi = x[i] if item_slice is None else x[i][item_slice]
            stdev = spread * (xi.max() - xi.min())
            noise = np.random.normal(0, stdev, tuple(xi.shape)).astype(np.float32)
            if item_slice is None:
                noisy[i] = xi + torch.tensor(noise)
            else:
                noisy[i][item_slice] = xi + torch.tensor(noise)
        yield s, noisy


def diag_loss(output, y):
    """``torch.diag(output[:, y]).mean()`` (lib/wam_2D.py:115)."""
    return torch.diag(output[:, y]).mean()


def _device_of(model):
    return next(model.parameters()).device


# ---------------------------------------------------------------------------- 2D
def single_pass_2d(model, x, y, wavelet, J, mode, image=True):
    """BaseWAM2D.__call__ up to the gradients. Returns (coeffs_np, grads_np)."""
    coeffs = ptwt.wavedec2(x, wavelet, level=J, mode=mode) if image else x
    leaves = [coeffs[0].requires_grad_()]
    for c in coeffs[1:]:
        leaves.append(ptwt.WaveletDetailTuple2d(c.horizontal.requires_grad_(),
                                               c.vertical.requires_grad_(),
                                               c.diagonal.requires_grad_()))
    img = ptwt.waverec2(leaves, wavelet)
    out = model(img.to(_device_of(model)))
    diag_loss(out, y).backward()
    np_c = [leaves[0].detach().cpu().numpy()] + [tuple(t.detach().cpu().numpy() for t in c) for c in leaves[1:]]
    np_g = [leaves[0].grad.cpu().numpy()] + [tuple(t.grad.cpu().numpy() for t in c) for c in leaves[1:]]
    return np_c, np_g


def mosaic_2d(coeffs, normalize, canvas_hw, base_hw):
    """visualize_grad_wam / _reproject_wam with an explicit canvas and index base.
    legacy: canvas (2*h1, 2*h1) [or (224,224) for _reproject_wam], base (224, 224)."""
    n = coeffs[0].shape[0]
    vis = np.zeros((n,) + tuple(canvas_hw))
    approx = np.abs(coeffs[0].mean(axis=1))
    if normalize:
        approx /= approx.max()
    vis[:, :approx.shape[1], :approx.shape[2]] = approx
    bh, bw = base_hw
    for i, (h, v, d) in enumerate(coeffs[1:][::-1]):
        eh, sh = int(bh / 2 ** i), int(bh / 2 ** (i + 1))
        ew, sw = int(bw / 2 ** i), int(bw / 2 ** (i + 1))
        h = np.abs(h.mean(axis=1))
        v = np.abs(v.mean(axis=1))
        d = np.abs(d.mean(axis=1))
        if normalize:
            h /= h.max()
            d /= d.max()
            v /= v.max()
        vis[:, sh:eh, sw:ew] = d[:, :(eh - sh), :(ew - sw)]
        vis[:, sh:eh, :sw] = v[:, :(eh - sh), :(ew - sw)]
        vis[:, :sh, sw:ew] = h[:, :(eh - sh), :(ew - sw)]
    return vis


def frame_geometry(frame, H, W, h1w, reproject=False):
    """(canvas_hw, base_hw) for the given frame policy."""
    if frame == "legacy":
        canvas = (224, 224) if reproject else (2 * h1w, 2 * h1w)
        return canvas, (224, 224)
    if frame == "native":
        return (H, W), (H, W)
    raise ValueError("frame must be 'legacy' or 'native'")


def smooth_2d(model, x, y, wavelet="haar", J=3, mode="reflect", n_samples=25, stdev_spread=0.25,
              random_seed=42, normalize=True, frame="legacy", keep_last=None, noise=None):
    """noise (test hook): float32 [n_samples, N, C, H, W] added instead of the legacy numpy stream
    (used to check the GPU's Philox perf mode with the same glue)."""
    H, W = x.shape[2], x.shape[3]
    avg = np.zeros((x.shape[0], H, W))
    last = None
    if noise is not None:
        stream = ((s, x + torch.from_numpy(np.ascontiguousarray(noise[s]))) for s in range(n_samples))
    else:
        stream = legacy_noise_stream(x, n_samples, stdev_spread, random_seed)
    for _, noisy in stream:
        c, g = single_pass_2d(model, noisy, y, wavelet, J, mode)
        canvas, base = frame_geometry(frame, H, W, g[-1][0].shape[-1])
        avg += mosaic_2d(g, normalize, canvas, base)
        last = (c, g)
    for k in range(avg.shape[0]):
        avg[k, :, :] /= n_samples
    if keep_last is not None:
        keep_last["coeffs"], keep_last["grads"] = last
    return avg


def ig_2d(model, x, y, wavelet="haar", J=3, mode="reflect", n_samples=25, normalize=True,
          frame="legacy"):
    H, W = x.shape[2], x.shape[3]
    coeffs = ptwt.wavedec2(x, wavelet, level=J, mode=mode)
    np_c = [coeffs[0].detach().numpy()] + [tuple(t.detach().numpy() for t in c) for c in coeffs[1:]]
    canvas, base = frame_geometry(frame, H, W, np_c[-1][0].shape[-1], reproject=True)
    baseline = mosaic_2d(np_c, True, canvas, base)
    alphas = np.linspace(0, 1, n_samples)
    crop = (224, 224) if frame == "legacy" else (H, W)
    grad_path = np.empty((x.shape[0], n_samples) + crop, dtype=np.float32)
    for i, alpha in enumerate(alphas):
        path = [coeffs[0] * alpha] + [ptwt.WaveletDetailTuple2d(c.horizontal * alpha, c.vertical * alpha,
                                                                c.diagonal * alpha) for c in coeffs[1:]]
        _, g = single_pass_2d(model, path, y, wavelet, J, mode, image=False)
        cv, bs = frame_geometry(frame, H, W, g[-1][0].shape[-1])
        grad_path[:, i, :, :] = mosaic_2d(g, normalize, cv, bs)[:, :crop[0], :crop[1]]
    integral = np.trapz(np.nan_to_num(grad_path), axis=1)
    return baseline * integral


def disentangle_scales_2d(grads, J, approx_coeffs=False):
    """BaseWAM2D.disentangle_scales (lib/wam_2D.py:133-198) on numpy coefficient gradients,
    float32 maps as in the reference (mean over C, |.|, / batch max, cv2 resize, (V + D) + H);
    the approximation row is written for the stale loop index only (:194-197)."""
    n = grads[0].shape[0]
    size = int(2 * grads[-1][0].shape[-1])
    vis = np.zeros((n, J + 1 if approx_coeffs else J, size, size))
    img_batch = None
    for i, (h, v, d) in enumerate(grads[1:][::-1]):
        h = np.abs(h.mean(axis=1))
        h /= h.max()
        d = np.abs(d.mean(axis=1))
        d /= d.max()
        v = np.abs(v.mean(axis=1))
        v /= v.max()
        for img_batch in range(n):
            vis[img_batch, i] = bilinear_resize(v[img_batch], (size, size)) + \
                bilinear_resize(d[img_batch], (size, size)) + bilinear_resize(h[img_batch], (size, size))
    if approx_coeffs:
        a = np.abs(grads[0].mean(axis=1))
        a /= a.max()
        vis[img_batch, J] = bilinear_resize(a[img_batch], (size, size))
    return vis


def bilinear_resize(a, out_hw):
    """cv2.resize(a, (w, h), INTER_LINEAR) for upsampling (half-pixel centres, edge clamp)."""
    t = torch.as_tensor(np.ascontiguousarray(a))[None, None]
    return F.interpolate(t, size=tuple(out_hw), mode="bilinear", align_corners=False)[0, 0].numpy()


def reproject_wam(avg, J, approx_coeffs=False):
    """WaveletAttribution2D.reproject_wam (lib/wam_2D.py:488-536)."""
    n, size = avg.shape[0], avg.shape[1]
    vis = np.zeros((n, J + 1 if approx_coeffs else J, size, size))
    for j in range(J):
        e, s = int(size / 2 ** j), int(size / 2 ** (j + 1))
        d = avg[:, s:e, s:e]
        v = avg[:, s:e, :s]
        h = avg[:, :s, s:e]
        for b in range(n):
            vis[b, j] = bilinear_resize(h[b], (size, size)) + bilinear_resize(v[b], (size, size)) + \
                bilinear_resize(d[b], (size, size))
    if approx_coeffs:
        e = int(size / 2 ** J)
        for b in range(n):
            vis[b, J] = bilinear_resize(avg[b, :e, :e], (size, size))
    return vis


# ---------------------------------------------------------------------------- 1D
def compute_melspec(rec, n_fft, sample_rate, n_mels):
    to_db = AmplitudeToDB()
    mel = MelSpectrogram(sample_rate=sample_rate, n_fft=n_fft, n_mels=n_mels)
    return torch.stack([to_db(mel(w)).T.squeeze(-1).unsqueeze(0) for w in rec])


def single_pass_1d(model, x, y, wavelet, J, mode, n_fft, sample_rate, n_mels, waveform=True):
    coeffs = ptwt.wavedec(x, wavelet, level=J, mode=mode) if waveform else x
    leaves = [c.requires_grad_() for c in coeffs]
    rec = ptwt.waverec(leaves, wavelet)
    mel = compute_melspec(rec, n_fft, sample_rate, n_mels)
    mel.retain_grad()
    out = model(mel.to(_device_of(model)))
    diag_loss(out, y).backward()
    return mel.grad.detach().cpu().numpy().squeeze(), [c.grad.cpu().numpy() for c in leaves]


def smooth_1d(model, x, y, wavelet="haar", J=3, mode="reflect", n_samples=25, stdev_spread=0.001,
              random_seed=42, n_fft=1024, sample_rate=44100, n_mels=128, noise=None):
    """noise (test hook): float32 [n_samples, N, W] added instead of the legacy numpy stream."""
    if isinstance(x, list):
        x = torch.tensor(np.array([wf / wf.max() for wf in x]).astype(np.float32))
    mels, grads = [], []
    if noise is not None:
        stream = ((s, x + torch.from_numpy(np.ascontiguousarray(noise[s]))) for s in range(n_samples))
    else:
        stream = legacy_noise_stream(x, n_samples, stdev_spread, random_seed)
    for _, noisy in stream:
        m, g = single_pass_1d(model, noisy, y, wavelet, J, mode, n_fft, sample_rate, n_mels)
        mels.append(m)
        grads.append(g)
    avg = [np.mean(np.array([g[j] for g in grads]), axis=0) for j in range(J + 1)]
    return np.mean(np.array(mels), axis=0), avg


def ig_1d(model, x, y, wavelet="haar", J=3, mode="reflect", n_samples=25, n_fft=1024,
          sample_rate=44100, n_mels=128):
    if isinstance(x, list):
        x = torch.tensor(np.array([wf / wf.max() for wf in x]).astype(np.float32))
    alphas = np.linspace(0, 1, n_samples)
    coeffs = ptwt.wavedec(x, wavelet, level=J, mode=mode)
    base_z = [c.detach().numpy() for c in coeffs]
    base_mel = compute_melspec(x, n_fft, sample_rate, n_mels).squeeze(1).detach().numpy()
    path_mel = np.empty((base_mel.shape[0], n_samples, base_mel.shape[1], base_mel.shape[2]))
    path_grads = []
    for i, a in enumerate(alphas):
        m, g = single_pass_1d(model, [a * c for c in coeffs], y, wavelet, J, mode, n_fft, sample_rate,
                              n_mels, waveform=False)
        path_mel[:, i] = m
        path_grads.append(g)
    int_mel = np.trapz(path_mel, axis=1)
    int_c = [np.trapz(np.array([pg[l] for pg in path_grads]), axis=0) for l in range(J + 1)]
    return base_mel * int_mel, [b * i for b, i in zip(base_z, int_c)]


# ---------------------------------------------------------------------------- 3D
def refactor_3d(coeffs_list, J, input_size):
    """BaseWAM3D.refactor (lib/wam_3D.py:127-166): |coeff| packed into the dyadic cube."""
    out = np.empty((len(coeffs_list), input_size, input_size, input_size), dtype=np.float32)
    idx = [int(input_size / 2 ** j) for j in range(J + 1)][::-1]
    idx.insert(0, 0)
    for k, c in enumerate(coeffs_list):
        for i in range(J + 1):
            s, e = idx[i], idx[i + 1]
            if s == 0:
                out[k, :e, :e, :e] = np.abs(c[i])
            else:
                lv = c[i]
                out[k, s:e, s:e, s:e] = np.abs(lv["ddd"])
                out[k, :s, :s, s:e] = np.abs(lv["aad"])
                out[k, :s, s:e, :s] = np.abs(lv["ada"])
                out[k, :s, s:e, s:e] = np.abs(lv["add"])
                out[k, s:e, :s, :s] = np.abs(lv["daa"])
                out[k, s:e, :s, s:e] = np.abs(lv["dad"])
                out[k, s:e, s:e, :s] = np.abs(lv["dda"])
    return out


def _np3(c, grads):
    f = (lambda t: t.grad.detach().squeeze().cpu().numpy()) if grads else \
        (lambda t: t.detach().squeeze().cpu().numpy())
    return [f(c[0])] + [{k: f(v) for k, v in d.items()} for d in c[1:]]


def single_pass_3d(model, x, y, wavelet, J, mode, input_size, shape=True):
    grads, recs = [], []
    items = [ptwt.wavedec3(x[i], wavelet, level=J, mode=mode) for i in range(x.shape[0])] if shape else x
    for coeffs in items:
        leaves = [coeffs[0].requires_grad_()] + [{k: v.requires_grad_() for k, v in d.items()} for d in coeffs[1:]]
        grads.append(leaves)
        recs.append(ptwt.waverec3(leaves, wavelet))
    xg = torch.stack(recs).to(_device_of(model))
    if y is None:
        model(xg.unsqueeze(0)).mean().backward()
    else:
        diag_loss(model(xg), y).backward()
    return refactor_3d([_np3(g, True) for g in grads], J, input_size)


def smooth_3d(model, x, y=None, wavelet="haar", J=3, mode="symmetric", n_samples=25,
              stdev_spread=0.0001, random_seed=42, noise=None):
    """noise (test hook): float32 [n_samples, N, D, H, W] added to channel 0 instead of the legacy
    numpy stream (lib/wam_3D.py:567-579 noises channel 0 only; other channels stay zero)."""
    S = x.shape[-1]
    avg = np.zeros((x.shape[0], S, S, S), dtype=np.float32)
    if noise is not None:
        def _stream():
            for s in range(n_samples):
                noisy = torch.zeros(x.shape)
                noisy[:, 0] = x[:, 0] + torch.from_numpy(np.ascontiguousarray(noise[s]))
                yield s, noisy
        stream = _stream()
    else:
        stream = legacy_noise_stream(x, n_samples, stdev_spread, random_seed, item_slice=0)
    for _, noisy in stream:
        avg += single_pass_3d(model, noisy, y, wavelet, J, mode, S)
        for k in range(avg.shape[0]):
            avg[k, :, :] /= n_samples  # legacy: inside the sample loop (lib/wam_3D.py:585-587)
    return avg


def ig_3d(model, x, y=None, wavelet="haar", J=3, mode="symmetric", n_samples=25, inner_size=None):
    """lib/wam_3D.py:614-643. ``inner_size`` = the size the inner refactor uses (legacy: 16)."""
    S = x.shape[-1]
    coeffs = [ptwt.wavedec3(x[i], wavelet, level=J, mode=mode) for i in range(x.shape[0])]
    base = refactor_3d([_np3(c, False) for c in coeffs], J, S)
    alphas = np.linspace(0, 1, n_samples)
    gp = np.empty((base.shape[0], n_samples, S, S, S), dtype=np.float32)
    for i, a in enumerate(alphas):
        path = [[c[0] * a] + [{k: v * a for k, v in d.items()} for d in c[1:]] for c in coeffs]
        gp[:, i] = single_pass_3d(model, path, y, wavelet, J, mode, inner_size or 16, shape=False)
    return base * np.trapz(np.nan_to_num(gp), axis=1)


def visualize_3d(grads, J, input_size):
    """WaveletAttribution3D.visualize (lib/wam_3D.py:662-719), incl. its orientation sum
    (add + ada + add + daa + dad + dda) and the batch-wide max of the level sum."""
    from scipy.ndimage import zoom
    idx = [int(input_size / 2 ** j) for j in range(J + 1)][::-1]
    idx.insert(0, 0)
    vis = np.empty((grads.shape[0], J + 2) + grads.shape[1:], dtype=np.float32)
    for i in range(grads.shape[0]):
        for j in range(J + 1):
            s, e = idx[j], idx[j + 1]
            g = grads[i]
            if s == 0:
                c = g[:e, :e, :e]
            else:
                ada, add = g[:s, s:e, :s], g[:s, s:e, s:e]
                daa, dad, dda = g[s:e, :s, :s], g[s:e, :s, s:e], g[s:e, s:e, :s]
                c = add + ada + add + daa + dad + dda
            up = zoom(c, int(input_size / c.shape[-1]), order=1)
            vis[i, j] = up / up.max()
    allv = np.sum(vis[:, :J + 1], axis=1)
    vis[:, -1] = allv / allv.max()
    return vis


def filter_voxels_3d(grads, coeffs, EPS, wavelet):
    """BaseWAM3D.filter_voxels (lib/wam_3D.py:439-495): approximation x min-max-normalised
    gradient, details x (|g| / max(g) >= EPS), waverec3 per volume (float64 oracle)."""
    from . import dwt
    out = []
    for grad, coeff in zip(grads, coeffs):
        ag = (grad[0] - np.min(grad[0])) / (np.max(grad[0] - np.min(grad[0])))
        rec = [coeff[0] * ag]
        for dg_l, dc_l in zip(grad[1:], coeff[1:]):
            rec.append({k: dc_l[k] * ((np.abs(dg_l[k]) / dg_l[k].max()) >= EPS) for k in dg_l})
        out.append(dwt.waverec3([rec[0].astype(np.float64)] + [{k: v.astype(np.float64) for k, v in d.items()}
                                                                 for d in rec[1:]], wavelet))
    return np.array(out)
