"""Mosaic / cube geometry as gather maps (host side, built once per plan and cached on device).

The reference writes per-subband maps into a canvas with numpy slice assignments
(``lib/wam_2D.py:233,238-261`` visualize_grad_wam; ``:291-339`` _reproject_wam;
``lib/wam_3D.py:136-163`` refactor). Later writes overwrite earlier ones, so every canvas pixel
has exactly one source (or none). Here the SAME slice assignments are executed once on index
canvases; the result is a per-pixel (source offset, band) map that the accumulate kernels gather
through. Shape errors the reference raises (its 224 frame, J >= 6, non-haar SmoothGrad, IG at
sizes other than 224) are raised by the very same numpy assignments.

Frame policies: ``legacy`` = the reference, bug-for-bug; ``native`` = a canvas
of the input's own size with indices derived from it (E1/E2: lets db4 SmoothGrad at 224 and IG
at 512 run; identical to ``legacy`` wherever legacy runs).
"""
import numpy as np
import torch

_CACHE = {}


def _band_index(plan, b):
    dims = plan.band_shapes[b]
    return plan.band_offsets[b] + np.arange(int(np.prod(dims)), dtype=np.int64).reshape(dims)


def _mosaic_2d(plan, canvas_hw, base_hw):
    """Index canvases (src, band) for visualize_grad_wam / _reproject_wam."""
    src = np.full(canvas_hw, -1, dtype=np.int64)
    band = np.full(canvas_hw, -1, dtype=np.int64)
    a = _band_index(plan, 0)
    src[:a.shape[0], :a.shape[1]] = a
    band[:a.shape[0], :a.shape[1]] = 0
    bh, bw = base_hw
    # reference loop: for i, coeff in enumerate(coeffs[1:][::-1]) -> finest level first
    for i in range(plan.levels):
        eh, sh = int(bh / 2 ** i), int(bh / 2 ** (i + 1))
        ew, sw = int(bw / 2 ** i), int(bw / 2 ** (i + 1))
        # bands of level i (0 = finest): ptwt order (H, V, D)
        b0 = 1 + (plan.levels - 1 - i) * 3
        h, v, d = (_band_index(plan, b0 + k) for k in range(3))
        for tgt_rows, tgt_cols, arr, bid in (
                (slice(sh, eh), slice(sw, ew), d, b0 + 2),
                (slice(sh, eh), slice(None, sw), v, b0 + 1),
                (slice(None, sh), slice(sw, ew), h, b0)):
            sub = arr[:(eh - sh), :(ew - sw)]
            src[tgt_rows, tgt_cols] = sub
            band[tgt_rows, tgt_cols] = np.full(sub.shape, bid)
    return src, band


def _to_dev(src, band, device):
    s = torch.as_tensor(np.ascontiguousarray(src.reshape(-1)).astype(np.int32)).to(device)
    b = torch.as_tensor(np.ascontiguousarray(band.reshape(-1)).astype(np.int32)).to(device)
    return s, b


def _bcast_error(a, b):
    return ValueError("operands could not be broadcast together with shapes %s %s %s" % (
        str(tuple(a)).replace(" ", ""), str(tuple(b)).replace(" ", ""), str(tuple(a)).replace(" ", "")))


def smooth_frame(plan, n, frame, device):
    """SmoothGrad 2D: returns ((src, band) device int32, (R_h, R_w)) for accumulating into the
    [n, H, W] float64 average (lib/wam_2D.py:388,406)."""
    H, W = plan.shape
    key = ("smooth", plan, frame)
    if key not in _CACHE:
        if frame == "legacy":
            r = 2 * plan.band_shapes[-1][1]  # img_size = 2 * finest horizontal width (:217)
            src, band = _mosaic_2d(plan, (r, r), (224, 224))
            if (r, r) != (H, W):
                # cache the geometry only: the message carries the batch size of each call
                _CACHE[key] = lambda n_, r=r: _bcast_error((n_, H, W), (n_, r, r))
            else:
                _CACHE[key] = (_to_dev(src, band, device), (r, r))
        elif frame == "native":
            src, band = _mosaic_2d(plan, (H, W), (H, W))
            _CACHE[key] = (_to_dev(src, band, device), (H, W))
        else:
            raise ValueError("frame must be 'legacy' or 'native'")
    v = _CACHE[key]
    if callable(v):
        raise v(n)
    return v


def ig_frames(plan, n, frame, device):
    """IG 2D: (baseline map on the _reproject_wam canvas, gradient map cropped like
    grad_path[:, i] = wam(...)[:, :224, :224]), both with frame (R_h, R_w)."""
    H, W = plan.shape
    key = ("ig", plan, frame)
    if key not in _CACHE:
        if frame == "legacy":
            r = 2 * plan.band_shapes[-1][1]
            gsrc, gband = _mosaic_2d(plan, (r, r), (224, 224))
            gsrc, gband = gsrc[:224, :224], gband[:224, :224]
            bsrc, bband = _mosaic_2d(plan, (224, 224), (224, 224))
            if gsrc.shape != (H, W):
                _CACHE[key] = lambda n_, gs=gsrc.shape: ValueError(
                    "could not broadcast input array from shape %s into shape %s" % (
                        str((n_,) + gs).replace(" ", ""), str((n_, H, W)).replace(" ", "")))
            else:
                _CACHE[key] = (_to_dev(bsrc, bband, device), _to_dev(gsrc, gband, device), (224, 224))
        elif frame == "native":
            gsrc, gband = _mosaic_2d(plan, (H, W), (H, W))
            _CACHE[key] = (_to_dev(gsrc, gband, device), _to_dev(gsrc, gband, device), (H, W))
        else:
            raise ValueError("frame must be 'legacy' or 'native'")
    v = _CACHE[key]
    if callable(v):
        raise v(n)
    return v


def mosaic_map(plan, canvas_hw, base_hw, device):
    """Generic access (used by BaseWAM2D.__call__ and tests)."""
    key = ("mosaic", plan, tuple(canvas_hw), tuple(base_hw))
    if key not in _CACHE:
        src, band = _mosaic_2d(plan, tuple(canvas_hw), tuple(base_hw))
        _CACHE[key] = _to_dev(src, band, device)
    return _CACHE[key]


def cube_map(plan, input_size, device):
    """BaseWAM3D.refactor (lib/wam_3D.py:127-166) as a gather map over item-major |g| maps.
    ``input_size`` is the refactor's cube size (the reference's self.input_size)."""
    key = ("cube", plan, int(input_size))
    if key not in _CACHE:
        S = int(input_size)
        J = plan.levels
        src = np.full((S, S, S), -1, dtype=np.int64)
        idx = [int(S / 2 ** j) for j in range(J + 1)][::-1]
        idx.insert(0, 0)
        for i in range(J + 1):
            s, e = idx[i], idx[i + 1]
            if s == 0:
                src[:e, :e, :e] = _band_index(plan, 0)
            else:
                b0 = 1 + (i - 1) * 7  # coeffs[i] = details of level J-i+1, ptwt key order aad..ddd
                keys = ["aad", "ada", "add", "daa", "dad", "dda", "ddd"]
                lv = {k: _band_index(plan, b0 + n) for n, k in enumerate(keys)}
                src[s:e, s:e, s:e] = lv["ddd"]
                src[:s, :s, s:e] = lv["aad"]
                src[:s, s:e, :s] = lv["ada"]
                src[:s, s:e, s:e] = lv["add"]
                src[s:e, :s, :s] = lv["daa"]
                src[s:e, :s, s:e] = lv["dad"]
                src[s:e, s:e, :s] = lv["dda"]
        _CACHE[key] = torch.as_tensor(src.reshape(-1).astype(np.int32)).to(device)
    return _CACHE[key]
