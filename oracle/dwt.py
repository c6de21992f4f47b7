"""numpy float64 restatement of the ptwt DWT semantics used by the reference (TEST INFRASTRUCTURE).

Reference call sites: ``lib/wam_2D.py:96`` (``ptwt.wavedec2``), ``lib/wam_2D.py:113``
(``ptwt.waverec2``), ``lib/wam_2D.py:430``; ``lib/wam_1D.py:109,117,370``;
``lib/wam_3D.py:194,206,222,620``. ptwt is an external dependency (not vendored; ptwt>=0.1.0,
de-facto 1.0.1); its rules are restated here from its published algorithm:

* analysis, per axis of length n with filter length L:
  p = (2L-3)//2 ; pad left p, pad right p + (n mod 2) (ptwt ``_get_pad``);
  boundary extension by mode (reflect / symmetric / zero / constant(=replicate) / periodic);
  lo[i] = sum_k dec_lo[L-1-k] * ext[2i+k]  (ptwt correlates with the flipped dec filter).
* synthesis, per axis: y[t] = sum_i a[i] rec_lo[t-2i] + d[i] rec_hi[t-2i] (conv_transpose,
  stride 2), crop p at both ends, plus one more at the end when the next finer coefficient is
  one shorter (ptwt ``_adjust_padding_at_reconstruction``).
* adjoint of synthesis w.r.t. its coefficients = analysis with zero padding using the filters
  reverse(rec_*) (= dec_* for orthogonal wavelets), recursing on the LL gradient.

N-d signals are processed separably; leading dims are batch. 2D subbands follow ptwt's
``WaveletDetailTuple2d(horizontal, vertical, diagonal)``: horizontal = hi along H, lo along W.
3D keys follow ptwt/pywt: letters for axes (-3,-2,-1), 'a' = lo, 'd' = hi.
"""
import itertools
import json
import os

import numpy as np

_FILTERS = None
_DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                     "wam_amd", "data", "filters.json")

MODES = ("reflect", "zero", "symmetric", "constant", "periodic")


def filter_bank(name):
    """(dec_lo, dec_hi, rec_lo, rec_hi) float64 arrays for a pywt wavelet name."""
    global _FILTERS
    if _FILTERS is None:
        with open(_DATA) as f:
            _FILTERS = json.load(f)["wavelets"]
    w = _FILTERS[name]
    return tuple(np.asarray(w[k], dtype=np.float64) for k in ("dec_lo", "dec_hi", "rec_lo", "rec_hi"))


def pad_amounts(n, L):
    p = (2 * L - 3) // 2
    return p, p + (n % 2)


def ext_index(idx, n, mode):
    """Map extended-signal positions idx (may be <0 or >=n) to source indices; -1 = zero."""
    idx = np.asarray(idx, dtype=np.int64)
    if mode == "zero":
        return np.where((idx >= 0) & (idx < n), idx, -1)
    if mode == "constant":  # ptwt maps 'constant' to torch 'replicate'
        return np.clip(idx, 0, n - 1)
    if mode == "periodic":  # torch 'circular'
        return np.mod(idx, n)
    if mode == "reflect":  # mirror without repeating the edge (torch 'reflect')
        if n == 1:
            return np.zeros_like(idx)
        per = 2 * n - 2
        r = np.mod(idx, per)
        return np.where(r >= n, per - r, r)
    if mode == "symmetric":  # mirror repeating the edge
        per = 2 * n
        r = np.mod(idx, per)
        return np.where(r >= n, per - 1 - r, r)
    raise ValueError("unknown mode %r" % (mode,))


def analysis_axis(x, lo, hi, axis, mode):
    """One analysis step along ``axis``. Returns (lo_out, hi_out)."""
    x = np.moveaxis(np.asarray(x, dtype=np.float64), axis, -1)
    n = x.shape[-1]
    L = len(lo)
    padl, padr = pad_amounts(n, L)
    src = ext_index(np.arange(-padl, n + padr), n, mode)
    xz = np.concatenate([x, np.zeros(x.shape[:-1] + (1,))], axis=-1)
    ext = xz[..., np.where(src < 0, n, src)]
    m = (n + padl + padr - L) // 2 + 1
    out_lo = np.zeros(x.shape[:-1] + (m,))
    out_hi = np.zeros(x.shape[:-1] + (m,))
    for k in range(L):
        seg = ext[..., k:k + 2 * m - 1:2]
        out_lo += lo[L - 1 - k] * seg
        out_hi += hi[L - 1 - k] * seg
    return np.moveaxis(out_lo, -1, axis), np.moveaxis(out_hi, -1, axis)


def synthesis_axis(a, d, rec_lo, rec_hi, axis, crop_end_extra=False):
    """Transposed-conv synthesis along ``axis`` followed by ptwt's crop."""
    a = np.moveaxis(np.asarray(a, dtype=np.float64), axis, -1)
    d = np.moveaxis(np.asarray(d, dtype=np.float64), axis, -1)
    m = a.shape[-1]
    L = len(rec_lo)
    y = np.zeros(a.shape[:-1] + (2 * m - 2 + L,))
    for k in range(L):
        y[..., k:k + 2 * m - 1:2] += rec_lo[k] * a + rec_hi[k] * d
    p = (2 * L - 3) // 2
    end = y.shape[-1] - p - (1 if crop_end_extra else 0)
    y = y[..., p:end] if p > 0 or crop_end_extra else y
    return np.moveaxis(y, -1, axis)


def _needs_extra(res_len, p, next_len):
    pred = res_len - 2 * p
    if next_len == pred:
        return False
    if next_len == pred - 1:
        return True
    raise AssertionError("padding error, please check if dec and rec wavelets are identical.")


def _syn_len(m, L):
    return 2 * m - 2 + L


# ---------------------------------------------------------------------------- generic n-d
def _axes(ndim):
    return tuple(range(-ndim, 0))


def dwtn_level(x, wavelet, mode, ndim):
    """One level of n-d analysis. Returns dict key->array with keys over {'a','d'}^ndim
    (first letter = axis -ndim)."""
    dec_lo, dec_hi, _, _ = filter_bank(wavelet) if isinstance(wavelet, str) else wavelet
    parts = {"": x}
    for ax in _axes(ndim):
        nxt = {}
        for key, arr in parts.items():
            lo, hi = analysis_axis(arr, dec_lo, dec_hi, ax, mode)
            nxt[key + "a"] = lo
            nxt[key + "d"] = hi
        parts = nxt
    return parts


def idwtn_level(parts, wavelet, ndim, extra=None):
    """Inverse of dwtn_level. ``extra[ax]`` = crop one more at the end of that axis."""
    _, _, rec_lo, rec_hi = filter_bank(wavelet) if isinstance(wavelet, str) else wavelet
    extra = extra or {}
    for ax in reversed(_axes(ndim)):
        nxt = {}
        for key in sorted({k[:-1] for k in parts}):
            nxt[key] = synthesis_axis(parts[key + "a"], parts[key + "d"], rec_lo, rec_hi, ax,
                                      crop_end_extra=extra.get(ax, False))
        parts = nxt
    return parts[""]


def wavedecn(x, wavelet, level, mode, ndim):
    coeffs = []
    a = np.asarray(x, dtype=np.float64)
    for _ in range(level):
        parts = dwtn_level(a, wavelet, mode, ndim)
        a = parts.pop("a" * ndim)
        coeffs.append(parts)
    return [a] + coeffs[::-1]


def waverecn(coeffs, wavelet, ndim):
    L = len(filter_bank(wavelet)[0]) if isinstance(wavelet, str) else len(wavelet[0])
    p = (2 * L - 3) // 2
    a = coeffs[0]
    details = coeffs[1:]
    for c_pos, det in enumerate(details):
        parts = dict(det)
        parts["a" * ndim] = a
        extra = {}
        if c_pos < len(details) - 1:
            nxt = next(iter(details[c_pos + 1].values()))
            for i, ax in enumerate(_axes(ndim)):
                m = a.shape[ax]
                extra[ax] = _needs_extra(_syn_len(m, L), p, nxt.shape[ax])
        a = idwtn_level(parts, wavelet, ndim, extra)
    return a


def adjointn(grad, coeff_shapes_like, wavelet, ndim):
    """VJP of waverecn w.r.t. its coefficients: zero-mode analysis with reverse(rec) filters.
    coeff_shapes_like: the number of levels, or a coefficient list of that depth."""
    _, _, rec_lo, rec_hi = filter_bank(wavelet) if isinstance(wavelet, str) else wavelet
    fb = (rec_lo[::-1], rec_hi[::-1], rec_lo, rec_hi)
    level = coeff_shapes_like if isinstance(coeff_shapes_like, int) else len(coeff_shapes_like) - 1
    out = []
    g = np.asarray(grad, dtype=np.float64)
    for _ in range(level):
        parts = dwtn_level(g, fb, "zero", ndim)
        g = parts.pop("a" * ndim)
        out.append(parts)
    return [g] + out[::-1]


# ---------------------------------------------------------------------------- ptwt-shaped API
_KEYS2 = ("da", "ad", "dd")  # horizontal, vertical, diagonal


def wavedec(x, wavelet, level, mode="reflect"):
    c = wavedecn(x, wavelet, level, mode, 1)
    return [c[0]] + [d["d"] for d in c[1:]]


def waverec(coeffs, wavelet):
    return waverecn([coeffs[0]] + [{"d": d} for d in coeffs[1:]], wavelet, 1)


def wavedec2(x, wavelet, level, mode="reflect"):
    c = wavedecn(x, wavelet, level, mode, 2)
    return [c[0]] + [tuple(d[k] for k in _KEYS2) for d in c[1:]]


def waverec2(coeffs, wavelet):
    return waverecn([coeffs[0]] + [dict(zip(_KEYS2, t)) for t in coeffs[1:]], wavelet, 2)


def adjoint2(grad, coeffs_like, wavelet):
    c = adjointn(grad, coeffs_like, wavelet, 2)
    return [c[0]] + [tuple(d[k] for k in _KEYS2) for d in c[1:]]


def adjoint1(grad, coeffs_like, wavelet):
    c = adjointn(grad, coeffs_like, wavelet, 1)
    return [c[0]] + [d["d"] for d in c[1:]]


KEYS3 = tuple("".join(t) for t in itertools.product("ad", repeat=3))[1:]


def wavedec3(x, wavelet, level, mode="reflect"):
    return wavedecn(x, wavelet, level, mode, 3)


def waverec3(coeffs, wavelet):
    return waverecn(coeffs, wavelet, 3)


def adjoint3(grad, coeffs_like, wavelet):
    return adjointn(grad, coeffs_like, wavelet, 3)


def level_sizes(n, L, level):
    """Coefficient lengths per level for one axis, finest first."""
    out = []
    for _ in range(level):
        padl, padr = pad_amounts(n, L)
        n = (n + padl + padr - L) // 2 + 1
        out.append(n)
    return out
