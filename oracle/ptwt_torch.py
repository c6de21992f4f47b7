"""torch-CPU restatement of the ptwt DWT the reference runs (TEST INFRASTRUCTURE / CPU baseline).

This is the algorithm the reference executes on the host (SURVEY.md finding 10: the reference's
DWT runs on the CPU because ``noisy_x = torch.zeros(x.shape)`` is a CPU tensor,
``lib/wam_2D.py:392``): boundary extension, stride-2 ``conv{1,2,3}d`` with outer-product filters,
``conv_transpose{1,2,3}d`` with ptwt's crop/adjust rule, and autograd for the adjoint. Same
semantics as ``oracle/dwt.py`` (the float64 numpy statement), expressed as the torch ops ptwt
uses, so that timing it on the host cores is a faithful proxy of the reference's CPU path.

API mirrors the subset of ptwt 1.0.1 the reference calls: ``wavedec/waverec``,
``wavedec2/waverec2``, ``wavedec3/waverec3`` and ``constants.WaveletDetailTuple2d``. It is also
used as the stand-in ``ptwt`` module when the reference glue is imported to produce glue goldens
(``tests/golden/make_glue_goldens.py``).
"""
import itertools
import types
from collections import namedtuple

import numpy as np
import torch
import torch.nn.functional as F

from . import dwt as _np_dwt

WaveletDetailTuple2d = namedtuple("WaveletDetailTuple2d", ["horizontal", "vertical", "diagonal"])
constants = types.SimpleNamespace(WaveletDetailTuple2d=WaveletDetailTuple2d)

_KEYS3 = tuple("".join(t) for t in itertools.product("ad", repeat=3))  # aaa first


def _filters(wavelet, dtype):
    name = wavelet if isinstance(wavelet, str) else wavelet.name
    dec_lo, dec_hi, rec_lo, rec_hi = _np_dwt.filter_bank(name)
    t = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=dtype)
    # analysis correlates with the flipped dec filters (ptwt _get_filter_tensors(flip=True))
    return t(dec_lo[::-1]), t(dec_hi[::-1]), t(rec_lo), t(rec_hi)


def _pad_axis(x, axis, L, mode):
    n = x.shape[axis]
    padl, padr = _np_dwt.pad_amounts(n, L)
    src = _np_dwt.ext_index(np.arange(-padl, n + padr), n, mode)
    if mode == "zero":
        return F.pad(x.movedim(axis, -1), (padl, padr)).movedim(-1, axis)
    return torch.index_select(x, axis, torch.as_tensor(src))


def _outer(vs):
    out = vs[0]
    for v in vs[1:]:
        out = out[..., None] * v
    return out


def _bank(lo, hi, ndim):
    """Stacked outer-product filters in 'a/d' key order (first letter = axis -ndim)."""
    keys = ["".join(t) for t in itertools.product("ad", repeat=ndim)]
    filt = torch.stack([_outer([lo if c == "a" else hi for c in k]) for k in keys])
    return keys, filt.unsqueeze(1)


_CONV = {1: F.conv1d, 2: F.conv2d, 3: F.conv3d}
_CONVT = {1: F.conv_transpose1d, 2: F.conv_transpose2d, 3: F.conv_transpose3d}


def _dec(x, wavelet, level, mode, ndim):
    lead = x.shape[:-ndim]
    a = x.reshape((-1, 1) + x.shape[-ndim:])
    dlo, dhi, _, _ = _filters(wavelet, x.dtype)
    L = dlo.numel()
    keys, filt = _bank(dlo, dhi, ndim)
    out = []
    for _ in range(level):
        for ax in range(-ndim, 0):
            a = _pad_axis(a, ax, L, mode)
        res = _CONV[ndim](a, filt, stride=2)
        parts = {k: res[:, i:i + 1] for i, k in enumerate(keys)}
        a = parts.pop("a" * ndim)
        out.append(parts)
    unfold = lambda t: t.reshape(lead + t.shape[-ndim:])
    return unfold(a), [{k: unfold(v) for k, v in d.items()} for d in out[::-1]]


def _rec(a, details, wavelet, ndim):
    lead = a.shape[:-ndim]
    _, _, rlo, rhi = _filters(wavelet, a.dtype)
    L = rlo.numel()
    p = (2 * L - 3) // 2
    keys, filt = _bank(rlo, rhi, ndim)
    res = a.reshape((-1, 1) + a.shape[-ndim:])
    for c_pos, det in enumerate(details):
        parts = [res] + [det[k].reshape((-1, 1) + det[k].shape[-ndim:]) for k in keys[1:]]
        res = _CONVT[ndim](torch.cat(parts, 1), filt, stride=2)
        for i, ax in enumerate(range(-ndim, 0)):
            end = p
            if c_pos < len(details) - 1:
                nxt = next(iter(details[c_pos + 1].values())).shape[ax]
                pred = res.shape[ax] - 2 * p
                if nxt == pred - 1:
                    end += 1
                elif nxt != pred:
                    raise AssertionError("padding error, please check if dec and rec wavelets are identical.")
            if p > 0 or end > 0:
                res = res.narrow(ax, p, res.shape[ax] - p - end)
    return res.reshape(lead + res.shape[-ndim:])


def wavedec(data, wavelet, *, mode="reflect", level=None, axis=-1):
    a, det = _dec(data, wavelet, level, mode, 1)
    return [a] + [d["d"] for d in det]


def waverec(coeffs, wavelet, axis=-1):
    return _rec(coeffs[0], [{"d": d} for d in coeffs[1:]], wavelet, 1)


def wavedec2(data, wavelet, *, mode="reflect", level=None, axes=(-2, -1)):
    a, det = _dec(data, wavelet, level, mode, 2)
    return [a] + [WaveletDetailTuple2d(d["da"], d["ad"], d["dd"]) for d in det]


def waverec2(coeffs, wavelet, axes=(-2, -1)):
    det = [{"da": t[0], "ad": t[1], "dd": t[2]} for t in coeffs[1:]]
    return _rec(coeffs[0], det, wavelet, 2)


def wavedec3(data, wavelet, *, mode="reflect", level=None, axes=(-3, -2, -1)):
    a, det = _dec(data, wavelet, level, mode, 3)
    return [a] + det


def waverec3(coeffs, wavelet, axes=(-3, -2, -1)):
    return _rec(coeffs[0], list(coeffs[1:]), wavelet, 3)


def as_module():
    """A module object usable as ``sys.modules['ptwt']`` (for golden generation only)."""
    mod = types.ModuleType("ptwt")
    for name in ("wavedec", "waverec", "wavedec2", "waverec2", "wavedec3", "waverec3"):
        setattr(mod, name, globals()[name])
    mod.constants = constants
    return mod
