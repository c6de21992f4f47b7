"""ptwt-shaped wavelet transforms on the GPU (the operator boundary below the WAM classes).

Mirrors the subset of ptwt 1.0.1 the reference calls (``wavedec``/``waverec``,
``wavedec2``/``waverec2``, ``wavedec3``/``waverec3``; call sites lib/wam_2D.py:96,113,430,
lib/wam_1D.py:109,117,370, lib/wam_3D.py:194,206,222,620): same argument names, same leading-dim
folding, same output containers, same sizes (odd lengths reconstruct to n+1).
``waverec*`` are differentiable: their backward is the HIP adjoint kernel (zero-padded analysis
with reverse(rec) filters), which is what the reference's ``loss.backward()`` computes through
ptwt's conv_transpose. ``wavedec*`` produce constants (WAM turns them into leaves); asking for a
gradient through them raises instead of silently returning a wrong one.
Inputs must be float32 CUDA (HIP) tensors -- there is no CPU path.
"""
import numpy as np
import torch

from ._lib import require_cuda
from .constants import KEYS3, WaveletDetailTuple2d
from .filters import get_wavelet
from .plan import get_plan


def _no_grad_input(x):
    if torch.is_grad_enabled() and x.requires_grad:
        raise NotImplementedError("wam_amd.wavedec*: gradients w.r.t. the analysed signal are not implemented "
                                  "(WAM differentiates w.r.t. the coefficients only)")


def _dec(data, wavelet, level, mode, ndim):
    require_cuda(data, "data")
    _no_grad_input(data)
    shape = tuple(data.shape[-ndim:])
    lead = tuple(data.shape[:-ndim])
    batch = int(np.prod(lead)) if lead else 1
    if level is None:
        level = 1
        L = len(get_wavelet(wavelet).dec_lo)
        n = min(shape)
        while (n // 2 ** (level + 1)) >= L - 1:
            level += 1
    plan = get_plan(ndim, shape, level, wavelet, mode, data.device)
    flat = plan.wavedec(data.detach().reshape((batch,) + shape))
    return plan, plan.split(flat, batch, lead)


class _WaverecFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, plan, batch, flat):
        ctx.plan = plan
        ctx.batch = batch
        return plan.waverec(flat.detach(), batch)[0]

    @staticmethod
    def backward(ctx, g):
        return None, None, ctx.plan.adjoint(g.contiguous())


def _rec(bands, wavelet, ndim):
    a = bands[0]
    require_cuda(a, "coefficients")
    lead = tuple(a.shape[:-ndim])
    batch = int(np.prod(lead)) if lead else 1
    finest = bands[-1].shape[-ndim:]
    L = len(get_wavelet(wavelet).dec_lo)
    levels = (len(bands) - 1) // ((1 << ndim) - 1)
    shape = tuple(2 * m + 2 - L for m in finest)
    plan = get_plan(ndim, shape, levels, wavelet, "zero", a.device)
    if [tuple(b.shape[-ndim:]) for b in bands] != [tuple(s) for s in plan.band_shapes]:
        raise AssertionError("padding error, please check if dec and rec wavelets are identical.")
    flat = torch.cat([b.reshape(-1) for b in bands])
    out = _WaverecFn.apply(plan, batch, flat)
    return out.reshape(lead + plan.rec_shape)


def wavedec(data, wavelet, *, mode="reflect", level=None, axis=-1):
    if axis != -1:
        raise NotImplementedError("axis != -1")
    _, bands = _dec(data, wavelet, level, mode, 1)
    return bands


def waverec(coeffs, wavelet, axis=-1):
    if axis != -1:
        raise NotImplementedError("axis != -1")
    return _rec(list(coeffs), wavelet, 1)


def wavedec2(data, wavelet, *, mode="reflect", level=None, axes=(-2, -1)):
    if tuple(axes) != (-2, -1):
        raise NotImplementedError("axes != (-2, -1)")
    plan, b = _dec(data, wavelet, level, mode, 2)
    return [b[0]] + [WaveletDetailTuple2d(*b[1 + 3 * i:4 + 3 * i]) for i in range(plan.levels)]


def waverec2(coeffs, wavelet, axes=(-2, -1)):
    if tuple(axes) != (-2, -1):
        raise NotImplementedError("axes != (-2, -1)")
    bands = [coeffs[0]] + [t for lv in coeffs[1:] for t in lv]
    return _rec(bands, wavelet, 2)


def wavedec3(data, wavelet, *, mode="reflect", level=None, axes=(-3, -2, -1)):
    if tuple(axes) != (-3, -2, -1):
        raise NotImplementedError("axes != (-3, -2, -1)")
    plan, b = _dec(data, wavelet, level, mode, 3)
    return [b[0]] + [{k: b[1 + 7 * i + j] for j, k in enumerate(KEYS3)} for i in range(plan.levels)]


def waverec3(coeffs, wavelet, axes=(-3, -2, -1)):
    if tuple(axes) != (-3, -2, -1):
        raise NotImplementedError("axes != (-3, -2, -1)")
    bands = [coeffs[0]] + [lv[k] for lv in coeffs[1:] for k in KEYS3]
    return _rec(bands, wavelet, 3)
