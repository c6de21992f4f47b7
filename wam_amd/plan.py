"""Python side of the C-ABI: plans (cached per device) and thin typed wrappers of every entry
point of include/wam_hip.h. torch allocates every device buffer; every call is asynchronous on
torch's current stream of the tensor's device."""
import collections
import ctypes
import threading

import numpy as np
import torch

from . import filters
from ._lib import c_f32, c_i64, c_vp, check, lib, ptr, require_cuda, stream_of

_CACHE = {}
_LOCK = threading.Lock()
PLAN_GENERIC = 1

class Plan:
    """Immutable transform plan (ndim, spatial shape, levels, wavelet, mode) on one device."""

    def __init__(self, ndim, shape, levels, wavelet, mode, device, flags=0):
        self.ndim = int(ndim)
        self.shape = tuple(int(s) for s in shape)
        self.levels = int(levels)
        self.wavelet = filters.get_wavelet(wavelet)
        self.mode = mode
        self.device = torch.device(device)
        self.flags = flags
        L = len(self.wavelet.dec_lo)
        arr = lambda v: (ctypes.c_double * L)(*v)
        shp = (ctypes.c_int64 * self.ndim)(*self.shape)
        handle = c_vp()
        with torch.cuda.device(self.device):
            check(lib.wam_plan_create_ex(ctypes.byref(handle), self.ndim, shp, self.levels, arr(self.wavelet.dec_lo),
                                         arr(self.wavelet.dec_hi), arr(self.wavelet.rec_lo),
                                         arr(self.wavelet.rec_hi), L, filters.mode_id(mode), flags))
        self._h = handle
        self.L = L
        self.nbands = lib.wam_plan_num_bands(handle)
        dims = (ctypes.c_int64 * self.ndim)()
        self.band_shapes = []
        for b in range(self.nbands):
            check(lib.wam_plan_band_shape(handle, b, dims))
            self.band_shapes.append(tuple(dims[:]))
        self.band_offsets = [lib.wam_plan_band_offset(handle, b) for b in range(self.nbands + 1)]
        self.coeff_numel = lib.wam_plan_coeff_numel(handle)
        check(lib.wam_plan_rec_shape(handle, dims))
        self.rec_shape = tuple(dims[:])
        self._ws = {}

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and lib is not None:
            lib.wam_plan_destroy(h)
            self._h = None

    # ---------------------------------------------------------------- layout helpers
    @property
    def handle(self):
        return self._h

    def workspace(self, batch):
        n = int(lib.wam_plan_workspace_bytes(self._h, batch))
        ws = self._ws.get("buf")
        if ws is None or ws.numel() < n:
            ws = torch.empty(n, dtype=torch.uint8, device=self.device)
            self._ws["buf"] = ws
        return ws

    def split(self, flat, batch, lead=None):
        """Band views of a band-major coefficient buffer; each band reshaped to lead + band dims."""
        lead = (batch,) if lead is None else tuple(lead)
        out = []
        for b in range(self.nbands):
            n = int(np.prod(self.band_shapes[b]))
            o = batch * self.band_offsets[b]
            out.append(flat[o:o + batch * n].view(lead + self.band_shapes[b]))
        return out

    def band_level(self, b):
        """(level index 0 = finest, sub index) of band b; approximation -> (levels-1, -1)."""
        if b == 0:
            return self.levels - 1, -1
        per = (1 << self.ndim) - 1
        return self.levels - 1 - (b - 1) // per, (b - 1) % per

    # ---------------------------------------------------------------- transforms
    def wavedec(self, x, out=None):
        """x: [batch, *shape] fp32 cuda -> band-major flat coefficients [batch * coeff_numel]."""
        require_cuda(x, "x")
        x = x.contiguous()
        batch = x.numel() // int(np.prod(self.shape))
        if tuple(x.shape[-self.ndim:]) != self.shape:
            raise ValueError("input spatial shape %s does not match the plan %s" % (tuple(x.shape), self.shape))
        if out is None:
            out = torch.empty(batch * self.coeff_numel, dtype=torch.float32, device=x.device)
        ws = self.workspace(batch)
        check(lib.wam_wavedec(self._h, batch, ptr(x), ptr(out), ptr(ws), stream_of(x.device)))
        return out

    def waverec(self, flat, batch, alphas=None, out=None):
        """flat band-major coefficients -> [n_alpha, batch, *rec_shape] (n_alpha = 1 without alphas)."""
        require_cuda(flat, "coefficients")
        n_alpha = 1 if alphas is None else len(alphas)
        a = None if alphas is None else (c_f32 * n_alpha)(*[float(np.float32(v)) for v in alphas])
        if out is None:
            out = torch.empty((n_alpha, batch) + self.rec_shape, dtype=torch.float32, device=flat.device)
        ws = self.workspace(batch)
        check(lib.wam_waverec(self._h, batch, ptr(flat.contiguous()), a, n_alpha, ptr(out), ptr(ws),
                              stream_of(flat.device)))
        return out

    def waverec_bf16_nhwc(self, flat, batch, channels, alphas=None, out=None):
        """flat band-major coefficients of `batch` planes (images x channels) -> the reconstruction as
        bf16 images [n_alpha * batch / channels, channels, *rec_shape] in channels_last memory (the
        explained model's input dtype and layout; RNE rounding, as torch's cast). WAM_CAP_BF16_NHWC."""
        require_cuda(flat, "coefficients")
        n_alpha = 1 if alphas is None else len(alphas)
        a = None if alphas is None else (c_f32 * n_alpha)(*[float(np.float32(v)) for v in alphas])
        if out is None:
            out = torch.empty((n_alpha * batch // channels, channels) + self.rec_shape, dtype=torch.bfloat16,
                              device=flat.device, memory_format=torch.channels_last)
        check(lib.wam_waverec_bf16_nhwc(self._h, batch, ptr(flat.contiguous()), a, n_alpha, channels, ptr(out),
                                        stream_of(flat.device)))
        return out

    def adjoint(self, grad, out=None):
        """grad [batch, *rec_shape] -> band-major coefficient gradients (waverec's VJP)."""
        require_cuda(grad, "grad")
        grad = grad.contiguous()
        batch = grad.numel() // int(np.prod(self.rec_shape))
        if out is None:
            out = torch.empty(batch * self.coeff_numel, dtype=torch.float32, device=grad.device)
        ws = self.workspace(batch)
        check(lib.wam_waverec_adjoint(self._h, batch, ptr(grad), ptr(out), ptr(ws), stream_of(grad.device)))
        return out

    # ---------------------------------------------------------------- fused WAM passes
    @property
    def caps(self):
        return lib.wam_plan_caps(self._h)

    def wavedec_noisy(self, x, sigma, n_samples, images, channels, seed, sample_base=0, out=None, image_base=0):
        """coefficients of x + sigma_i N(0,1) (Philox) for n_samples x images x channels planes;
        image_base = global index of x's first image (Philox counter of a batch-sharded rank)."""
        require_cuda(x, "x")
        x = x.contiguous()
        batch = n_samples * images * channels
        if out is None:
            out = torch.empty(batch * self.coeff_numel, dtype=torch.float32, device=x.device)
        ws = self.workspace(batch)
        check(lib.wam_wavedec_noisy_ex(self._h, n_samples, images, channels, ptr(x), ptr(sigma),
                                       ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), sample_base, image_base, ptr(out),
                                       ptr(ws), stream_of(x.device)))
        return out

    def adjoint_maps(self, grad, groups, group_items, channels, full=False, maps=None, band_max=None):
        """waverec VJP fused with the channel-mean |.| epilogue -> (maps, band_max[, coeff grads]).
        grad: fp32 [images * channels, *rec_shape], or a bf16 channels_last [images, channels,
        *rec_shape] tensor (the model's own gradient; WAM_CAP_BF16_NHWC, full=False). maps / band_max:
        optional outputs (band_max zero-filled by the caller)."""
        if grad.dtype == torch.bfloat16:
            require_cuda(grad[:0].float(), "grad")  # the device check only
        else:
            require_cuda(grad, "grad")
        images = groups * group_items
        dev = grad.device
        maps = torch.empty(images * self.coeff_numel, dtype=torch.float32, device=dev) if maps is None else maps
        bmax = torch.zeros((groups, self.nbands), dtype=torch.float32, device=dev) if band_max is None else band_max
        if grad.dtype == torch.bfloat16:
            if full or grad.dim() != 4:
                raise ValueError("bf16 input gradients: an [images, channels, H, W] tensor, full=False")
            nhwc = grad.is_contiguous(memory_format=torch.channels_last)
            if not (nhwc or grad.is_contiguous()):
                grad = grad.contiguous(memory_format=torch.channels_last)
                nhwc = True
            check(lib.wam_waverec_adjoint_maps_bf16(self._h, groups, group_items, channels, int(nhwc), ptr(grad),
                                                    ptr(maps), ptr(bmax), stream_of(dev)))
            return maps, bmax, None
        grad = grad.contiguous()
        cg = torch.empty(images * channels * self.coeff_numel, dtype=torch.float32, device=dev) if full else None
        ws = self.workspace(images * channels)
        check(lib.wam_waverec_adjoint_maps(self._h, groups, group_items, channels, ptr(grad), ptr(maps), ptr(bmax),
                                           ptr(cg), ptr(ws), stream_of(dev)))
        return maps, bmax, cg


def get_plan(ndim, shape, levels, wavelet, mode, device, generic=False, flags=None):
    w = filters.get_wavelet(wavelet)
    device = torch.device(device)
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    fl = (PLAN_GENERIC if generic else 0) if flags is None else int(flags)
    key = (ndim, tuple(int(s) for s in shape), int(levels), w, mode, device, fl)
    with _LOCK:
        p = _CACHE.get(key)
        if p is None:
            p = Plan(ndim, shape, levels, w, mode, device, fl)
            _CACHE[key] = p
    return p


PLAN_NO_ROWS = 2
PLAN_NO_PLANE = 4
PLAN_NO_COOP = 8
PLAN_FORCE_COOP = 16
CAP_NOISY_WAVEDEC = 1
CAP_ADJOINT_MAPS = 2
CAP_BF16_NHWC = 4


def timing_enable(on=True):
    lib.wam_timing_enable(1 if on else 0)


def timing_drain():
    """[(kernel name, ms, algorithmic bytes)] for every launch since the last drain."""
    out = []
    cap = 4096
    while True:
        names = ctypes.create_string_buffer(64 * cap)
        ms = (c_f32 * cap)()
        nb = (ctypes.c_double * cap)()
        n = lib.wam_timing_drain(cap, names, ms, nb)
        for i in range(n):
            out.append((names.raw[64 * i:64 * (i + 1)].split(b"\0", 1)[0].decode(), ms[i], nb[i]))
        if n < cap:
            return out


# -------------------------------------------------------------------- WAM epilogue wrappers
# (device, stream, items, len) -> zero-initialised workspace of the split sigma reduction (its
# arrival counters are reset by every call, so one buffer serves the calls of that shape issued in
# order on one stream; calls on another stream get their own); least recently used entries go first
_SIGMA_WS = collections.OrderedDict()
_SIGMA_WS_MAX = 16


def item_sigma(x, item_stride, length, spread):
    """sigma_i = fp32(spread) * (max - min) of item i (lib/wam_2D.py:396-399, lib/wam_1D.py:311-314,
    lib/wam_3D.py:567-569), as a full-chip split reduction."""
    items = x.numel() // item_stride
    sigma = torch.empty(items, dtype=torch.float32, device=x.device)
    if items == 0:
        return sigma
    st = stream_of(x.device)
    key = (str(x.device), int(st.value or 0), int(items), int(length))
    ws = _SIGMA_WS.get(key)
    if ws is None:
        nb = int(lib.wam_item_sigma_ws_bytes(items, length))
        ws = _SIGMA_WS[key] = torch.zeros((nb + 7) // 8, dtype=torch.float64, device=x.device)
        while len(_SIGMA_WS) > _SIGMA_WS_MAX:
            _SIGMA_WS.popitem(last=False)
    _SIGMA_WS.move_to_end(key)
    check(lib.wam_item_sigma_ws(items, item_stride, length, ptr(x), float(np.float32(spread)), ptr(sigma), ptr(ws),
                                ws.numel() * 8, st))
    return sigma


def noise_add(x, sigma, n_samples, items, item_stride, noised_len, seed=0, sample_base=0, host_noise=None, out=None,
              item_base=0):
    if out is None:
        out = torch.empty((n_samples * items * item_stride,), dtype=torch.float32, device=x.device)
    check(lib.wam_noise_add_ex(n_samples, items, item_stride, noised_len, ptr(x), ptr(sigma), ptr(host_noise),
                               ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), sample_base, item_base, ptr(out),
                               stream_of(x.device)))
    return out


def subband_maps(plan, coeff_grads, groups, group_items, channels, maps=None, band_max=None, want_max=True):
    """|channel mean| maps (item-major) and per-group band maxima (None when want_max=False)."""
    items = groups * group_items
    dev = coeff_grads.device
    if maps is None:
        maps = torch.empty(items * plan.coeff_numel, dtype=torch.float32, device=dev)
    if not want_max:
        band_max = None
    elif band_max is None:
        band_max = torch.zeros((groups, plan.nbands), dtype=torch.float32, device=dev)
    else:
        band_max.zero_()
    check(lib.wam_subband_maps(plan.handle, groups, group_items, channels, ptr(coeff_grads), ptr(maps),
                               ptr(band_max), stream_of(dev)))
    return maps, band_max


_INV = {}


def _inverse_map(gmap, maps_item_len):
    """(dst, cband) per packed coefficient from the per-pixel (src, band) mosaic map, or None when
    the map is not injective (cached per map)."""
    src, band = gmap
    key = (src.data_ptr(), band.data_ptr(), int(maps_item_len))
    if key not in _INV:
        valid = src >= 0
        pix = torch.nonzero(valid).reshape(-1)
        s = src[valid].long()
        dst = torch.full((maps_item_len,), -1, dtype=torch.int32, device=src.device)
        cband = torch.zeros((maps_item_len,), dtype=torch.int32, device=src.device)
        ok = s.numel() == 0 or (int(s.max()) < maps_item_len and torch.unique(s).numel() == s.numel())
        if ok:
            dst[s] = pix.to(torch.int32)
            cband[s] = band[valid]
        _INV[key] = (dst, cband, gmap) if ok else None  # gmap kept alive: its pointers are the key
    v = _INV[key]
    return None if v is None else v[:2]


def frame_accumulate(groups, group_items, gmap, maps, maps_item_len, band_max, n_bands, normalize, frame):
    src, band = gmap
    inv = _inverse_map(gmap, maps_item_len)
    if inv is not None:  # coefficient order: contiguous map reads
        check(lib.wam_frame_accumulate_coef(groups, group_items, maps_item_len, src.numel(), ptr(inv[0]), ptr(inv[1]),
                                            ptr(maps), ptr(band_max), n_bands, int(bool(normalize)), ptr(frame),
                                            stream_of(frame.device)))
        return
    check(lib.wam_frame_accumulate(groups, group_items, src.numel(), ptr(src), ptr(band), ptr(maps),
                                   maps_item_len, ptr(band_max), n_bands, int(bool(normalize)), ptr(frame),
                                   stream_of(frame.device)))


def frame_trapz(groups, k0, group_items, gmap, maps, maps_item_len, band_max, n_bands, normalize, prev, acc,
                weights=None):
    src, band = gmap
    inv = _inverse_map(gmap, maps_item_len)
    if inv is not None:  # coefficient order: contiguous map reads (prev / acc are zero outside the mosaic)
        check(lib.wam_frame_trapz_coef(groups, k0, group_items, maps_item_len, src.numel(), ptr(inv[0]),
                                       ptr(inv[1]), ptr(maps), ptr(band_max), n_bands, int(bool(normalize)),
                                       ptr(weights), ptr(prev), ptr(acc), stream_of(acc.device)))
        return
    check(lib.wam_frame_trapz(groups, k0, group_items, src.numel(), ptr(src), ptr(band), ptr(maps), maps_item_len,
                              ptr(band_max), n_bands, int(bool(normalize)), ptr(weights), ptr(prev), ptr(acc),
                              stream_of(acc.device)))


def cube_accumulate(groups, k0, group_items, src, maps, maps_item_len, mode, n_total, acc, prev=None, weights=None):
    check(lib.wam_cube_accumulate(groups, k0, group_items, src.numel(), ptr(src), ptr(maps), maps_item_len, mode,
                                  float(n_total), ptr(weights), ptr(prev), ptr(acc), stream_of(acc.device)))


def accumulate_f32(src, groups, acc, scale=0.0):
    check(lib.wam_accumulate_f32(groups, acc.numel(), ptr(src), float(scale), ptr(acc), stream_of(acc.device)))


def trapz_stream(src, groups, k0, prev, acc, weights=None):
    if acc.dtype == torch.float64:
        check(lib.wam_trapz_f32(groups, k0, acc.numel(), ptr(src), ptr(weights), None, None, ptr(prev), ptr(acc),
                                stream_of(acc.device)))
    else:
        check(lib.wam_trapz_f32(groups, k0, acc.numel(), ptr(src), ptr(weights), ptr(prev), ptr(acc), None, None,
                                stream_of(acc.device)))


def reproject_scales(avg, levels, approx):
    """avg: [items, size, size] float64 cuda -> [items, levels(+1), size, size] float64."""
    items, size = avg.shape[0], avg.shape[1]
    out = torch.empty((items, levels + (1 if approx else 0), size, size), dtype=torch.float64, device=avg.device)
    check(lib.wam_reproject_scales(items, size, levels, int(bool(approx)), ptr(avg.contiguous()), ptr(out),
                                   stream_of(avg.device)))
    return out


def disentangle_scales(plan, maps, band_max, items, approx, size):
    """BaseWAM2D.disentangle_scales on device maps -> [items, J(+1), size, size] float64."""
    out = torch.empty((items, plan.levels + (1 if approx else 0), size, size), dtype=torch.float64,
                      device=maps.device)
    check(lib.wam_disentangle_scales(plan.handle, items, ptr(maps), ptr(band_max), int(bool(approx)), int(size),
                                     ptr(out), stream_of(maps.device)))
    return out
