"""WAM for images on MI355X: drop-in for the reference's ``lib/wam_2D.py``.

Same classes, constructor arguments, call signatures, return types and side attributes as
``BaseWAM2D`` (lib/wam_2D.py:50-264) and ``WaveletAttribution2D`` (:343-536). What changes is
where the work happens: every wavelet transform, its adjoint, the SmoothGrad noise, the IG path
scaling, the per-subband channel-mean |.| with batch-global maxima and the mosaic accumulation
run as HIP kernels (libwam_hip.so) on the model's GPU; several noise samples / IG steps are
batched into one model forward/backward; nothing goes back to the host but the final map.

Build-only keyword arguments (all optional, after the reference's own):
  noise          'numpy' (default) = the reference's legacy np.random stream, bit-identical noise;
                 'philox' = counter-based Philox4x32-10 generated on the GPU (fast path).
  frame          'legacy' (default) = the reference's hard-coded 224 canvas, including its errors;
                 'native' = canvas of the input's own size (runs db4 SmoothGrad at 224, IG at 512).
  sample_batch   noise samples / IG steps per model call (default: as many as fit 256 images).
  autocast_dtype e.g. torch.bfloat16: run the explained model under autocast (WAM stays fp32).
  channels_last  feed the model NHWC tensors.
  optimize_model run an eval-mode model as a traced copy with BatchNorm folded into the convs, a
                 polyphase input-gradient for the stride-2 input conv and weights cast once to
                 autocast_dtype (wam_amd/model_opt.py); same function up to fp rounding.
  dist           True / ProcessGroup: shard the work over torch.distributed ranks (RCCL on ROCm);
                 every rank returns the full map.
  dist_axis      'samples' = noise samples / IG steps in contiguous ranges, partial maps summed by
                 one all-reduce; 'images' = the input batch in contiguous ranges, the per-sample
                 batch-global band maxima combined by an all-reduce MAX before normalising and the
                 rows gathered at the end; 'auto' (default) = 'images' when every rank gets an
                 image, else 'samples'.
  bf16_handoff   True (default): with a bf16 channels_last folded model (optimize_model +
                 autocast_dtype=torch.bfloat16 + channels_last) the SmoothGrad synthesis writes the
                 model's input as bf16 NHWC and the maps pass reads its bf16 NHWC gradient (no
                 cast / layout passes; the same values as the fp32 hand-off); False: fp32 hand-off.
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import frames
from .profiling import phase
from .constants import WaveletDetailTuple2d
from .engine import (GradModel, LegacyNoise, Shard, auto_group, chunks, ig_weights, model_device, param_grad_sum,
                     require_gpu_device, wam_budget_bytes, wam_group)
from .plan import (CAP_ADJOINT_MAPS, CAP_BF16_NHWC, CAP_NOISY_WAVEDEC, disentangle_scales, frame_accumulate, frame_trapz,
                   get_plan, item_sigma, noise_add, reproject_scales, subband_maps)


def _to_numpy_2d(plan, flat, batch_items, n, c, first_item=0):
    views = plan.split(flat, batch_items)
    out = []
    for b, v in enumerate(views):
        arr = v[first_item * c:(first_item + n) * c].reshape((n, c) + plan.band_shapes[b]).detach().cpu().numpy()
        out.append(arr)
    res = [out[0]]
    for lv in range(plan.levels):
        res.append(WaveletDetailTuple2d(out[1 + 3 * lv], out[2 + 3 * lv], out[3 + 3 * lv]))
    return res


def to_numpy(coeffs, dimension, grads=True):
    """lib/wam_2D.py:10-48: coefficient containers (tensors with .grad) -> numpy containers."""
    f = (lambda t: t.grad.detach().cpu().numpy()) if grads else (lambda t: t.detach().cpu().numpy())
    if dimension == 1:
        return [f(c) for c in coeffs]
    if dimension == 2:
        return [f(coeffs[0])] + [WaveletDetailTuple2d(f(c.horizontal), f(c.vertical), f(c.diagonal))
                                 for c in coeffs[1:]]
    raise ValueError("dimension must be 1 or 2")


def _reproject_wam(coeffs, normalize_coeffs):
    """lib/wam_2D.py:268-341 on host numpy coefficients (224 canvas, 224-based indices); the
    reference's debugging prints (:334-335) are not reproduced."""
    batch = coeffs[0].shape[0]
    vis = np.zeros((batch, 224, 224))
    ap = np.abs(coeffs[0].mean(axis=1))
    if normalize_coeffs:
        ap /= ap.max()
    vis[:, :ap.shape[1], :ap.shape[2]] = ap
    for i, coeff in enumerate(coeffs[1:][::-1]):
        e, s = int(224 / 2 ** i), int(224 / 2 ** (i + 1))
        hz = np.abs(coeff.horizontal.mean(axis=1))
        vt = np.abs(coeff.vertical.mean(axis=1))
        dg = np.abs(coeff.diagonal.mean(axis=1))
        if normalize_coeffs:
            hz /= hz.max()
            dg /= dg.max()
            vt /= vt.max()
        vis[:, s:e, s:e] = dg[:, :(e - s), :(e - s)]
        vis[:, s:e, :s] = vt[:, :(e - s), :(e - s)]
        vis[:, :s, s:e] = hz[:, :(e - s), :(e - s)]
    return vis


def _bilinear_np(a, size):
    t = torch.as_tensor(np.ascontiguousarray(a))[None, None]
    return F.interpolate(t, size=(size, size), mode="bilinear", align_corners=False)[0, 0].numpy()


class BaseWAM2D:
    """Single gradient pass in the wavelet domain (lib/wam_2D.py:50-264)."""

    def __init__(self, model, wavelet="haar", J=3, device=None, mode="reflect", approx_coeffs=False,
                 normalize_coeffs=True, *, frame="legacy", autocast_dtype=None, channels_last=False,
                 optimize_model=False, _grad=None):
        self.wavelet = wavelet
        self.J = J
        self.mode = mode
        self.approx_coeffs = approx_coeffs
        self.normalize_coeffs = normalize_coeffs
        if device is not None:
            model = model.to(device)
            self.model = model
            self.device = device
        else:
            self.model = model
            self.device = next(model.parameters()).device
        self.frame = frame
        self.autocast_dtype = autocast_dtype
        self.channels_last = channels_last
        self._grad = _grad if _grad is not None else GradModel(self.model, autocast_dtype, channels_last, optimize_model)
        self._pass = None
        self._wavelet_coeffs = None
        self._gradient_coeffs = None
        self._scales = None

    # ------------------------------------------------------------------ device helpers
    @property
    def _dev(self):
        return require_gpu_device(model_device(self.model, self.device))

    def _prep(self, x):
        if not isinstance(x, torch.Tensor):
            x = torch.as_tensor(np.asarray(x))
        return x.detach().to(self._dev, dtype=torch.float32).contiguous()

    # ------------------------------------------------------------------ lazy side attributes
    def _record_pass(self, plan, coeff_flat, grad_flat, batch_items, first_item, n, c, coeff_items=None,
                     coeff_first=None, grad_img=None):
        """Keep the last gradient pass (the reference's self.wavelet_coeffs / gradient_coeffs /
        scales, lib/wam_2D.py:120-128) on the device; host copies are made on first access.
        grad_img (optional): the input gradient [n*c, *rec] of that pass -- its coefficient
        gradients are then computed on access instead of in the hot loop."""
        ci = batch_items if coeff_items is None else coeff_items
        cf = first_item if coeff_first is None else coeff_first
        self._pass = (plan, (coeff_flat, ci, cf), (grad_flat, batch_items, first_item), n, c, grad_img)
        self._wavelet_coeffs = None
        self._gradient_coeffs = None
        self._scales = None

    @property
    def wavelet_coeffs(self):
        if self._wavelet_coeffs is None and self._pass is not None:
            plan, (cf, b, f), _, n, c, _ = self._pass
            self._wavelet_coeffs = _to_numpy_2d(plan, cf, b, n, c, f)
        return self._wavelet_coeffs

    @wavelet_coeffs.setter
    def wavelet_coeffs(self, v):
        self._wavelet_coeffs = v

    @staticmethod
    def _planes(plan, gimg, n, c):
        """A recorded input gradient as fp32 planes [n * c, *rec] (a bf16 channels_last gradient of
        the model hand-off widened: exact)."""
        if gimg.dtype != torch.float32:
            gimg = gimg.float().contiguous()
        return gimg.reshape((n * c,) + tuple(plan.rec_shape))

    @property
    def gradient_coeffs(self):
        if self._gradient_coeffs is None and self._pass is not None:
            plan, _, (gf, b, f), n, c, gimg = self._pass
            if gimg is not None:
                gf, b, f = plan.adjoint(self._planes(plan, gimg, n, c)), n * c, 0
            self._gradient_coeffs = _to_numpy_2d(plan, gf, b, n, c, f)
        return self._gradient_coeffs

    @gradient_coeffs.setter
    def gradient_coeffs(self, v):
        self._gradient_coeffs = v

    @property
    def scales(self):
        if self._scales is None and self._pass is not None:
            self._scales = self._scales_dev()
        return self._scales

    def _scales_dev(self):
        """disentangle_scales of the recorded pass on the GPU: coefficient gradients -> |channel
        mean| maps + batch maxima (wam_subband_maps) -> bilinear reprojection (k_disentangle)."""
        plan, _, (gf, b, f), n, c, gimg = self._pass
        if gimg is not None:
            gf, b, f = plan.adjoint(self._planes(plan, gimg, n, c)), n * c, 0
        views = plan.split(gf, b)
        cg = torch.cat([v[f * c:(f + n) * c].reshape(-1) for v in views])  # this pass's n*c items
        maps, bmax = subband_maps(plan, cg, 1, n, c)
        size = int(2 * plan.band_shapes[-1][1])
        return disentangle_scales(plan, maps, bmax, n, self.approx_coeffs, size).cpu().numpy()

    @scales.setter
    def scales(self, v):
        self._scales = v

    # ------------------------------------------------------------------ reference API
    @staticmethod
    def _adjoint_maps(plan, g, groups, n, c, full):
        """Backward of waverec2 + channel-mean |.| maps + per-sample band maxima: one fused HIP
        pass when the plan supports it, else the adjoint followed by wam_subband_maps."""
        if (plan.caps & CAP_ADJOINT_MAPS) and c in (1, 3):
            return plan.adjoint_maps(g, groups, n, c, full=full)
        cg = plan.adjoint(g)
        maps, bmax = subband_maps(plan, cg, groups, n, c)
        return maps, bmax, cg

    def _coeff_plan(self, coeffs):
        """Plan for an explicit coefficient list (image=False): the even spatial size whose
        decomposition has these coefficient shapes (what ptwt.waverec2 reconstructs)."""
        h1, w1 = coeffs[-1].horizontal.shape[-2:]
        from .filters import get_wavelet
        L = len(get_wavelet(self.wavelet).dec_lo)
        shape = (2 * h1 + 2 - L, 2 * w1 + 2 - L)
        plan = get_plan(2, shape, len(coeffs) - 1, self.wavelet, self.mode, self._dev)
        want = [tuple(coeffs[0].shape[-2:])] + [tuple(t.shape[-2:]) for c in coeffs[1:] for t in c]
        if want != [tuple(s) for s in plan.band_shapes]:
            raise AssertionError("padding error, please check if dec and rec wavelets are identical.")
        return plan

    def __call__(self, x, y, image=True):
        dev = self._dev
        if image:
            x = self._prep(x)
            n, c, h, w = x.shape
            plan = get_plan(2, (h, w), self.J, self.wavelet, self.mode, dev)
            flat = plan.wavedec(x.view(n * c, h, w))
        else:
            coeffs = x
            plan = self._coeff_plan(coeffs)
            n, c = coeffs[0].shape[:2]
            bands = [coeffs[0]] + [t for lv in coeffs[1:] for t in lv]
            flat = torch.cat([b.detach().to(dev, torch.float32).reshape(-1) for b in bands])
        img = plan.waverec(flat, n * c)[0].view((n, c) + plan.rec_shape)
        g = self._grad(img, y, 1, n)
        maps, bmax, cg = self._adjoint_maps(plan, g.view((n * c,) + plan.rec_shape), 1, n, c, full=True)
        self._record_pass(plan, flat, cg, n * c, 0, n, c)
        if self.frame == "native":
            canvas, base = plan.shape, plan.shape
        else:
            r = 2 * plan.band_shapes[-1][1]
            canvas, base = (r, r), (224, 224)
        gmap = frames.mosaic_map(plan, canvas, base, dev)
        frame = torch.zeros(n * canvas[0] * canvas[1], dtype=torch.float64, device=dev)
        frame_accumulate(1, n, gmap, maps, plan.coeff_numel, bmax, plan.nbands, self.normalize_coeffs, frame)
        return frame.view(n, canvas[0], canvas[1]).cpu().numpy()

    def disentangle_scales(self, coeffs, approx_coeffs=False):
        """lib/wam_2D.py:133-198 (per-sample side attribute; evaluated lazily on access)."""
        batch_size = coeffs[0].shape[0]
        img_size = int(2 * coeffs[-1].horizontal.shape[-1])
        num_levels = self.J
        vis = np.zeros((batch_size, num_levels + 1 if approx_coeffs else num_levels, img_size, img_size))
        img_batch = 0
        for i, coeff in enumerate(coeffs[1:][::-1]):
            hz = np.abs(coeff.horizontal.mean(axis=1))
            hz /= hz.max()
            dg = np.abs(coeff.diagonal.mean(axis=1))
            dg /= dg.max()
            vt = np.abs(coeff.vertical.mean(axis=1))
            vt /= vt.max()
            for img_batch in range(batch_size):
                vis[img_batch, i] = (_bilinear_np(vt[img_batch], img_size) + _bilinear_np(dg[img_batch], img_size) +
                                     _bilinear_np(hz[img_batch], img_size))
        if approx_coeffs:
            ap = np.abs(coeffs[0].mean(axis=1))
            ap /= ap.max()
            vis[img_batch, num_levels] = _bilinear_np(ap[img_batch], img_size)  # reference: stale img_batch
        return vis

    def visualize_grad_wam(self, coeffs):
        """lib/wam_2D.py:200-264 on host coefficient gradients (numpy lists)."""
        batch = coeffs[0].shape[0]
        size = int(2 * coeffs[-1].horizontal.shape[-1])
        vis = np.zeros((batch, size, size))
        ap = np.abs(coeffs[0].mean(axis=1))
        if self.normalize_coeffs:
            ap /= ap.max()
        vis[:, :ap.shape[1], :ap.shape[2]] = ap
        for i, coeff in enumerate(coeffs[1:][::-1]):
            e, s = int(224 / 2 ** i), int(224 / 2 ** (i + 1))
            hz = np.abs(coeff.horizontal.mean(axis=1))
            vt = np.abs(coeff.vertical.mean(axis=1))
            dg = np.abs(coeff.diagonal.mean(axis=1))
            if self.normalize_coeffs:
                hz /= hz.max()
                dg /= dg.max()
                vt /= vt.max()
            vis[:, s:e, s:e] = dg[:, :(e - s), :(e - s)]
            vis[:, s:e, :s] = vt[:, :(e - s), :(e - s)]
            vis[:, :s, s:e] = hz[:, :(e - s), :(e - s)]
        return vis


class WaveletAttribution2D(BaseWAM2D):
    """SmoothGrad / Integrated-Gradients WAM (lib/wam_2D.py:343-536)."""

    def __init__(self, model, wavelet="haar", method="smooth", J=3, device=None, mode="reflect", approx_coeffs=False,
                 normalize_coeffs=True, n_samples=25, stdev_spread=0.25, random_seed=42, *, noise="numpy",
                 frame="legacy", sample_batch=None, autocast_dtype=None, channels_last=False, dist=None,
                 optimize_model=False, dist_axis="auto", bf16_handoff=True):
        super().__init__(model, wavelet=wavelet, J=J, device=device, mode=mode, approx_coeffs=approx_coeffs,
                         normalize_coeffs=normalize_coeffs, frame=frame, autocast_dtype=autocast_dtype,
                         channels_last=channels_last, optimize_model=optimize_model)
        self.method = method
        self.n_samples = n_samples
        self.stdev_spread = stdev_spread
        self.random_seed = random_seed
        if noise not in ("numpy", "philox"):
            raise ValueError("noise must be 'numpy' or 'philox'")
        self.noise = noise
        self.sample_batch = sample_batch
        self.dist = dist
        if dist_axis not in ("auto", "samples", "images"):
            raise ValueError("dist_axis must be 'auto', 'samples' or 'images'")
        self.dist_axis = dist_axis
        # a bf16 channels_last model gets its input from the synthesis in that form and hands its
        # gradient to the maps pass in it (no cast / layout passes); False: the fp32 hand-off
        self.bf16_handoff = bool(bf16_handoff)
        self.wam = BaseWAM2D(model, wavelet=wavelet, J=J, mode=mode, device=device, approx_coeffs=approx_coeffs,
                             normalize_coeffs=normalize_coeffs, frame=frame, autocast_dtype=autocast_dtype,
                             channels_last=channels_last, _grad=self._grad)
        self._avg_dev = None
        self._scales_res = None

    # ------------------------------------------------------------------ .scales
    # The reference recomputes self.scales = reproject_wam(result) at the end of every SmoothGrad /
    # IG call (lib/wam_2D.py:413,457). Here the reprojection runs inside the call on the device
    # (k_reproject); the float64 host copy is made on first access of .scales.
    @property
    def scales(self):
        if self._scales is None and self._scales_res is not None:
            self._scales = self._scales_host(self._scales_res, self.J, self.approx_coeffs)
        elif self._scales is None and self._avg_dev is not None:
            self._scales = self._reproject_dev(self._avg_dev, self.J, self.approx_coeffs)
        return self._scales

    @scales.setter
    def scales(self, v):
        self._scales = v

    def _set_result(self, avg_dev):
        self._avg_dev = avg_dev
        self._scales = None
        self._scales_res = None
        if avg_dev.shape[1] == avg_dev.shape[2]:
            self._scales_res = reproject_scales(avg_dev.contiguous(), self.J, self.approx_coeffs)

    # ------------------------------------------------------------------ estimators
    def _wam_group(self, plan, n, c, model_group, total, shard, axis):
        """Samples / IG steps per transform pass. On the images axis every rank cuts the range at
        the same points (one all-reduce MAX of the band maxima per pass), so the memory budget,
        which follows each device's free memory, is agreed on first (MIN over the ranks)."""
        per_sample = 4 * n * (c * plan.coeff_numel + 2 * c * int(np.prod(plan.rec_shape)) + plan.coeff_numel)
        budget = wam_budget_bytes(plan.device)
        if axis == "images":
            budget = shard.agree_min(budget, plan.device)
        return wam_group(model_group, total, per_sample, budget)

    def _gradients(self, imgs, y, groups, n, model_group, batch=None):
        """Input gradients of `groups` stacked reference calls, model run `model_group` at a time;
        batch = (first, total) when the n images are a rank's slice of the reference batch."""
        if groups <= model_group:
            return self._grad(imgs, y, groups, n, batch=batch)
        out = torch.empty_like(imgs)
        for s0, cnt in chunks(0, groups, model_group):
            # each model group's gradient is written straight into its rows (one copy, no staging)
            self._grad(imgs[s0 * n:(s0 + cnt) * n], y, cnt, n, batch=batch, out=out[s0 * n:(s0 + cnt) * n])
        return out

    @staticmethod
    def _group_items(shard, axis, N, n):
        """Image count that sizes the sample / step chunks. On the images axis it is the largest
        rank's share ceil(N / world), the same on every rank, so all ranks cut the sample range
        at the same points and issue the same collectives (a rank-local count would pair
        band-maximum tensors of different sizes and samples across ranks)."""
        return -(-N // shard.world) if axis == "images" else n

    def _split(self, n, n_steps):
        """(shard, axis, image range, sample/step range) of this rank."""
        shard = Shard(self.dist)
        axis = self.dist_axis
        if axis == "auto":
            axis = "images" if n >= shard.world else "samples"
        if shard.world == 1:
            axis = "samples"
        if axis == "images" and n < shard.world:
            raise ValueError("dist_axis='images' needs at least one image per rank (%d images, %d ranks)"
                             % (n, shard.world))
        if axis == "images":
            return shard, axis, shard.range(n), (0, n_steps)
        return shard, axis, (0, n), shard.range(n_steps)

    def _handoff_groups(self, plan, img, y, cnt, n, c, group, batch):
        """Model input gradients and WAM maps of `cnt` samples whose reconstruction img is bf16
        channels_last [cnt * n, c, *rec] (wam_waverec_bf16_nhwc), one model group at a time: each
        group's bf16 gradient goes straight into the maps pass (wam_waverec_adjoint_maps_bf16_nhwc,
        widened on load: the maps equal the fp32 path's bit for bit) and its rows of maps / band_max.
        -> (maps, band_max, the last sample's input gradient)."""
        K = plan.coeff_numel
        maps = torch.empty(cnt * n * K, dtype=torch.float32, device=img.device)
        bmax = torch.zeros((cnt, plan.nbands), dtype=torch.float32, device=img.device)
        gk = None
        for g0, gc in chunks(0, cnt, group):
            with phase("model"):
                gk = self._grad(img[g0 * n:(g0 + gc) * n], y, gc, n, batch=batch, native=True)
            with phase("adjoint+maps"):
                if gk.dtype != torch.bfloat16:  # a loss scale was applied in fp32
                    gk = gk.reshape((gc * n * c,) + tuple(plan.rec_shape))
                plan.adjoint_maps(gk, gc, n, c, maps=maps[g0 * n * K:(g0 + gc) * n * K], band_max=bmax[g0:g0 + gc])
        last = gk[-n:] if gk.dim() == 4 else gk[-n * c:]
        return maps, bmax, last

    def smooth_gradcam(self, x, y):
        """lib/wam_2D.py:379-415."""
        dev = self._dev
        x = self._prep(x)
        N, c, h, w = x.shape
        plan = get_plan(2, (h, w), self.J, self.wavelet, self.mode, dev)
        item = c * h * w
        sigma_all = item_sigma(x, item, item, self.stdev_spread)
        shard, axis, (i_lo, i_hi), (s_lo, s_hi) = self._split(N, self.n_samples)
        n = i_hi - i_lo                      # this rank's images
        xs, sigma = x[i_lo:i_hi], sigma_all[i_lo:i_hi]
        batch = (i_lo, N) if axis == "images" else None
        gmap, (rh, rw) = frames.smooth_frame(plan, n, self.frame, dev)
        # chunk sizes from a rank-independent image count: on the images axis every rank must cut
        # the sample range at the same points (one all-reduce MAX of the band maxima per chunk)
        n_ref = self._group_items(shard, axis, N, n)
        group = auto_group(self.model, n_ref, self.sample_batch)
        # parity mode streams the host-generated legacy noise one model group at a time
        wgroup = group if self.noise == "numpy" else self._wam_group(plan, n_ref, c, group, s_hi - s_lo, shard, axis)
        frame = torch.zeros(n * rh * rw, dtype=torch.float64, device=dev)
        handoff = (self._grad.feeds_bf16_nhwc and c in (1, 3) and bool(plan.caps & CAP_BF16_NHWC)
                   and self.bf16_handoff)
        legacy = None
        if self.noise == "numpy":
            legacy = LegacyNoise(sigma_all.cpu().numpy(), (c, h, w), self.random_seed, self.n_samples, dev)
        rec = plan.rec_shape
        last = None
        with param_grad_sum(self._grad.params(), shard):  # .grad as one process leaves it
            for s0, cnt in chunks(s_lo, s_hi, wgroup):
                with phase("noise+wavedec2"):
                    if legacy is not None:
                        noisy = noise_add(xs, sigma, cnt, n, item, item, host_noise=legacy.chunk(s0, cnt, i_lo, i_hi))
                        flat = plan.wavedec(noisy.view(cnt * n * c, h, w))
                    elif plan.caps & CAP_NOISY_WAVEDEC:  # noise fused on the load
                        flat = plan.wavedec_noisy(xs, sigma, cnt, n, c, self.random_seed, s0, image_base=i_lo)
                    else:
                        noisy = noise_add(xs, sigma, cnt, n, item, item, seed=self.random_seed, sample_base=s0,
                                          item_base=i_lo)
                        flat = plan.wavedec(noisy.view(cnt * n * c, h, w))
                if handoff:
                    # the model's own dtype and layout across the boundary: bf16 NHWC reconstruction
                    # in, bf16 NHWC gradient out, maps per model group straight from it
                    with phase("waverec2"):
                        img = plan.waverec_bf16_nhwc(flat, cnt * n * c, c)
                    maps, bmax, last_g = self._handoff_groups(plan, img, y, cnt, n, c, group, batch)
                else:
                    with phase("waverec2"):
                        img = plan.waverec(flat, cnt * n * c)[0].view((cnt * n, c) + rec)
                    with phase("model"):
                        g = self._gradients(img, y, cnt, n, group, batch)
                    with phase("adjoint+maps"):
                        maps, bmax, _ = self._adjoint_maps(plan, g.view((cnt * n * c,) + rec), cnt, n, c, full=False)
                    last_g = g[(cnt - 1) * n:].reshape((n * c,) + rec)
                if axis == "images":
                    with phase("all_reduce_max"):
                        shard.all_reduce_max(bmax)  # per-sample maxima over the whole batch (A.6)
                with phase("accumulate"):
                    frame_accumulate(cnt, n, gmap, maps, plan.coeff_numel, bmax, plan.nbands, self.normalize_coeffs,
                                     frame)
                last = (plan, flat, None, cnt * n * c, (cnt - 1) * n, n, c)
        if legacy is not None:
            legacy.finish()
        if last is not None:
            self.wam._record_pass(*last, grad_img=last_g)
        with phase("collectives"):
            if axis == "images":
                frame = shard.all_gather_rows(frame.view(n, rh * rw), N).reshape(-1)
            else:
                shard.all_reduce_sum(frame)
        avg = frame.view(N, rh, rw) / self.n_samples
        self._set_result(avg)
        return avg.cpu().numpy()

    def intergrated_wam(self, x, y):
        """lib/wam_2D.py:417-459 (trapezoid over alpha = linspace(0, 1, n_samples), dx = 1)."""
        dev = self._dev
        x = self._prep(x)
        N, c, h, w = x.shape
        plan = get_plan(2, (h, w), self.J, self.wavelet, self.mode, dev)
        shard, axis, (i_lo, i_hi), (k_lo, k_hi) = self._split(N, self.n_samples)
        n = i_hi - i_lo
        batch = (i_lo, N) if axis == "images" else None
        bmap, gmap, (rh, rw) = frames.ig_frames(plan, n, self.frame, dev)
        z = plan.wavedec(x[i_lo:i_hi].reshape(n * c, h, w))
        zmaps, zmax = subband_maps(plan, z, 1, n, c)
        if axis == "images":
            shard.all_reduce_max(zmax)
        base = torch.zeros(n * rh * rw, dtype=torch.float64, device=dev)
        frame_accumulate(1, n, bmap, zmaps, plan.coeff_numel, zmax, plan.nbands, True, base)
        alphas = np.linspace(0, 1, self.n_samples)
        n_ref = self._group_items(shard, axis, N, n)
        group = auto_group(self.model, n_ref, self.sample_batch)
        wgroup = self._wam_group(plan, n_ref, c, group, k_hi - k_lo, shard, axis)
        acc = torch.zeros(n * rh * rw, dtype=torch.float32, device=dev)
        prev = torch.zeros_like(acc)
        rec = plan.rec_shape
        last = None
        with param_grad_sum(self._grad.params(), shard):
            for k0, cnt in chunks(k_lo, k_hi, wgroup):
                with phase("waverec2(alpha)"):
                    img = plan.waverec(z, n * c, alphas=alphas[k0:k0 + cnt]).view((cnt * n, c) + rec)
                with phase("model"):
                    g = self._gradients(img, y, cnt, n, group, batch)
                with phase("adjoint+maps"):
                    maps, bmax, _ = self._adjoint_maps(plan, g.view((cnt * n * c,) + rec), cnt, n, c, full=False)
                if axis == "images":
                    with phase("all_reduce_max"):
                        shard.all_reduce_max(bmax)
                weights = None
                if axis == "samples" and shard.world > 1:
                    weights = torch.from_numpy(ig_weights(k0, cnt, self.n_samples)).to(dev)
                with phase("trapz"):
                    frame_trapz(cnt, k0, n, gmap, maps, plan.coeff_numel, bmax, plan.nbands, self.normalize_coeffs,
                                prev, acc, weights)
                last = (plan, float(alphas[k0 + cnt - 1]))
                last_g = g[(cnt - 1) * n:].reshape((n * c,) + rec)
        if last is not None:
            plan_, alpha = last
            coeff = z * float(np.float32(alpha))  # the path coefficients alpha * z of the last step
            self.wam._record_pass(plan_, coeff, None, n * c, 0, n, c, grad_img=last_g)
        with phase("collectives"):
            if axis == "images":
                # base holds ONE normalised fp32 map per pixel added to 0.0 in fp64 (frame_accumulate of
                # a single sample), so its fp32 copy is exact: the gather moves half the bytes
                base = shard.all_gather_rows(base.view(n, rh * rw).float(), N).double()
                acc = shard.all_gather_rows(acc.view(n, rh * rw), N)
            else:
                shard.all_reduce_sum(acc)
        out = base.view(N, rh, rw) * acc.view(N, rh, rw).double()
        self._set_result(out)
        return out.cpu().numpy()

    def alter(self, alpha, coeffs):
        """lib/wam_2D.py:461-476."""
        altered = [coeffs[0] * alpha]
        for coeff in coeffs[1:]:
            altered.append(WaveletDetailTuple2d(coeff.horizontal * alpha, coeff.vertical * alpha,
                                                coeff.diagonal * alpha))
        return altered

    def __call__(self, x, y):
        if self.method == "smooth":
            return self.smooth_gradcam(x, y)
        if self.method == "integratedgrad":
            return self.intergrated_wam(x, y)
        return None

    # ------------------------------------------------------------------ reprojection
    def _reproject_dev(self, avg_dev, num_levels, approx_coeffs):
        if avg_dev.shape[2] != avg_dev.shape[1]:
            raise NotImplementedError("reproject_wam on a non-square map")
        return self._scales_host(reproject_scales(avg_dev.contiguous(), self.J, approx_coeffs), num_levels,
                                 approx_coeffs)

    def _scales_host(self, sc_dev, num_levels, approx_coeffs):
        """device reprojection [N, J(+1), S, S] -> the reference's .scales array (levels as asked)."""
        n, size = sc_dev.shape[0], sc_dev.shape[2]
        sc = sc_dev.cpu().numpy()
        out = np.zeros((n, num_levels + 1 if approx_coeffs else num_levels, size, size))
        for j in range(self.J):
            if j >= out.shape[1]:
                raise IndexError("index %d is out of bounds for axis 1 with size %d" % (j, out.shape[1]))
            out[:, j] = sc[:, j]
        if approx_coeffs:
            out[:, num_levels] = sc[:, self.J]
        return out

    def reproject_wam(self, average_gradients, num_levels, approx_coeffs=False):
        """lib/wam_2D.py:488-536 (cv2 INTER_LINEAR reprojection as a HIP kernel)."""
        avg = torch.as_tensor(np.asarray(average_gradients, dtype=np.float64)).to(self._dev)
        return self._reproject_dev(avg, num_levels, approx_coeffs)
