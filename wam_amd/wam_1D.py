"""WAM for audio on MI355X: drop-in for the reference's ``lib/wam_1D.py`` attribution classes.

``BaseWAM1D`` (lib/wam_1D.py:54-246) and ``WaveletAttribution1D`` (:249-435) with the same
constructor arguments, ``__call__`` signatures, returns ``(melspec gradients, [coefficient
gradients per level])`` and side attributes (``wavelet_coeffs``, ``gradient_coeffs``,
``melspecs``, ``grad_coeffs``, ``rates``). wavedec / waverec / the adjoint, the SmoothGrad noise,
the IG path scaling and the sample accumulators are HIP kernels; the mel front-end is a batched
torch.stft on the GPU (wam_amd/melspec.py). Build-only kwargs as in wam_amd.wam_2D (noise,
sample_batch, autocast_dtype, dist).
"""
import numpy as np
import torch

from .engine import (Shard, auto_group, chunks, ig_weights, input_gradient, LegacyNoise, model_device,
                     param_grad_sum, require_gpu_device, trainable_params)
from .melspec import kernel_supported, mel_adjoint, mel_forward, melspec_db
from .profiling import phase
from .plan import CAP_NOISY_WAVEDEC, accumulate_f32, get_plan, item_sigma, noise_add, trapz_stream


def normalize(data):
    """lib/wam_1D.py:439-440 (min-max over the whole array)."""
    return (data - np.min(data)) / (np.max(data) - np.min(data))


def process_in_chunks(melspec, chunk_size, sr, n_fft, nnls="lbfgsb"):
    """lib/wam_1D.py:442-448: librosa.feature.inverse.mel_to_stft of a [n_mels, T] power mel
    spectrogram in time chunks of chunk_size frames, hstacked -> [1 + n_fft // 2, T] float32
    magnitudes. Each chunk is one librosa NNLS problem (its objective is scaled by the chunk's own
    size), solved as librosa solves it: clipped pinv start on the device, scipy's L-BFGS-B driving
    float64 objective / gradient evaluations on the device (wam_amd.melspec.nnls_lbfgsb).
    nnls="exact" (build-only keyword) returns the exact NNLS minimiser of every frame instead
    (batched FISTA; the chunks are then one batch and chunk_size is only validated)."""
    from .melspec import mel_to_stft
    chunk_size = int(chunk_size)
    if chunk_size == 0:
        raise ValueError("range() arg 3 must not be zero")
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
    m = torch.as_tensor(np.asarray(melspec, dtype=np.float32))
    m = m.to(require_gpu_device(dev or "cpu"))
    if nnls == "exact":
        if chunk_size < 0:
            raise ValueError("need at least one array to concatenate")
        return mel_to_stft(m, sr, n_fft, nnls="exact").cpu().numpy()
    parts = [mel_to_stft(m[:, i:i + chunk_size], sr, n_fft, nnls=nnls) for i in range(0, m.shape[1], chunk_size)]
    if not parts:  # np.hstack([]) in the reference
        raise ValueError("need at least one array to concatenate")
    return torch.cat(parts, dim=1).cpu().numpy()


def _peak_normalise(x):
    return torch.tensor(np.array([wf / wf.max() for wf in x]).astype(np.float32))


class BaseWAM1D:
    def __init__(self, model, wavelet="haar", J=2, mode="symmetric", device=None, approx_coeffs=False, n_mels=128,
                 n_fft=1024, sample_rate=44100, *, autocast_dtype=None):
        self.wavelet = wavelet
        self.J = J
        self.mode = mode
        self.approx_coeffs = approx_coeffs
        self.n_mels = n_mels
        self.n_fft = n_fft
        self.sample_rate = sample_rate
        if device is not None:
            model = model.to(device)
            self.model = model
            self.device = device
        else:
            self.model = model
            self.device = next(model.parameters()).device
        self.autocast_dtype = autocast_dtype
        self._pass = None
        self._wc = None
        self._gc = None

    @property
    def _dev(self):
        return require_gpu_device(model_device(self.model, self.device))

    # ------------------------------------------------------------------ lazy side attributes
    def _split_np(self, plan, flat, items, first, n):
        return [v[first:first + n].detach().cpu().numpy() for v in plan.split(flat, items)]

    @property
    def wavelet_coeffs(self):
        if self._wc is None and self._pass is not None:
            plan, (cf, ci, c0), _, n = self._pass
            self._wc = self._split_np(plan, cf, ci, c0, n)
        return self._wc

    @wavelet_coeffs.setter
    def wavelet_coeffs(self, v):
        self._wc = v

    @property
    def gradient_coeffs(self):
        if self._gc is None and self._pass is not None:
            plan, _, (gf, gi, g0), n = self._pass
            self._gc = self._split_np(plan, gf, gi, g0, n)
        return self._gc

    @gradient_coeffs.setter
    def gradient_coeffs(self, v):
        self._gc = v

    def _record(self, plan, cf, ci, c0, gf, gi, g0, n):
        self._pass = (plan, (cf, ci, c0), (gf, gi, g0), n)
        self._wc = self._gc = None

    # ------------------------------------------------------------------ core pass (batched groups)
    def _grads(self, plan, flat, items, y, groups, n):
        """waverec -> melspec -> model -> (melspec grad [items,1,T,M], coefficient grads flat)."""
        return self._grads_from_rec(plan, plan.waverec(flat, items)[0], y, groups, n)

    def _grads_from_rec(self, plan, rec, y, groups, n):
        args = (self.n_fft, self.sample_rate, self.n_mels)
        if kernel_supported(self.n_fft, self.n_mels):  # k_mel_fwd -> model -> k_mel_adj
            mel = mel_forward(rec, *args).unsqueeze(1)
            g_mel = input_gradient(self.model, mel, y, groups, n, self.autocast_dtype)
            return g_mel, plan.adjoint(mel_adjoint(rec, g_mel, *args))
        rec_leaf = rec.detach().requires_grad_(True)
        with torch.enable_grad():
            mel = melspec_db(rec_leaf, *args)
        g_mel = input_gradient(self.model, mel.detach(), y, groups, n, self.autocast_dtype)
        (g_rec,) = torch.autograd.grad(mel, rec_leaf, grad_outputs=g_mel)
        return g_mel, plan.adjoint(g_rec.contiguous())

    def compute_melspec(self, reconstruction, n_fft=1024, sample_rate=44100, n_mels=128):
        """lib/wam_1D.py:194-219: [N, W] -> [N, 1, T, n_mels] (on the GPU)."""
        rec = torch.as_tensor(reconstruction)
        rec = rec.to(self._dev, torch.float32) if rec.device.type != "cuda" else rec
        return melspec_db(rec, n_fft, sample_rate, n_mels)

    def __call__(self, x, y, rates=None, waveform=True):
        self.rates = rates
        dev = self._dev
        if waveform:
            if isinstance(x, list):
                x = _peak_normalise(x)
            x = x.detach().to(dev, torch.float32).contiguous()
            n, w = x.shape
            plan = get_plan(1, (w,), self.J, self.wavelet, self.mode, dev)
            flat = plan.wavedec(x)
        else:
            coeffs = list(x)
            n = coeffs[0].shape[0]
            from .filters import get_wavelet
            L = len(get_wavelet(self.wavelet).dec_lo)
            plan = get_plan(1, (2 * coeffs[-1].shape[-1] + 2 - L,), len(coeffs) - 1, self.wavelet, self.mode, dev)
            flat = torch.cat([c.detach().to(dev, torch.float32).reshape(-1) for c in coeffs])
        g_mel, cg = self._grads(plan, flat, n, y, 1, n)
        self._record(plan, flat, n, 0, cg, n, 0, n)
        grads = [v.detach().cpu().numpy() for v in plan.split(cg, n)]
        return g_mel.detach().cpu().numpy().squeeze(), grads

    def filter(self, EPS):
        """lib/wam_1D.py:221-246: keep the coefficients whose |gradient| / max(gradient) (signed
        max over the band, as the reference) exceeds EPS and reconstruct (pywt.waverec ->
        wam_waverec). Masks on the device; returns [N, rec_len] float32."""
        if self._pass is None:
            raise AttributeError("'BaseWAM1D' object has no attribute 'gradient_coeffs'")
        plan, (cf, ci, c0), (gf, gi, g0), n = self._pass
        cb = [v[c0:c0 + n] for v in plan.split(cf, ci)]
        gb = [v[g0:g0 + n] for v in plan.split(gf, gi)]
        flat = torch.cat([(c * ((g.abs() / g.max()) > EPS).float()).reshape(-1) for c, g in zip(cb, gb)])
        return plan.waverec(flat, n)[0].cpu().numpy()

    def visualize_grad_wam(self, coeffs):
        """lib/wam_1D.py:152-192 (host numpy pseudo-scaleogram)."""
        batch = coeffs[0].shape[0]
        max_length = coeffs[-1].shape[1]
        sc = np.ones((batch, self.J + 1, max_length)) * np.nan
        for i in range(batch):
            samples = [c[i] for c in coeffs]
            ap = np.abs(samples[0])
            ap /= ap.max()
            sc[i, 0, :ap.shape[0]] = ap
            for j, d in enumerate(samples[1:]):
                d = np.abs(d)
                d /= d.max()
                sc[i, j + 1, :d.shape[0]] = d
        return sc


class WaveletAttribution1D(BaseWAM1D):
    def __init__(self, model, wavelet="haar", J=3, method="smooth", mode="reflect", device=None, approx_coeffs=False,
                 n_mels=128, n_fft=1024, sample_rate=44100, n_samples=25, stdev_spread=0.001, random_seed=42, *,
                 noise="numpy", sample_batch=None, autocast_dtype=None, dist=None):
        super().__init__(model, wavelet=wavelet, J=J, device=device, mode=mode, approx_coeffs=approx_coeffs,
                         n_mels=n_mels, n_fft=n_fft, sample_rate=sample_rate, autocast_dtype=autocast_dtype)
        self.n_samples = n_samples
        self.stdev_spread = stdev_spread
        self.random_seed = random_seed
        self.method = method
        if noise not in ("numpy", "philox"):
            raise ValueError("noise must be 'numpy' or 'philox'")
        self.noise = noise
        self.sample_batch = sample_batch
        self.dist = dist
        self.wam = BaseWAM1D(model, wavelet=wavelet, J=J, mode=mode, device=device, approx_coeffs=approx_coeffs,
                             n_mels=n_mels, n_fft=n_fft, sample_rate=sample_rate, autocast_dtype=autocast_dtype)

    def smooth_wam(self, x, y):
        """lib/wam_1D.py:294-343: mean over noisy samples of the raw gradients."""
        dev = self._dev
        if isinstance(x, list):
            x = _peak_normalise(x)
        x = x.detach().to(dev, torch.float32).contiguous()
        n, w = x.shape
        plan = get_plan(1, (w,), self.J, self.wavelet, self.mode, dev)
        sigma = item_sigma(x, w, w, self.stdev_spread)
        shard = Shard(self.dist)
        s_lo, s_hi = shard.range(self.n_samples)
        group = auto_group(self.model, n, self.sample_batch)
        legacy = None
        if self.noise == "numpy":
            legacy = LegacyNoise(sigma.cpu().numpy(), (w,), self.random_seed, self.n_samples, dev)
        # accumulators exist before the loop: a rank whose sample range is empty (n_samples <
        # world size) still joins the all-reduce with zeros
        self._mel_shape = (n, 1, plan.rec_shape[0] // (self.n_fft // 2) + 1, self.n_mels)
        mel_acc = torch.zeros(int(np.prod(self._mel_shape)), dtype=torch.float32, device=dev)
        c_acc = torch.zeros(n * plan.coeff_numel, dtype=torch.float32, device=dev)
        with param_grad_sum(trainable_params(self.model), shard):
            for s0, cnt in chunks(s_lo, s_hi, group):
                with phase("noise+wavedec"):
                    if legacy is None and plan.caps & CAP_NOISY_WAVEDEC:  # noise fused on the load
                        flat = plan.wavedec_noisy(x, sigma, cnt, n, 1, self.random_seed, s0)
                    else:
                        host = None if legacy is None else legacy.chunk(s0, cnt)
                        noisy = noise_add(x, sigma, cnt, n, w, w, seed=self.random_seed, sample_base=s0,
                                          host_noise=host)
                        flat = plan.wavedec(noisy.view(cnt * n, w))
                with phase("waverec+mel+model+adjoint"):
                    g_mel, cg = self._grads(plan, flat, cnt * n, y, cnt, n)
                if g_mel.numel() != cnt * mel_acc.numel():
                    raise RuntimeError("melspec gradient shape %s does not match %s" % (tuple(g_mel.shape),
                                                                                         self._mel_shape))
                accumulate_f32(g_mel, cnt, mel_acc)
                for b in range(plan.nbands):
                    nb = int(np.prod(plan.band_shapes[b]))
                    src = cg[cnt * n * plan.band_offsets[b]:cnt * n * (plan.band_offsets[b] + nb)]
                    accumulate_f32(src, cnt, c_acc[n * plan.band_offsets[b]:n * (plan.band_offsets[b] + nb)])
                self.wam._record(plan, flat, cnt * n, (cnt - 1) * n, cg, cnt * n, (cnt - 1) * n, n)
        if legacy is not None:
            legacy.finish()
        with phase("collectives"):
            shard.all_reduce_sum(mel_acc)
            shard.all_reduce_sum(c_acc)
        accumulate_f32(mel_acc, 0, mel_acc, scale=float(self.n_samples))
        accumulate_f32(c_acc, 0, c_acc, scale=float(self.n_samples))
        mel = mel_acc.view(self._mel_shape).cpu().numpy().squeeze()
        avg = [v.cpu().numpy() for v in plan.split(c_acc, n)]
        self.melspecs = mel
        self.grad_coeffs = avg
        return mel, avg

    def alter(self, alpha, coeffs):
        return [alpha * c for c in coeffs]

    def integrated_wam(self, x, y):
        """lib/wam_1D.py:353-421."""
        dev = self._dev
        if isinstance(x, list):
            x = _peak_normalise(x)
        x = x.detach().to(dev, torch.float32).contiguous()
        n, w = x.shape
        plan = get_plan(1, (w,), self.J, self.wavelet, self.mode, dev)
        alphas = np.linspace(0, 1, self.n_samples)
        z = plan.wavedec(x)
        base_z = [v.cpu().numpy() for v in plan.split(z, n)]
        base_mel = melspec_db(x, self.n_fft, self.sample_rate, self.n_mels).squeeze(1).detach()
        shard = Shard(self.dist)
        k_lo, k_hi = shard.range(self.n_samples)
        group = auto_group(self.model, n, self.sample_batch)
        mel_acc = torch.zeros(base_mel.numel(), dtype=torch.float64, device=dev)
        mel_prev = torch.zeros_like(mel_acc)
        c_acc = torch.zeros(n * plan.coeff_numel, dtype=torch.float32, device=dev)
        c_prev = torch.zeros_like(c_acc)
        with param_grad_sum(trainable_params(self.model), shard):
            for k0, cnt in chunks(k_lo, k_hi, group):
                img = plan.waverec(z, n, alphas=alphas[k0:k0 + cnt]).view(cnt * n, -1)
                g_mel, cg = self._grads_from_rec(plan, img, y, cnt, n)
                weights = None
                if shard.world > 1:
                    weights = torch.from_numpy(ig_weights(k0, cnt, self.n_samples)).to(dev)
                trapz_stream(g_mel, cnt, k0, mel_prev, mel_acc, weights)
                for b in range(plan.nbands):
                    nb = int(np.prod(plan.band_shapes[b]))
                    lo, hi = n * plan.band_offsets[b], n * (plan.band_offsets[b] + nb)
                    src = cg[cnt * n * plan.band_offsets[b]:cnt * n * (plan.band_offsets[b] + nb)]
                    trapz_stream(src, cnt, k0, c_prev[lo:hi], c_acc[lo:hi], weights)
        shard.all_reduce_sum(mel_acc)
        shard.all_reduce_sum(c_acc)
        mel = base_mel.cpu().numpy() * mel_acc.view(base_mel.shape).cpu().numpy()
        prod = [b * i for b, i in zip(base_z, [v.cpu().numpy() for v in plan.split(c_acc, n)])]
        self.melspecs = mel
        self.grad_coeffs = prod
        return mel, prod

    def __call__(self, x, y):
        if self.method == "smooth":
            return self.smooth_wam(x, y)
        elif self.method == "integratedgrad":
            return self.integrated_wam(x, y)


class VisualizerWAM1D(WaveletAttribution1D):
    """lib/wam_1D.py:451-643: filtering of the explained waveforms by their attributions.

    On the device: the wavelet-domain filters (hard threshold 'ht', soft 'st', scale-weighted
    'modulation') on wam_wavedec / wam_waverec, the mel-spectrogram filters, the power mel
    spectrogram. The reference's spectrograms come from librosa (absent offline, parity
    unpinned): ``spectrogram_from_waveform`` restates librosa.stft's magnitude (hann window,
    centred, constant padding -- librosa >= 0.10 -- hop n_fft // 4) with torch.stft on the GPU;
    ``compute_spectrogram`` is librosa's mel_to_stft (NNLS of the Slaney mel basis by librosa's own
    L-BFGS-B scheme, objective evaluated on the device, then sqrt; wam_amd.melspec.nnls_lbfgsb), which
    ``filtered_spectrogram_from_melspec`` uses on the source and the filtered mel spectrograms."""

    def __init__(self, model, x, wavelet="haar", J=3, method="smooth", mode="reflect", device=None,
                 approx_coeffs=False, n_mels=128, n_fft=1024, sample_rate=44100, n_samples=25, stdev_spread=0.001,
                 random_seed=42, **kw):
        super().__init__(model, wavelet, J, method, mode, device, approx_coeffs, n_mels, n_fft, sample_rate, n_samples,
                         stdev_spread, random_seed, **kw)
        self.source_spectrograms = None
        self.x = x

    def _wave(self, x):
        if isinstance(x, list):
            return _peak_normalise(x).to(self._dev)
        return torch.as_tensor(np.asarray(x), dtype=torch.float32).to(self._dev)

    def compute_melspec(self, x):
        """power mel spectrograms [N, n_mels, frames] float32 (no dB), as the reference (:460-478)."""
        from .melspec import melspec_power
        return melspec_power(self._wave(x), self.n_fft, self.sample_rate, self.n_mels).cpu().numpy()

    def compute_spectrogram(self, melspecs, chunk_size=100, nnls="lbfgsb"):
        """lib/wam_1D.py:478-488: the STFT magnitudes of power mel spectrograms [N, n_mels, T] by
        librosa.feature.inverse.mel_to_stft per waveform, in chunks of chunk_size frames
        (process_in_chunks) -> [N, 1 + n_fft // 2, T] float32: librosa's NNLS (clipped pinv start,
        scipy L-BFGS-B over float64 objective evaluations on the device), i.e. the reference's
        result. nnls="exact" (build-only keyword) returns the exact NNLS minimiser of every frame
        (one batched device solve; not the reference's early-stopped iterate: the minimiser is not
        unique and the two differ in the basis' null space)."""
        from .melspec import mel_to_stft
        if nnls == "exact":
            if int(chunk_size) < 1:
                raise ValueError("range() arg 3 must not be zero")
            m = torch.as_tensor(np.asarray(melspecs, dtype=np.float32)).to(self._dev)
            return mel_to_stft(m, self.sample_rate, self.n_fft, nnls="exact").cpu().numpy()
        return np.array([process_in_chunks(m, chunk_size, self.sample_rate, self.n_fft, nnls=nnls)
                         for m in np.asarray(melspecs, dtype=np.float32)])

    def filter_melspec(self, audio_melspecs, grad_melspecs, filtering_method, EPS=0.2):
        """lib/wam_1D.py:491-519 (hard threshold of the min-max-normalised gradient, or modulation)."""
        a = torch.as_tensor(np.asarray(audio_melspecs)).to(self._dev)
        g = torch.as_tensor(np.asarray(grad_melspecs)).to(self._dev).permute(0, 2, 1)
        if filtering_method == "ht":
            g = (g - g.min()) / (g.max() - g.min())
            return (a * (g > EPS).to(a.dtype)).cpu().numpy()
        elif filtering_method == "modulation":
            return (a * g.abs()).cpu().numpy()
        return None

    def spectrogram_from_waveform(self, waveform):
        """|librosa.stft(waveform, n_fft, hop_length=n_fft // 4)| (hann, centred, constant pad)."""
        w = self._wave(waveform)
        win = torch.hann_window(self.n_fft, device=w.device, dtype=w.dtype)
        st = torch.stft(w, n_fft=self.n_fft, hop_length=self.n_fft // 4, win_length=self.n_fft, window=win,
                        center=True, pad_mode="constant", return_complex=True)
        return st.abs().cpu().numpy()

    def _filtered_coeffs(self, coefficients, gradients, filtering_method="ht", EPS=0.2):
        """wavelet-domain filters of :532-587 on device bands -> list of filtered bands."""
        cs = [torch.as_tensor(np.asarray(c), dtype=torch.float32).to(self._dev) for c in coefficients]
        gs = [torch.as_tensor(np.asarray(g), dtype=torch.float32).to(self._dev) for g in gradients]

        def normalize(d):
            return (d - d.min()) / (d.max() - d.min())
        if filtering_method == "ht":
            return [c * ((g.abs() / g.max()) > EPS).to(c.dtype) for c, g in zip(cs, gs)]
        if filtering_method == "st":
            return [c * torch.clamp(normalize(c * g) - EPS, min=0) for c, g in zip(cs, gs)]
        if filtering_method == "modulation":
            imp = torch.stack([g.sum(dim=1) for g in gs])                   # [levels, N]
            nimp = (imp / imp.sum(dim=0, keepdim=True)).t()                 # [N, levels]
            return [c * g.abs() * nimp[:, j:j + 1] for j, (c, g) in enumerate(zip(cs, gs))]
        raise UnboundLocalError("local variable 'filtered_coeffs' referenced before assignment")

    def filter_from_wavelet_coefficients(self, coefficients, gradients, filtering_method="ht", EPS=0.2):
        """lib/wam_1D.py:532-587: filter in the wavelet domain, reconstruct (pywt.waverec ->
        wam_waverec); returns [N, rec_len] float32."""
        fc = self._filtered_coeffs(coefficients, gradients, filtering_method, EPS)
        n = fc[0].shape[0]
        from .filters import get_wavelet
        L = len(get_wavelet(self.wavelet).dec_lo)
        plan = get_plan(1, (2 * fc[-1].shape[-1] + 2 - L,), len(fc) - 1, self.wavelet, self.mode, self._dev)
        return plan.waverec(torch.cat([c.reshape(-1) for c in fc]), n)[0].cpu().numpy()

    def filtered_spectrogram_from_wavelet_coefficients(self, grad_coeffs, filtering_method, EPS=0.2):
        """lib/wam_1D.py:589-617: spectrograms of x and of x filtered in the wavelet domain."""
        x = np.asarray(self.x)
        if x.dtype == np.int16:
            x = np.array([wf / wf.max() for wf in self.x]).astype(np.float32)
            self.x = x
        self.source_spectrograms = self.spectrogram_from_waveform(x)
        xd = torch.as_tensor(np.asarray(x), dtype=torch.float32).to(self._dev)
        plan = get_plan(1, (xd.shape[-1],), self.J, self.wavelet, self.mode, self._dev)
        coeffs = plan.split(plan.wavedec(xd.reshape(-1, xd.shape[-1])), xd.reshape(-1, xd.shape[-1]).shape[0])
        sounds = self.filter_from_wavelet_coefficients(coeffs, grad_coeffs, filtering_method=filtering_method, EPS=EPS)
        return self.source_spectrograms, self.spectrogram_from_waveform(sounds)

    def filtered_spectrogram_from_melspec(self, grad_melspecs, filtering_method, EPS=0.2, chunk_size=100,
                                          nnls="lbfgsb"):
        """lib/wam_1D.py:619-643 (nnls: build-only keyword, see compute_spectrogram)."""
        audio = self.compute_melspec(self.x)
        self.source_spectrograms = self.compute_spectrogram(audio, chunk_size=chunk_size, nnls=nnls)
        return self.source_spectrograms, self.compute_spectrogram(
            self.filter_melspec(audio, grad_melspecs, filtering_method, EPS=EPS), chunk_size=chunk_size, nnls=nnls)
