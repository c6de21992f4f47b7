"""Shared host logic of the WAM classes: device placement, the model's input gradient with the
reference's loss semantics, SmoothGrad noise streams, sample / step sharding across ranks.

Loss (lib/wam_2D.py:115, lib/wam_1D.py:125, lib/wam_3D.py:237): ``torch.diag(output[:, y]).mean()``.
For an int y its gradient is 1/N^2 on out[i, y]; for a sequence it is 1/N on out[i, y_i]. Several
noise samples (or IG steps) are stacked into ONE model batch of groups x N images; the loss is the
sum of the per-group losses, so each group gets exactly the gradient of its own reference call
(models must not couple batch items -- eval-mode BatchNorm is fine; training-mode models are run
one group per call).
Parameter gradients: the reference's ``loss.backward()`` leaves every parameter that requires
grad with its gradient accumulated in ``.grad`` (lib/wam_2D.py:116, lib/wam_1D.py:126,
lib/wam_3D.py:237-238). The same backward here takes ``torch.autograd.grad`` with respect to the
input and to those parameters and adds the latter into ``.grad`` -- the sum over the stacked
groups is the sum of the reference's per-call gradients. A model whose parameters are frozen
(requires_grad False, as the bench does) pays for the input gradient only. ``optimize_model=True``
runs a folded copy of the model and does not touch the user's parameters. Sharded calls
(dist=True) all-reduce the increments once per call (``param_grad_sum``), so every rank's .grad
holds the single-process gradient.
"""
import collections
import contextlib
import math
import os

import numpy as np
import torch
import torch.distributed as tdist


def model_device(model, device=None):
    if device is not None:
        return torch.device(device)
    return next(model.parameters()).device


def require_gpu_device(device):
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError("wam_amd runs the WAM path on the GPU only; the explained model lives on %s. "
                           "Pass device='cuda' or move the model to a HIP device." % device)
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    return device


def _is_int_label(y):
    return isinstance(y, (int, np.integer)) or (isinstance(y, torch.Tensor) and y.dim() == 0)


def seed_gradient(out, y, groups, n, unit=False, batch=None):
    """d loss / d out for `groups` stacked reference calls of n items each.
    batch = (first, total): the n items are items [first, first + n) of a reference batch of
    `total` items (a batch-sharded rank); the loss scale and y's indexing follow the whole batch.
    unit=True: the seed holds 1.0 where the loss gradient is non-zero and the loss scale (1/N^2,
    1/N or 1/k) is returned beside it, so a low-precision model output (bf16) does not round the
    scale -- the caller applies it to the fp32 input gradient. A power-of-two scale (c2: 1/64) is
    exact in bf16 and commutes with every rounding of the backward (absent under- / overflow), so
    it is seeded directly (scale None): the same gradient without the caller's fp32 pass over it.
    Returns (seed, scale or None)."""
    first, total = (0, n) if batch is None else batch
    go = torch.zeros_like(out, dtype=torch.float32)
    rows = torch.arange(groups * n, device=out.device)
    if _is_int_label(y):
        val = torch.tensor(1.0, dtype=torch.float32) / (total * total)
        rr, cc = rows, torch.full((groups * n,), int(y), dtype=torch.long, device=out.device)
    else:
        yy = torch.as_tensor(np.asarray([int(v) for v in (y.tolist() if isinstance(y, torch.Tensor) else y)]),
                             dtype=torch.long)
        # the reference's diag(output[:, y]) takes min(N, len(y)) entries (all N when len(y) == N)
        k = min(total, yy.numel())
        val = torch.tensor(1.0, dtype=torch.float32) / k
        sel = torch.arange(n)[first + torch.arange(n) < k]       # local items with a diagonal entry
        rr = (torch.arange(groups)[:, None] * n + sel[None, :]).reshape(-1).to(out.device)
        cc = yy[first + sel].repeat(groups).to(out.device)
    if unit and math.frexp(float(val))[0] != 0.5:  # not a power of two
        go[rr, cc] = 1.0
        return go.to(out.dtype), float(val)
    go[rr, cc] = val.to(out.device)
    return go.to(out.dtype), None


def trainable_params(model):
    return [p for p in model.parameters() if p.requires_grad] if isinstance(model, torch.nn.Module) else []


def input_gradient(model, img, y, groups, n, autocast_dtype=None, channels_last=False, y_none_mean=False,
                   input_dtype=None, batch=None, params=None, out=None, native=False):
    """Gradient of the summed per-group reference losses w.r.t. img (fp32, contiguous; written into
    `out` when given). params (default: the model's parameters that require grad): their gradients
    are accumulated into .grad, as the reference's loss.backward() does. The gradient is taken
    w.r.t. the tensor the model is fed (bf16 and / or channels_last) and converted to img's dtype
    and layout by ONE copy into the result -- autograd's cast and the layout copy were two more
    passes over it; the values are the same (the bf16 -> fp32 cast is exact).
    native=True: img is already the fed tensor (e.g. bf16 channels_last from
    wam_waverec_bf16_nhwc) and the gradient is returned in that dtype, in whichever dense layout
    (NCHW or NHWC) the model's backward produced it, without any conversion pass, whenever no loss
    scale has to be applied after the backward (power-of-two scales are seeded; otherwise the fp32
    contiguous gradient is returned as without native)."""
    img = img.detach().requires_grad_(True)
    inp = img if input_dtype is None else img.to(input_dtype)
    inp = inp.contiguous(memory_format=torch.channels_last) if channels_last and img.dim() == 4 else inp
    params = trainable_params(model) if params is None else list(params)
    ctx = torch.autocast("cuda", dtype=autocast_dtype) if autocast_dtype is not None else contextlib.nullcontext()
    with torch.enable_grad():
        with ctx:
            res = model(inp)
        # allow_unused: parameters outside the graph (an eval-mode auxiliary head, a conditional
        # branch) get no gradient, exactly as loss.backward() leaves their .grad untouched
        if y_none_mean:
            scale = None
            gs = torch.autograd.grad(res.float().mean(), [inp] + params, allow_unused=True)
        else:
            seed, scale = seed_gradient(res, y, groups, n, unit=res.dtype != torch.float32, batch=batch)
            gs = torch.autograd.grad(res, [inp] + params, grad_outputs=seed, allow_unused=True)
    g = gs[0]
    if g is None:
        raise RuntimeError("the model's output does not depend on its input")
    with torch.no_grad():
        if native and out is None and scale is None and g.dtype == img.dtype and (
                g.is_contiguous() or g.is_contiguous(memory_format=torch.channels_last)):
            out = g  # the fed dtype, NCHW or NHWC: the maps pass reads either
        elif native and out is None:  # a scale to apply: the fp32 contiguous gradient
            out = torch.empty(img.shape, dtype=torch.float32, device=img.device)
            out.copy_(g)
        elif out is None and g.dtype == img.dtype and g.is_contiguous():
            out = g
        else:
            out = torch.empty(img.shape, dtype=img.dtype, device=img.device) if out is None else out
            out.copy_(g)
        if scale is not None:
            out.mul_(scale)
        for p, gp in zip(params, gs[1:]):
            if gp is None:
                continue
            gp = gp if scale is None else gp * scale
            _accumulate_param_grad(p, gp)
    return out


# Parameter gradients of a sharded call (dist=True): while a `param_grad_sum` block is open the
# per-rank increments are collected here instead of in .grad, then summed over the ranks once and
# added to .grad -- every rank ends with the single-process call's gradient, as the reference's
# loss.backward() leaves it (lib/wam_2D.py:116).
_PARAM_SINK = None


def _accumulate_param_grad(p, gp):
    if _PARAM_SINK is not None:
        prev = _PARAM_SINK.get(p)
        _PARAM_SINK[p] = gp.float().clone() if prev is None else prev.add_(gp.float())
        return
    if p.grad is None:
        p.grad = gp.to(p.dtype).clone()
    else:
        p.grad.add_(gp.to(p.grad.dtype))


@contextlib.contextmanager
def param_grad_sum(params, shard):
    """Collect the parameter-gradient increments of one sharded call and all-reduce them (SUM,
    one flat buffer, every rank in the same parameter order -- a rank with no work contributes
    zeros) before adding them to .grad. A no-op for one rank or a model without trainable
    parameters."""
    global _PARAM_SINK
    params = list(params)
    if shard.world == 1 or not params:
        yield
        return
    prev, _PARAM_SINK = _PARAM_SINK, {}
    try:
        yield
        sink = _PARAM_SINK
    finally:
        _PARAM_SINK = prev
    # one flat SUM: the increments, then one has-gradient flag per parameter. A parameter that no
    # rank reached (an unused head, a branch not taken) keeps .grad untouched, as loss.backward()
    # leaves it in the single-process call; zeros would make optimizers treat it as a gradient.
    dev = params[0].device
    flags = torch.tensor([1.0 if p in sink else 0.0 for p in params], dtype=torch.float32, device=dev)
    flat = torch.cat([(sink[p] if p in sink else torch.zeros(p.shape, dtype=torch.float32, device=p.device))
                      .reshape(-1).to(dev) for p in params] + [flags])
    shard.all_reduce_sum(flat)
    got = flat[-len(params):].tolist()
    off = 0
    for p, f in zip(params, got):
        gp = flat[off:off + p.numel()].view(p.shape)
        off += p.numel()
        if f > 0:
            _accumulate_param_grad(p, gp)


class GradModel:
    """How the explained model is run for its input gradient. optimize=False: the user's model as
    is (autocast if requested). optimize=True: a traced, BN-folded, frozen copy cast once to
    autocast_dtype (wam_amd/model_opt.py), built on first use on the model's device."""

    def __init__(self, model, autocast_dtype=None, channels_last=False, optimize=False):
        self.model = model
        self.autocast_dtype = autocast_dtype
        self.channels_last = channels_last
        self.optimize = optimize
        self._run = None

    def _runner(self):
        if self._run is None:
            if self.optimize:
                from .model_opt import optimize_for_input_grad
                run = optimize_for_input_grad(self.model, dtype=self.autocast_dtype)
                if self.channels_last:
                    run = run.to(memory_format=torch.channels_last)
                self._run = run
            else:
                self._run = self.model
        return self._run

    def params(self):
        """The parameters whose .grad a call accumulates (none for the folded copy)."""
        return [] if self.optimize else trainable_params(self.model)

    @property
    def feeds_bf16_nhwc(self):
        """The model is fed bf16 channels_last images (the folded bf16 copy): the WAM path can hand
        them over in that form (wam_waverec_bf16_nhwc) and take the gradient back in it."""
        return self.optimize and self.autocast_dtype == torch.bfloat16 and self.channels_last

    def __call__(self, img, y, groups, n, y_none_mean=False, batch=None, out=None, native=False):
        run = self._runner()
        if self.optimize:  # a folded copy: the user's parameters are not touched
            return input_gradient(run, img, y, groups, n, None, self.channels_last, y_none_mean,
                                  input_dtype=self.autocast_dtype, batch=batch, params=[], out=out, native=native)
        return input_gradient(run, img, y, groups, n, self.autocast_dtype, self.channels_last, y_none_mean,
                              batch=batch, out=out)


def legacy_noise(sigmas, item_shape, seed, samples, n_total=None):
    """The reference's stream (lib/wam_2D.py:385-403): np.random.seed(seed) then, for every sample
    and item in order, np.random.normal(0, sigma_i, item_shape) in float64 cast to float32.
    Yields (s, float32 array [items, *item_shape]) for s in `samples` (a sorted list); earlier
    samples are generated and discarded so the stream position is identical on every rank.
    Uses (and leaves advanced) the global numpy RNG, exactly like the reference."""
    np.random.seed(seed)
    want = set(samples)
    last = max(samples) if samples else -1
    for s in range(last + 1):
        arr = np.empty((len(sigmas),) + tuple(item_shape), dtype=np.float32)
        for i, sg in enumerate(sigmas):
            arr[i] = np.random.normal(0, sg, tuple(item_shape)).astype(np.float32)
        if s in want:
            yield s, arr


# (seed, item numel, items, samples, device) -> (device float64 [samples, items, numel] standard
# normals, numpy global RNG state after them); least recently used entries go first
_GAUSS_CACHE = collections.OrderedDict()
GAUSS_CACHE_BYTES = 4 << 30


def clear_noise_cache():
    _GAUSS_CACHE.clear()


class LegacyNoise:
    """The reference's noise stream (lib/wam_2D.py:385-403, lib/wam_1D.py:305-322,
    lib/wam_3D.py:567-579): np.random.seed(seed), then for every sample s and item i in order
    np.random.normal(0, sigma_i, item_shape) in float64, cast to float32 -- replayed on the device.

    numpy's legacy normal is ``loc + scale * gauss`` over the unscaled MT19937 / polar sequence, and
    that sequence depends only on (seed, item size, items, samples), not on the images. It is drawn
    with np.random.standard_normal (the same generator calls in the same order) and scaled on the
    device: float32(sigma_i * g) is the reference's value bit for bit (IEEE fp64 product,
    round-to-nearest cast; 0.0 + v = v).

    Two forms, same values:
    * cached (the whole draw fits GAUSS_CACHE_BYTES): drawn once per (seed, item size, items,
      samples), kept on the device in float64 (bounded LRU cache);
    * streamed (larger draws): nothing is kept; chunk() draws the requested samples on the host in
      stream order (samples before a rank's range are drawn and discarded), uploads and scales
      them, and drops them -- host and device memory stay at one chunk.
    The global numpy RNG is left where the reference leaves it, after all n_samples samples: a cache
    hit restores that state; the streamed form draws the rest of the stream in finish()."""

    def __init__(self, sigmas, item_shape, seed, n_samples, device):
        numel = int(np.prod(item_shape))
        items = len(sigmas)
        self.numel, self.items, self.n_samples = numel, items, int(n_samples)
        self.device = device
        self.sigma = torch.tensor([float(v) for v in sigmas], dtype=torch.float64, device=device)
        self.shape = tuple(item_shape)
        self.g = None
        self._rs = None
        key = (int(seed), numel, items, int(n_samples), str(device))
        ent = _GAUSS_CACHE.get(key)
        if ent is None and n_samples * items * numel * 8 <= GAUSS_CACHE_BYTES:
            rs = np.random.RandomState(seed)
            g = np.empty((n_samples, items, numel), dtype=np.float64)
            for s in range(n_samples):
                for i in range(items):
                    g[s, i] = rs.standard_normal(numel)
            ent = (torch.from_numpy(g).to(device), rs.get_state())
            _GAUSS_CACHE[key] = ent
            while sum(v[0].numel() * 8 for v in _GAUSS_CACHE.values()) > GAUSS_CACHE_BYTES:
                _GAUSS_CACHE.popitem(last=False)
        if ent is not None:
            _GAUSS_CACHE.move_to_end(key)
            np.random.set_state(ent[1])
            self.g = ent[0]
        else:
            self._rs = np.random.RandomState(seed)   # streamed: private generator, global state at finish()
            self._next = 0                           # next sample of the stream

    @property
    def streamed(self):
        return self.g is None

    def _draw(self, s0, cnt):
        """float64 standard normals [cnt, items, numel] of samples s0.. (streamed form)."""
        if s0 < self._next:
            raise RuntimeError("streamed legacy noise is drawn in sample order (sample %d after %d)"
                               % (s0, self._next))
        while self._next < s0:  # samples before the requested range: drawn and discarded
            for _ in range(self.items):
                self._rs.standard_normal(self.numel)
            self._next += 1
        g = np.empty((cnt, self.items, self.numel), dtype=np.float64)
        for s in range(cnt):
            for i in range(self.items):
                g[s, i] = self._rs.standard_normal(self.numel)
        self._next += cnt
        return g

    def chunk(self, s0, cnt, i_lo=0, i_hi=None):
        """float32 noise [cnt, items, *item_shape] of samples s0 .. s0+cnt-1, items [i_lo, i_hi)."""
        i_hi = self.items if i_hi is None else i_hi
        if self.g is not None:
            g = self.g[s0:s0 + cnt, i_lo:i_hi]
        else:
            g = torch.from_numpy(self._draw(s0, cnt)[:, i_lo:i_hi]).to(self.device)
        z = g * self.sigma[i_lo:i_hi, None]
        return z.float().view((cnt, i_hi - i_lo) + self.shape)

    def finish(self):
        """Leave the global numpy RNG at the reference's end state (after all n_samples)."""
        if self._rs is not None:
            if self._next < self.n_samples:
                self._draw(self.n_samples, 0)
            np.random.set_state(self._rs.get_state())
            self._rs = None


# ------------------------------------------------------------------------------ distribution
class Shard:
    """Which noise samples / IG steps this process evaluates, and how partial results combine.
    dist=None/False: everything local. dist=True: the default torch.distributed group (RCCL on
    ROCm for cuda tensors); or pass a ProcessGroup."""

    def __init__(self, dist=None):
        if dist is None or dist is False or not (tdist.is_available() and tdist.is_initialized()):
            self.group, self.rank, self.world = None, 0, 1
        else:
            self.group = None if dist is True else dist
            self.rank = tdist.get_rank(self.group)
            self.world = tdist.get_world_size(self.group)

    def range(self, n):
        """Contiguous block of [0, n) for this rank (ragged: the first n % world ranks get one more)."""
        return Shard.range_of(self.rank, self.world, n)

    def all_reduce_sum(self, t):
        if self.world > 1:
            tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=self.group)
        return t

    def all_reduce_max(self, t):
        if self.world > 1:
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX, group=self.group)
        return t

    def agree_min(self, value, device):
        """The smallest of the ranks' `value`s (an int), on every rank: sizes that decide how many
        collectives a rank issues must be the same everywhere."""
        if self.world == 1:
            return int(value)
        t = torch.tensor([float(value)], dtype=torch.float64, device=device)
        tdist.all_reduce(t, op=tdist.ReduceOp.MIN, group=self.group)
        return int(t.item())

    def all_gather_rows(self, t, n):
        """t: this rank's rows [range(n)] of an [n, ...] tensor -> the whole tensor on every rank
        (ragged ranges padded to the longest for the collective)."""
        if self.world == 1:
            return t
        q = -(-n // self.world)
        pad = t.new_zeros((q,) + tuple(t.shape[1:]))
        pad[:t.shape[0]] = t
        parts = [torch.empty_like(pad) for _ in range(self.world)]
        tdist.all_gather(parts, pad, group=self.group)
        out = []
        for r in range(self.world):
            lo, hi = Shard.range_of(r, self.world, n)
            out.append(parts[r][:hi - lo])
        return torch.cat(out)

    @staticmethod
    def range_of(rank, world, n):
        q, r = divmod(n, world)
        start = rank * q + min(rank, r)
        return start, start + q + (1 if rank < r else 0)


def ig_weights(k0, cnt, n):
    """Trapezoid weights (dx = 1) of path steps k0..k0+cnt-1 out of n, for the sharded form
    acc = sum_k w_k G_k (== np.trapz up to fp32 summation order)."""
    if n == 1:
        return np.zeros(cnt, dtype=np.float32)
    return np.array([0.5 if k in (0, n - 1) else 1.0 for k in range(k0, k0 + cnt)], dtype=np.float32)


def legacy3d_weights(s0, cnt, n):
    """Weights of the reference's in-loop 3D averaging (lib/wam_3D.py:582-587):
    avg_{s+1} = (avg_s + cube_s) / n  =>  avg_n = sum_s cube_s * n^-(n-s)."""
    return np.array([float(n) ** (-(n - s)) for s in range(s0, s0 + cnt)], dtype=np.float32)


def chunks(start, stop, size):
    out = []
    s = start
    while s < stop:
        out.append((s, min(size, stop - s)))
        s += size
    return out


BUDGET_BYTES = None   # explicit override of wam_budget_bytes (bytes), e.g. for memory-tight models


def wam_budget_bytes(device=None):
    """Device memory the WAM buffers of one transform pass may take: an eighth of the device's HBM,
    8-64 GiB (36 GiB on a 288 GB MI355X), capped by half of what is free on the device now (free
    HBM plus this process's cached, unallocated blocks: the model's own footprint and other
    processes -- ranks sharing the device included -- are already out of it), rounded down to a
    tier (multiples of 4 GiB from 8 GiB up, powers of two below) so that the split of a call into
    passes (and with it the fp32 summation order of the trapezoid / frame sums) does not follow the
    caching allocator from call to call.
    Larger passes read the trapezoid accumulators and the synthesis details fewer times per call.
    Ranks that share one device (LOCAL_WORLD_SIZE > device count, e.g. the one-GPU gloo rehearsals)
    read its free memory before the others have allocated, so each claims its share of the half.
    BUDGET_BYTES overrides it."""
    if BUDGET_BYTES is not None:
        return int(BUDGET_BYTES)
    budget = 8 << 30
    try:
        if torch.cuda.is_available():
            total = torch.cuda.get_device_properties(device).total_memory
            budget = min(max(total // 8, 8 << 30), 64 << 30)
            free, _ = torch.cuda.mem_get_info(device)
            free += torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device)
            budget = min(budget, max(free // (2 * ranks_per_device()), 1 << 30))
    except (RuntimeError, AssertionError, ValueError):
        pass
    return budget_tier(budget)


def ranks_per_device():
    """Local ranks sharing each visible device: ceil(LOCAL_WORLD_SIZE / device count), >= 1."""
    try:
        lws = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    except ValueError:
        lws = 1
    nd = torch.cuda.device_count() if torch.cuda.is_available() else 1
    return max(1, -(-lws // max(1, nd)))


def budget_tier(b):
    """Round a byte budget down to its tier: multiples of 4 GiB from 8 GiB, powers of two below."""
    b = int(b)
    if b >= 8 << 30:
        return (b >> 32) << 32
    return 1 << (max(b, 1).bit_length() - 1)


def wam_group(model_group, total, bytes_per_sample, budget_bytes=None):
    """Samples (IG steps) per WAM transform launch: a multiple of the model group, as many as the
    rank's range and a device-memory budget allow (wam_budget_bytes). The transforms then run on
    thousands of planes per launch (full-chip grids, one launch per pass) while the model still sees
    `model_group`."""
    if budget_bytes is None:
        budget_bytes = wam_budget_bytes()
    k = max(1, int(budget_bytes // max(1, bytes_per_sample)) // max(1, model_group))
    return max(1, min(total, k * model_group))


def auto_group(model, n_items, requested, cap_items=256):
    if requested is not None:
        return max(1, int(requested))
    if getattr(model, "training", False):
        return 1
    return max(1, cap_items // max(1, n_items))
