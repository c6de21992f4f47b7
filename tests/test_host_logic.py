"""Host-side logic of wam_amd on the CPU: mosaic / cube gather maps vs the reference's slice
assignments, loss seed gradients vs autograd of diag(out[:, y]).mean(), the numpy noise stream,
sample/step sharding and the sharded-accumulation weights."""
import math

import numpy as np
import pytest
import torch

from oracle import dwt, wam_ref
from wam_amd import engine, frames


class FakePlan:
    """Band layout of a plan without a device (sizes from the oracle's level rules)."""

    def __init__(self, ndim, shape, J, wavelet):
        L = len(dwt.filter_bank(wavelet)[0])
        per_axis = [dwt.level_sizes(n, L, J) for n in shape]
        self.ndim, self.shape, self.levels = ndim, tuple(shape), J
        per = (1 << ndim) - 1
        self.band_shapes = [tuple(a[J - 1] for a in per_axis)]
        for lv in range(J - 1, -1, -1):
            self.band_shapes += [tuple(a[lv] for a in per_axis)] * per
        self.band_offsets = [0]
        for s in self.band_shapes:
            self.band_offsets.append(self.band_offsets[-1] + int(np.prod(s)))
        self.coeff_numel = self.band_offsets[-1]
        self.nbands = len(self.band_shapes)

    def __hash__(self):
        return hash((self.ndim, self.shape, self.levels, tuple(self.band_shapes)))


def _apply(gmap_src, gmap_band, maps_item, bmax, normalize):
    src = gmap_src.numpy()
    band = gmap_band.numpy()
    out = np.zeros(src.shape, dtype=np.float64)
    ok = src >= 0
    v = maps_item[src[ok]]
    if normalize:
        v = v / bmax[band[ok]]
    out[ok] = v
    return out


@pytest.mark.parametrize("wav,size,J,frame", [("haar", 224, 3, "legacy"), ("db4", 224, 3, "native"),
                                              ("sym8", 96, 2, "native"), ("haar", 224, 5, "legacy"),
                                              ("db6", 104, 3, "native")])
def test_mosaic_gather_map_matches_reference_assignments(wav, size, J, frame):
    rs = np.random.RandomState(0)
    p = FakePlan(2, (size, size), J, wav)
    n = 2
    bands = [np.abs(rs.standard_normal((n,) + s)).astype(np.float32) for s in p.band_shapes]
    # oracle container order = ptwt band order: [A_J, (H,V,D)_J, ..., (H,V,D)_1]
    grads = [bands[0][:, None]] + [tuple(bands[1 + 3 * i + k][:, None] for k in range(3)) for i in range(J)]
    (src, band), (rh, rw) = frames.smooth_frame(p, n, frame, "cpu")
    canvas, base = wam_ref.frame_geometry(frame, size, size, p.band_shapes[-1][1])
    ref = wam_ref.mosaic_2d(grads, True, canvas, base)
    bmax = np.array([b.max() for b in bands], dtype=np.float32)
    for i in range(n):
        packed = np.concatenate([b[i].reshape(-1) for b in bands])
        got = _apply(src, band, packed, bmax, True).reshape(rh, rw)
        assert np.array_equal(got, ref[i])


def test_legacy_frame_errors():
    with pytest.raises(ValueError):
        frames.smooth_frame(FakePlan(2, (224, 224), 3, "db4"), 1, "legacy", "cpu")  # 230 canvas
    with pytest.raises(ValueError):
        frames.ig_frames(FakePlan(2, (128, 128), 3, "haar"), 1, "legacy", "cpu")   # IG is 224-only
    with pytest.raises(ValueError):
        frames.smooth_frame(FakePlan(2, (224, 224), 6, "haar"), 1, "legacy", "cpu")  # J >= 6
    frames.ig_frames(FakePlan(2, (224, 224), 3, "sym8"), 1, "legacy", "cpu")        # runs in the reference


def test_cube_map_matches_refactor():
    rs = np.random.RandomState(1)
    p = FakePlan(3, (16, 16, 16), 2, "haar")
    bands = [rs.standard_normal(s).astype(np.float32) for s in p.band_shapes]
    keys = ["aad", "ada", "add", "daa", "dad", "dda", "ddd"]
    c = [bands[0]] + [{k: bands[1 + 7 * i + j] for j, k in enumerate(keys)} for i in range(2)]
    ref = wam_ref.refactor_3d([c], 2, 16)[0]
    src = frames.cube_map(p, 16, "cpu").numpy()
    packed = np.abs(np.concatenate([b.reshape(-1) for b in bands]))
    assert (src >= 0).all()
    assert np.array_equal(packed[src].reshape(16, 16, 16), ref)


@pytest.mark.parametrize("y,n", [(3, 4), ([1, 5, 2, 2], 4), (torch.tensor([0, 1, 2]), 3), ([4, 5], 3), (7, 1)])
def test_seed_gradient_matches_autograd_of_reference_loss(y, n):
    groups = 3
    out = torch.randn(groups * n, 10, requires_grad=True)
    loss = sum(torch.diag(out[s * n:(s + 1) * n][:, y]).mean() for s in range(groups))
    (g_ref,) = torch.autograd.grad(loss, out)
    g, scale = engine.seed_gradient(out.detach(), y, groups, n)
    assert scale is None and torch.equal(g, g_ref)
    # unit seed + fp32 scale (the bf16-model form): same gradient, the scale applied afterwards;
    # a power-of-two scale is seeded directly (exact in bf16)
    gu, scale = engine.seed_gradient(out.detach(), y, groups, n, unit=True)
    if scale is None:
        assert torch.equal(gu, g_ref) and math.frexp(float(g_ref.abs().max()))[0] == 0.5
    else:
        assert set(gu.unique().tolist()) <= {0.0, 1.0}
        assert torch.equal(gu * scale, g_ref)


def test_bf16_power_of_two_seed_equals_unit_seed_then_scale():
    """The bf16 backward seeded with a power-of-two loss scale gives the unit-seed gradient times
    that scale bit for bit (rounding commutes with power-of-two scaling)."""
    torch.manual_seed(3)
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.ReLU(), torch.nn.Flatten(),
                            torch.nn.Linear(8 * 6 * 6, 10)).to(torch.bfloat16)
    img = torch.randn(8, 3, 8, 8)
    y = [1, 2, 3, 4, 5, 6, 7, 0]  # k = 8: scale 1/8
    run = lambda t: m(t.to(torch.bfloat16))
    g = engine.input_gradient(run, img, y, 1, 8)
    x = img.detach().requires_grad_(True)
    out = run(x)
    seed = torch.zeros_like(out)
    seed[torch.arange(8), torch.tensor(y)] = 1.0
    (gu,) = torch.autograd.grad(out, x, grad_outputs=seed)
    assert torch.equal(g, gu * 0.125)


@pytest.mark.parametrize("y,n", [(3, 5), ([1, 5, 2, 2, 0], 5), ([4, 5], 5), (list(range(7)), 5)])
def test_seed_gradient_batch_slices(y, n):
    """A batch-sharded rank seeds exactly its rows of the whole batch's loss gradient."""
    groups = 2
    out = torch.randn(groups * n, 10)
    full, _ = engine.seed_gradient(out, y, groups, n)
    full = full.view(groups, n, 10)
    for lo, hi in [(0, 2), (2, 4), (4, 5), (1, 5)]:
        part, _ = engine.seed_gradient(out.view(groups, n, 10)[:, lo:hi].reshape(-1, 10), y, groups, hi - lo,
                                       batch=(lo, n))
        assert torch.equal(part.view(groups, hi - lo, 10), full[:, lo:hi])


def test_input_gradient_bf16_scale_not_rounded():
    """The 1/N^2 loss scale is applied in fp32 after a bf16 backward (1/9 is not a bf16 value)."""
    torch.manual_seed(0)
    lin = torch.nn.Linear(4, 5).to(torch.bfloat16)
    img = torch.randn(3, 4)
    g = engine.input_gradient(lambda t: lin(t.to(torch.bfloat16)), img, 2, 1, 3)
    want = lin.weight[2].float() * float(torch.tensor(1.0) / 9)
    assert torch.equal(g, want.expand(3, 4).contiguous())


@pytest.mark.parametrize("y", [3, [1, 4]])
def test_input_gradient_accumulates_parameter_grads_like_reference(y):
    """The reference's loss.backward() leaves the model's parameter gradients accumulated in .grad
    (lib/wam_2D.py:116) over every call; input_gradient over stacked groups leaves their sum."""
    import testmodels
    torch.manual_seed(1)
    groups, n = 3, 2
    img = torch.randn(groups * n, 3, 32, 32)
    ref_m, m = testmodels.TinySmooth2D(), testmodels.TinySmooth2D()
    for s in range(groups):  # the reference: one call (one backward) per sample
        x = img[s * n:(s + 1) * n].clone().requires_grad_(True)
        torch.diag(ref_m(x)[:, y]).mean().backward()
    engine.input_gradient(m, img[:n], y, 1, n)             # a first call ...
    engine.input_gradient(m, img[n:], y, groups - 1, n)    # ... then two stacked groups: accumulated
    for (name, p), q in zip(m.named_parameters(), ref_m.parameters()):
        assert torch.allclose(p.grad, q.grad, rtol=1e-5, atol=1e-7), name
    frozen = testmodels.TinySmooth2D()
    for p in frozen.parameters():
        p.requires_grad_(False)
    engine.input_gradient(frozen, img, y, groups, n)
    assert all(p.grad is None for p in frozen.parameters())


def test_input_gradient_unused_trainable_parameters():
    """A trainable submodule outside the graph (an eval-mode auxiliary head) gets no gradient and
    raises nothing, as loss.backward() leaves it (autograd.grad without allow_unused)."""
    import testmodels

    class WithAux(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.body = testmodels.TinySmooth2D()
            self.aux = torch.nn.Linear(3, 3)   # never called in forward

        def forward(self, x):
            return self.body(x)

    torch.manual_seed(2)
    m = WithAux()
    img = torch.randn(4, 3, 16, 16)
    g = engine.input_gradient(m, img, [1, 2], 2, 2)
    assert g.shape == img.shape and torch.isfinite(g).all()
    assert m.aux.weight.grad is None and m.aux.bias.grad is None
    assert all(p.grad is not None for p in m.body.parameters())
    gm = engine.GradModel(m)
    assert len(gm.params()) == len(list(m.parameters()))
    assert engine.GradModel(m, optimize=True).params() == []


def test_param_grad_sum_single_rank_is_plain_accumulation():
    """One rank: param_grad_sum is a no-op and .grad accumulates directly."""
    import testmodels
    torch.manual_seed(3)
    a, b = testmodels.TinySmooth2D(), testmodels.TinySmooth2D()
    img = torch.randn(2, 3, 16, 16)
    engine.input_gradient(a, img, 1, 1, 2)
    with engine.param_grad_sum(engine.trainable_params(b), engine.Shard(None)):
        engine.input_gradient(b, img, 1, 1, 2)
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p.grad, q.grad)


def test_wam_budget_override():
    old = engine.BUDGET_BYTES
    try:
        engine.BUDGET_BYTES = 12345
        assert engine.wam_budget_bytes() == 12345
        assert engine.wam_group(2, 100, 1000, engine.wam_budget_bytes()) == 12
    finally:
        engine.BUDGET_BYTES = old
    assert engine.wam_budget_bytes() >= 1 << 30


def test_wam_budget_ranks_sharing_a_device(monkeypatch):
    """two ranks on one device (LOCAL_WORLD_SIZE 2, one visible device) each claim half of
    the half of the free memory they both see; one rank per device claims the half."""
    class Props:
        total_memory = 288 << 30
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda d=None: Props())
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda d=None: (100 << 30, 288 << 30))
    monkeypatch.setattr(torch.cuda, "memory_reserved", lambda d=None: 0)
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda d=None: 0)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert engine.ranks_per_device() == 1 and engine.wam_budget_bytes() == 36 << 30
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert engine.ranks_per_device() == 2 and engine.wam_budget_bytes() == 24 << 30
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert engine.ranks_per_device() == 1 and engine.wam_budget_bytes() == 36 << 30


def test_wam_budget_tiers(monkeypatch):
    """The default budget is rounded to a tier, so a call's split into passes does not drift with
    the allocator."""
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert engine.budget_tier(36 << 30) == 36 << 30
    assert engine.budget_tier((37 << 30) + 12345) == 36 << 30
    assert engine.budget_tier(9 << 30) == 8 << 30
    assert engine.budget_tier(3 << 30) == 2 << 30
    assert engine.budget_tier(1 << 30) == 1 << 30
    b = engine.wam_budget_bytes()
    assert b == engine.budget_tier(b) and b >= 1 << 30


def test_legacy_noise_stream_matches_reference_loop():
    x = torch.tensor(np.random.RandomState(3).standard_normal((3, 2, 5, 5)).astype(np.float32))
    sig = [float(0.25 * (x[i].max() - x[i].min())) for i in range(3)]
    ref = [noisy for _, noisy in wam_ref.legacy_noise_stream(x, 4, 0.25, 42)]
    got = dict(engine.legacy_noise(sig, (2, 5, 5), 42, [1, 3]))
    for s in (1, 3):
        assert np.array_equal((x + torch.tensor(got[s])).numpy(), ref[s].numpy())


def _np_state_equal(a, b):
    return a[0] == b[0] and np.array_equal(a[1], b[1]) and a[2:] == b[2:]


@pytest.mark.parametrize("shape,items,samples", [((2, 5, 5), 3, 4), ((7,), 2, 5), ((3, 4, 4, 4), 1, 3)])
def test_legacy_noise_device_replay_bit_exact(shape, items, samples):
    """engine.LegacyNoise (unscaled stream drawn once, scaled on the device in fp64, cast to fp32)
    equals the reference loop np.random.normal(0, sigma_i, shape).astype(float32) bit for bit, for
    full and partial (sharded) sample / item ranges, on a cache miss and a cache hit, and leaves the
    global numpy RNG in the reference's end state both times (odd item sizes: the polar method's
    cached second value carries across items)."""
    engine.clear_noise_cache()
    sig = [0.1 + 0.37 * i for i in range(items)]
    want = dict(engine.legacy_noise(sig, shape, 42, list(range(samples))))
    end = np.random.get_state()
    for attempt in range(2):  # miss, then hit
        np.random.seed(7)  # a different state: the replay must not depend on it
        ln = engine.LegacyNoise(np.asarray(sig), shape, 42, samples, "cpu")
        assert _np_state_equal(np.random.get_state(), end)
        full = ln.chunk(0, samples).numpy()
        for s in range(samples):
            assert np.array_equal(full[s], want[s]), (attempt, s)
        part = ln.chunk(1, samples - 1, items - 1, items).numpy()
        for k in range(samples - 1):
            assert np.array_equal(part[k], want[1 + k][items - 1:items])
    assert len(engine._GAUSS_CACHE) == 1
    engine.clear_noise_cache()


@pytest.mark.parametrize("shape,items,samples", [((2, 5, 5), 3, 5), ((7,), 2, 6)])
def test_legacy_noise_streamed_above_cap_bit_exact(monkeypatch, shape, items, samples):
    """A draw above the cache cap is streamed chunk by chunk (nothing cached, host and device
    memory one chunk) and gives the cached form's bits; a rank's later sample range (earlier
    samples drawn and discarded) too; finish() leaves the global RNG at the reference's end state."""
    engine.clear_noise_cache()
    sig = [0.2 + 0.31 * i for i in range(items)]
    want = dict(engine.legacy_noise(sig, shape, 42, list(range(samples))))
    end = np.random.get_state()
    monkeypatch.setattr(engine, "GAUSS_CACHE_BYTES", 8)  # nothing fits
    for s_lo in (0, 2):
        np.random.seed(7)
        ln = engine.LegacyNoise(np.asarray(sig), shape, 42, samples, "cpu")
        assert ln.streamed and len(engine._GAUSS_CACHE) == 0
        got = {}
        for s0, cnt in engine.chunks(s_lo, samples - 1, 2):
            part = ln.chunk(s0, cnt).numpy()
            for k in range(cnt):
                got[s0 + k] = part[k]
        for s, v in got.items():
            assert np.array_equal(v, want[s]), (s_lo, s)
        with pytest.raises(RuntimeError):
            ln.chunk(0, 1)  # streamed draws go forward only
        ln.finish()
        assert _np_state_equal(np.random.get_state(), end)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("n", [1, 3, 25, 64])
def test_shard_ranges_partition(world, n):
    seen = []
    for r in range(world):
        s = engine.Shard.__new__(engine.Shard)
        s.group, s.rank, s.world = None, r, world
        lo, hi = s.range(n)
        seen.extend(range(lo, hi))
        assert hi - lo in (n // world, n // world + 1)
    assert seen == list(range(n))


def test_sharded_weights_reproduce_sequential_forms():
    rs = np.random.RandomState(5)
    for n in (1, 2, 5, 25):
        G = rs.standard_normal((n, 7)).astype(np.float32)
        ref = np.trapz(G, axis=0)
        w = np.concatenate([engine.ig_weights(k0, c, n) for k0, c in engine.chunks(0, n, 3)])
        assert np.allclose((w[:, None] * G).sum(0), ref, rtol=1e-5, atol=1e-6)
        cube = np.abs(G)
        avg = np.zeros(7, dtype=np.float32)
        for s in range(n):
            avg = (avg + cube[s]) / np.float32(n)
        w3 = engine.legacy3d_weights(0, n, n)
        assert np.allclose((w3[:, None] * cube).sum(0), avg, rtol=1e-5, atol=1e-30)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_image_axis_chunks_rank_independent(world):
    """dist_axis='images': every rank cuts the sample / step range at the same points whatever its
    share of an uneven batch (one all-reduce MAX of the band maxima per chunk must pair equal
    tensors of the same samples)."""
    from types import SimpleNamespace
    from wam_amd.wam_2D import WaveletAttribution2D
    model = torch.nn.Linear(1, 1).eval()
    for N in range(world, 41):
        plans = set()
        for r in range(world):
            lo, hi = engine.Shard.range_of(r, world, N)
            shard = SimpleNamespace(world=world, rank=r)
            n_ref = WaveletAttribution2D._group_items(shard, "images", N, hi - lo)
            group = engine.auto_group(model, n_ref, None)
            plans.add(tuple(engine.chunks(0, 25, group)))
        assert len(plans) == 1, (N, plans)


def test_auto_group():
    m = torch.nn.Linear(2, 2).eval()
    assert engine.auto_group(m, 64, None) == 4
    assert engine.auto_group(m, 1, None) == 256
    assert engine.auto_group(m.train(), 64, None) == 1
    assert engine.auto_group(m, 64, 3) == 3


def test_philox_known_answers():
    """Random123 known-answer vectors for Philox4x32-10 (the host restatement of rng.hpp)."""
    from tests.helpers import philox4x32_10
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in kat:
        got = philox4x32_10(*[np.array([v]) for v in ctr], *key)
        assert tuple(int(v[0]) for v in got) == want


def test_mel_tables_csr_matches_filterbank():
    """MelTables (the tables k_mel_fwd / k_mel_adj read): both CSR forms rebuild the dense
    filterbank, bins ascending within a band and bands ascending within a bin; twiddles/window."""
    from wam_amd.melspec import MelTables, mel_filterbank
    for n_fft, n_mels, sr in [(1024, 128, 16000), (1024, 128, 44100), (256, 40, 8000)]:
        t = MelTables(n_fft, n_mels, sr, "cpu")
        fb, win = mel_filterbank(n_fft, n_mels, sr, "cpu")
        tab, idx = t.tables.numpy(), t.index.numpy()
        nf, nnz, M = n_fft // 2 + 1, t.nnz, n_fft // 2
        band_ptr = idx[:n_mels + 1]
        band_bin = idx[n_mels + 1:n_mels + 1 + nnz]
        bin_ptr = idx[n_mels + 1 + nnz:n_mels + 1 + nnz + M + 2]
        bin_band = idx[n_mels + 1 + nnz + M + 2:]
        band_w, bin_w = tab[3 * n_fft:3 * n_fft + nnz], tab[3 * n_fft + nnz:]
        assert len(bin_band) == nnz and len(bin_w) == nnz
        d1, d2 = np.zeros((nf, n_mels), np.float32), np.zeros((nf, n_mels), np.float32)
        for m in range(n_mels):
            bins = band_bin[band_ptr[m]:band_ptr[m + 1]]
            assert np.all(np.diff(bins) > 0)
            d1[bins, m] = band_w[band_ptr[m]:band_ptr[m + 1]]
        for k in range(nf):
            bands = bin_band[bin_ptr[k]:bin_ptr[k + 1]]
            assert np.all(np.diff(bands) > 0)
            d2[k, bands] = bin_w[bin_ptr[k]:bin_ptr[k + 1]]
        assert np.array_equal(d1, fb.numpy()) and np.array_equal(d2, fb.numpy())
        assert np.array_equal(tab[:n_fft], win.numpy())
        tw = tab[n_fft:3 * n_fft].reshape(-1, 2)
        assert np.allclose(tw[:, 0] + 1j * tw[:, 1], np.exp(-2j * np.pi * np.arange(n_fft) / n_fft), atol=1e-7)


@pytest.mark.parametrize("hw", [(256, 256), (230, 230), (112, 112), (300, 200), (224, 257), (96, 96), (225, 224)])
def test_pil_bilinear_tables_reproduce_pillow(hw):
    """Eval2DWAM's default Resize((224, 224)) on non-224 reconstructions (src/evaluators.py:593-598):
    the host tables (wam_amd.evaluation.pil_bilinear_coeffs) driven through the two fixed-point
    passes the HIP kernels run (restated here in numpy) give Pillow's own bytes."""
    from PIL import Image
    from wam_amd.evaluation import pil_bilinear_coeffs
    H, W = hw
    u8 = np.random.RandomState(H * 7 + W).randint(0, 256, (H, W, 3)).astype(np.uint8)
    ref = np.asarray(Image.fromarray(u8).resize((224, 224), Image.BILINEAR))
    src = u8.astype(np.int64)
    half, bits = 1 << 21, 22
    if W != 224:
        _, bh, kh = pil_bilinear_coeffs(W, 224)
        src = np.stack([np.clip((half + (src[:, b0:b0 + c] * kh[x, :c, None]).sum(1)) >> bits, 0, 255)
                        for x, (b0, c) in enumerate(bh)], 1)
    if H != 224:
        _, bv, kv = pil_bilinear_coeffs(H, 224)
        src = np.stack([np.clip((half + (src[b0:b0 + c] * kv[y, :c, None, None]).sum(0)) >> bits, 0, 255)
                        for y, (b0, c) in enumerate(bv)], 0)
    assert np.array_equal(src.astype(np.uint8), ref)


def test_wam_group_budget():
    """IG / SmoothGrad transform passes: multiples of the model group within the memory budget; the
    default budget is an eighth of the device's HBM, 8-64 GiB (8 GiB without a GPU)."""
    from wam_amd.engine import wam_budget_bytes, wam_group
    b = wam_budget_bytes()
    assert (8 << 30) <= b <= (64 << 30)
    if not torch.cuda.is_available():
        assert b == 8 << 30
    per = int(1.36e9)
    assert wam_group(2, 64, per, budget_bytes=8 << 30) == 6
    assert wam_group(2, 64, per, budget_bytes=36 << 30) == 28
    assert wam_group(2, 5, per, budget_bytes=36 << 30) == 5
    assert wam_group(4, 64, 100 << 30, budget_bytes=8 << 30) == 4


def test_profiling_phase_ranges(monkeypatch):
    """wam_amd.profiling.phase: a no-op unless WAM_PROFILE=1; when on, each phase pushes and pops one
    roctx range named wam:<name>, also when the body raises (CPU: a stand-in for the roctx library)."""
    from wam_amd import profiling
    calls = []

    class FakeRoctx:
        def roctxRangePushA(self, s):
            calls.append(("push", s))
            return 0

        def roctxRangePop(self):
            calls.append(("pop",))
            return 0

    monkeypatch.setattr(profiling, "ENABLED", False)
    with profiling.phase("model"):
        pass
    assert calls == []
    monkeypatch.setattr(profiling, "ENABLED", True)
    monkeypatch.setattr(profiling, "_LIB", FakeRoctx())
    with profiling.phase("model"):
        pass
    with pytest.raises(RuntimeError):
        with profiling.phase("trapz"):
            raise RuntimeError("x")
    assert calls == [("push", b"wam:model"), ("pop",), ("push", b"wam:trapz"), ("pop",)]
