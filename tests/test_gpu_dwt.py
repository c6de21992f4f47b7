"""GPU parity of the HIP wavelet kernels (through the C-ABI) against the oracle / pywt fixtures.

Tolerance (fp32 kernels vs float64 references): max |err| <= 2e-6 * max(|ref|, 1) per band
(one fp32 rounding per tap; filters are fp32 casts of pywt's float64 tables, as in ptwt).
"""
import numpy as np
import pytest
import torch

from tests.helpers import flat_bands, max_rel, npz, pywt_cases, pywt_coeffs

pytestmark = pytest.mark.gpu

TOL = 2e-6


@pytest.fixture(scope="module")
def wam():
    import wam_amd
    from wam_amd import plan
    assert torch.cuda.is_available()
    return plan


def _tol(ref):
    return TOL * max(1.0, float(np.abs(ref).max()))


def _run_dec(P, x, dim, J, wav, mode, generic=False):
    lead = x.shape[0]
    shape = x.shape[1:]
    p = P.get_plan(dim, shape, J, wav, mode, "cuda", generic=generic)
    xt = torch.tensor(x, dtype=torch.float32, device="cuda")
    flat = p.wavedec(xt)
    return p, [b.cpu().numpy().astype(np.float64) for b in p.split(flat, lead)]


@pytest.mark.parametrize("dim", [1, 2, 3])
@pytest.mark.parametrize("generic", [False, True])
def test_wavedec_matches_pywt(wam, dim, generic):
    if dim != 2 and not generic:
        pytest.skip("fused kernels are 2D")
    d = npz("pywt_dwt.npz")
    for case, wav, mode, J in pywt_cases(dim):
        x = d[case + "_x"]
        _, got = _run_dec(wam, x, dim, J, wav, mode, generic)
        ref = flat_bands(pywt_coeffs(case, dim, J), dim)
        assert len(got) == len(ref)
        for b, (g, r) in enumerate(zip(got, ref)):
            assert g.shape == r.shape, (case, b, g.shape, r.shape)
            assert np.abs(g - r).max() <= _tol(r), (case, wav, mode, b, np.abs(g - r).max())


@pytest.mark.parametrize("dim", [1, 2, 3])
@pytest.mark.parametrize("generic", [False, True])
def test_waverec_matches_pywt(wam, dim, generic):
    """Synthesis of RANDOM coefficients (not an analysis output) vs pywt.waverec*."""
    if dim != 2 and not generic:
        pytest.skip("fused kernels are 2D")
    d = npz("pywt_dwt.npz")
    for case, wav, mode, J in pywt_cases(dim):
        rc = flat_bands(pywt_coeffs(case, dim, J, prefix="r"), dim)
        lead = rc[0].shape[0]
        x = d[case + "_x"]
        p = wam.get_plan(dim, x.shape[1:], J, wav, mode, "cuda", generic=generic)
        flat = torch.cat([torch.tensor(b, dtype=torch.float32).reshape(-1) for b in rc]).cuda()
        out = p.waverec(flat, lead)[0].cpu().numpy()
        ref = d[case + "_rrec"]
        assert out.shape == ref.shape, (case, out.shape, ref.shape)
        assert np.abs(out - ref).max() <= _tol(ref) * 4, (case, wav, mode, np.abs(out - ref).max())


@pytest.mark.parametrize("dim", [1, 2, 3])
def test_adjoint_matches_oracle(wam, dim):
    from oracle import dwt as odwt
    rs = np.random.RandomState(5)
    for case, wav, mode, J in pywt_cases(dim)[::3]:
        x = npz("pywt_dwt.npz")[case + "_x"]
        for generic in ([False, True] if dim == 2 else [True]):
            p = wam.get_plan(dim, x.shape[1:], J, wav, mode, "cuda", generic=generic)
            g = rs.standard_normal((x.shape[0],) + p.rec_shape)
            got = p.adjoint(torch.tensor(g, dtype=torch.float32, device="cuda"))
            got = [b.cpu().numpy() for b in p.split(got, x.shape[0])]
            ref = odwt.adjointn(g, [0] * (J + 1), wav, dim)
            ref = [ref[0]] + [lv[k] for lv in ref[1:] for k in (("da", "ad", "dd") if dim == 2 else sorted(lv))]
            if dim == 3:
                keys = ["aad", "ada", "add", "daa", "dad", "dda", "ddd"]
                ref = odwt.adjointn(g, [0] * (J + 1), wav, 3)
                ref = [ref[0]] + [lv[k] for lv in ref[1:] for k in keys]
            for b, (gb, rb) in enumerate(zip(got, ref)):
                assert gb.shape == rb.shape
                assert np.abs(gb - rb).max() <= _tol(rb) * 4, (case, b, np.abs(gb - rb).max())


@pytest.mark.parametrize("wav,shape,J", [("haar", (224, 224), 3), ("db4", (224, 224), 3), ("db4", (225, 223), 3),
                                         ("sym8", (512, 512), 5), ("db6", (64, 96), 2)])
def test_adjoint_dot_product(wam, wav, shape, J):
    """<waverec(c), g> == <c, adjoint(g)> (float64 accumulation of fp32 kernel outputs)."""
    p = wam.get_plan(2, shape, J, wav, "reflect", "cuda")
    torch.manual_seed(0)
    B = 3
    c = torch.randn(B * p.coeff_numel, device="cuda")
    g = torch.randn((B,) + p.rec_shape, device="cuda")
    lhs = (p.waverec(c, B)[0].double() * g.double()).sum().item()
    rhs = (c.double() * p.adjoint(g).double()).sum().item()
    assert abs(lhs - rhs) <= 1e-5 * (abs(lhs) + c.numel() ** 0.5), (lhs, rhs)


@pytest.mark.parametrize("wav,shape,J,B", [("db4", (224, 224), 3, 192), ("haar", (224, 224), 3, 192),
                                           ("sym8", (512, 512), 5, 24), ("db6", (225, 131), 3, 8)])
def test_fused_equals_generic_full_size(wam, wav, shape, J, B):
    fused = wam.get_plan(2, shape, J, wav, "reflect", "cuda")
    gen = wam.get_plan(2, shape, J, wav, "reflect", "cuda", generic=True)
    torch.manual_seed(1)
    x = torch.randn((B,) + shape, device="cuda")
    cf, cg = fused.wavedec(x), gen.wavedec(x)
    assert (cf - cg).abs().max().item() <= 1e-5 * cg.abs().max().item()
    rf, rg = fused.waverec(cf, B), gen.waverec(cf, B)
    assert (rf - rg).abs().max().item() <= 1e-5 * rg.abs().max().item()
    g = torch.randn((B,) + fused.rec_shape, device="cuda")
    af, ag = fused.adjoint(g), gen.adjoint(g)
    assert (af - ag).abs().max().item() <= 1e-5 * ag.abs().max().item()


@pytest.mark.parametrize("dim,wav,shape,J,mode", [
    (2, "db4", (224, 224), 3, "reflect"), (2, "haar", (224, 224), 3, "reflect"),
    (2, "sym8", (512, 512), 5, "reflect"), (2, "db4", (225, 225), 3, "symmetric"),
    (1, "db6", (80000,), 5, "reflect"), (3, "haar", (128, 128, 128), 2, "symmetric"),
    (3, "db4", (40, 36, 34), 2, "zero")])
def test_roundtrip_full_size(wam, dim, wav, shape, J, mode):
    """DWT -> IDWT round trip (reported; identity up to fp32 rounding), at BASELINE sizes."""
    p = wam.get_plan(dim, shape, J, wav, mode, "cuda")
    B = 4 if dim != 3 else 1
    torch.manual_seed(2)
    x = torch.randn((B,) + shape, device="cuda")
    r = p.waverec(p.wavedec(x), B)[0]
    sl = tuple(slice(0, s) for s in shape)
    err = (r[(slice(None),) + sl] - x).abs().max().item()
    print("roundtrip %s %s %s: max abs err %.3e" % (wav, shape, mode, err))
    assert err <= 1e-5 * x.abs().max().item()


def test_alpha_scaling_matches_scaled_coefficients(wam):
    p = wam.get_plan(2, (224, 224), 3, "db4", "reflect", "cuda")
    torch.manual_seed(3)
    c = torch.randn(6 * p.coeff_numel, device="cuda")
    alphas = np.linspace(0, 1, 5)
    out = p.waverec(c, 6, alphas=alphas)
    for i, a in enumerate(alphas):
        ref = p.waverec(c * float(np.float32(a)), 6)[0]
        assert torch.equal(out[i], ref)


@pytest.mark.parametrize("wav,shape,J", [("db4", (224, 224), 3), ("sym8", (100, 130), 2), ("haar", (64, 66), 4)])
def test_alpha_groups_row_synthesis(wam, wav, shape, J):
    """Row-kernel plans synthesise the IG alphas in groups (one launch per level per group, the
    details read once per group): 11 alphas (several groups, a partial last one) equal the
    single-alpha synthesis of the pre-scaled coefficients bit for bit."""
    p = wam.get_plan(2, shape, J, wav, "reflect", "cuda", flags=wam.PLAN_NO_PLANE)
    torch.manual_seed(5)
    B = 5
    c = torch.randn(B * p.coeff_numel, device="cuda")
    alphas = np.linspace(0, 1, 11)
    out = p.waverec(c, B, alphas=alphas)
    assert out.shape == (11, B) + p.rec_shape
    for i, a in enumerate(alphas):
        assert torch.equal(out[i], p.waverec(c * float(np.float32(a)), B)[0]), i


def test_transforms_api_autograd(wam):
    """wam_amd.waverec2 backward == the oracle's autograd through ptwt's conv_transpose."""
    import wam_amd
    from oracle import ptwt_torch
    torch.manual_seed(4)
    x = torch.randn(2, 3, 45, 37)
    cs = wam_amd.wavedec2(x.cuda(), "db4", level=2, mode="reflect")
    ref_cs = ptwt_torch.wavedec2(x.double(), "db4", level=2, mode="reflect")
    for a, b in zip(flat_bands(cs, 2), flat_bands(ref_cs, 2)):
        assert a.shape == b.shape
        assert (a.double().cpu() - b).abs().max().item() <= 1e-5
    leaves = [t.detach().requires_grad_() for t in flat_bands(cs, 2)]
    rec = wam_amd.waverec2([leaves[0]] + [wam_amd.WaveletDetailTuple2d(*leaves[1 + 3 * i:4 + 3 * i])
                                          for i in range(2)], "db4")
    g = torch.randn_like(rec)
    rec.backward(g)
    rl = [t.detach().requires_grad_() for t in flat_bands(ref_cs, 2)]
    rr = ptwt_torch.waverec2([rl[0]] + [ptwt_torch.WaveletDetailTuple2d(*rl[1 + 3 * i:4 + 3 * i])
                                        for i in range(2)], "db4")
    assert rr.shape == rec.shape
    assert (rr - rec.double().cpu()).abs().max().item() <= 1e-5
    rr.backward(g.double().cpu())
    for a, b in zip(leaves, rl):
        assert (a.grad.double().cpu() - b.grad).abs().max().item() <= 1e-5


def test_matlab_known_answers(wam):
    """Single-level MATLAB R2012a answers (pywt test data) through the 1D kernels."""
    d = npz("matlab_dwt.npz")
    cases = sorted({k.rsplit("_", 1)[0] for k in d.files})
    for c in cases:
        mode, wav, n = c.split("_")
        x = d[c + "_x"][None, :]
        _, got = _run_dec(wam, x, 1, 1, wav, mode, generic=True)
        assert max_rel(got[0][0], d[c + "_ma"]) < 1e-5, c
        assert max_rel(got[1][0], d[c + "_md"]) < 1e-5, c


# ------------------------------------------------------------------------------ fused WAM passes
@pytest.mark.parametrize("wav,shape,J,mode", [("db4", (224, 224), 3, "reflect"), ("haar", (224, 224), 3, "zero"),
                                              ("sym8", (96, 128), 2, "symmetric"), ("db6", (60, 44), 2, "constant"),
                                              ("haar", (512, 512), 5, "periodic"), ("db4", (37, 53), 2, "reflect"),
                                              ("sym4", (300, 700), 3, "symmetric"), ("db10", (33, 260), 1, "zero"),
                                              ("coif1", (7, 9), 1, "periodic")])
def test_fused_2d_paths_agree(wam, wav, shape, J, mode):
    """The 2D analysis implementations (row-resident, column-strip, per-axis) agree: bit-exact
    between the fused kernels (same tap order), to fp32 rounding with the per-axis one."""
    torch.manual_seed(5)
    B = 6
    x = torch.randn((B,) + shape, device="cuda")
    rows = wam.get_plan(2, shape, J, wav, mode, "cuda")
    col = wam.get_plan(2, shape, J, wav, mode, "cuda", flags=wam.PLAN_NO_ROWS)
    gen = wam.get_plan(2, shape, J, wav, mode, "cuda", generic=True)
    cr, cc, cg = rows.wavedec(x), col.wavedec(x), gen.wavedec(x)
    assert torch.equal(cr, cc)
    assert (cr - cg).abs().max().item() <= 1e-5 * cg.abs().max().item()
    g = torch.randn((B,) + rows.rec_shape, device="cuda")
    ar, ac, ag = rows.adjoint(g), col.adjoint(g), gen.adjoint(g)
    assert torch.equal(ar, ac)
    assert (ar - ag).abs().max().item() <= 1e-5 * ag.abs().max().item()


@pytest.mark.parametrize("wav,shape,J,mode", [("db5", (70, 90), 2, "reflect"), ("db6", (64, 130), 3, "symmetric"),
                                              ("db7", (100, 77), 2, "zero"), ("sym8", (150, 150), 3, "reflect"),
                                              ("db9", (61, 95), 2, "constant"), ("db10", (128, 40), 1, "reflect")])
def test_row_synthesis_matches_generic(wam, wav, shape, J, mode):
    """Per-level row synthesis (k_dwt2_syn; long filters on packed FMAs over a static register
    ring with lcm(L/2, prefetch) rows per iteration, odd L/2 included) vs the per-axis synthesis,
    with IG alphas in groups."""
    torch.manual_seed(8)
    B = 4
    rows = wam.get_plan(2, shape, J, wav, mode, "cuda", flags=wam.PLAN_NO_PLANE)
    gen = wam.get_plan(2, shape, J, wav, mode, "cuda", generic=True)
    c = gen.wavedec(torch.randn((B,) + shape, device="cuda"))
    al = [0.0, 0.3, 0.7, 1.0, 0.5, 0.9]
    a, g = rows.waverec(c, B, alphas=al), gen.waverec(c, B, alphas=al)
    assert (a - g).abs().max().item() <= 1e-5 * g.abs().max().item()


@pytest.mark.parametrize("wav,J", [("db4", 3), ("haar", 3), ("sym8", 2)])
def test_noisy_wavedec_equals_noise_then_wavedec(wam, wav, J):
    p = wam.get_plan(2, (224, 224), J, wav, "reflect", "cuda")
    assert p.caps & wam.CAP_NOISY_WAVEDEC
    torch.manual_seed(6)
    N, C, S = 5, 3, 3
    x = torch.randn(N, C, 224, 224, device="cuda")
    sigma = wam.item_sigma(x, C * 224 * 224, C * 224 * 224, 0.25)
    fused = p.wavedec_noisy(x, sigma, S, N, C, seed=1234, sample_base=7)
    noisy = wam.noise_add(x, sigma, S, N, C * 224 * 224, C * 224 * 224, seed=1234, sample_base=7)
    ref = p.wavedec(noisy.view(S * N * C, 224, 224))
    assert torch.equal(fused, ref)


@pytest.mark.parametrize("n,J,wav,mode,S,N", [(80000, 5, "db6", "reflect", 3, 2), (9000, 5, "db6", "constant", 2, 3),
                                            (4096, 3, "haar", "symmetric", 4, 2), (1000, 4, "sym8", "zero", 2, 2),
                                            (40, 3, "db4", "reflect", 3, 1), (50000, 4, "coif2", "reflect", 2, 2)])
def test_noisy_dwt1_equals_noise_then_wavedec(wam, n, J, wav, mode, S, N):
    """1D tile analysis with the SmoothGrad noise fused on the load -- interior tiles (aligned groups
    of 4, one Philox call each, samples fastest), persistent and generic boundary tiles (per-sample
    calls) -- vs wam_noise_add + the same analysis: bit-identical, with a sample base and a seed."""
    p = wam.get_plan(1, (n,), J, wav, mode, "cuda")
    assert p.caps & wam.CAP_NOISY_WAVEDEC
    torch.manual_seed(13)
    x = torch.randn(N, n, device="cuda")
    sigma = wam.item_sigma(x, n, n, 0.2)
    fused = p.wavedec_noisy(x, sigma, S, N, 1, seed=91, sample_base=5)
    noisy = wam.noise_add(x, sigma, S, N, n, n, seed=91, sample_base=5)
    ref = p.wavedec(noisy.view(S * N, n))
    assert torch.equal(fused, ref)


@pytest.mark.parametrize("shape,J,mode,S,N", [((128, 128, 128), 2, "symmetric", 2, 3), ((16, 12, 20), 1, "reflect", 3, 2),
                                              ((8, 16, 24), 2, "zero", 5, 1), ((6, 10, 4), 1, "symmetric", 2, 4)])
def test_noisy_haar3_equals_noise_then_wavedec(wam, shape, J, mode, S, N):
    """3D Haar analysis with the SmoothGrad noise fused on the load (single-channel volumes, the
    samples of a volume chunk in consecutive workgroups) vs wam_noise_add + the block kernel:
    bit-identical, with a sample base and a non-zero seed; channels != 1 is refused."""
    p = wam.get_plan(3, shape, J, "haar", mode, "cuda")
    assert p.caps & wam.CAP_NOISY_WAVEDEC
    torch.manual_seed(12)
    vol = shape[0] * shape[1] * shape[2]
    x = torch.randn((N, 1) + shape, device="cuda")
    sigma = wam.item_sigma(x, vol, vol, 0.3)
    fused = p.wavedec_noisy(x, sigma, S, N, 1, seed=77, sample_base=3)
    noisy = wam.noise_add(x, sigma, S, N, vol, vol, seed=77, sample_base=3)
    ref = p.wavedec(noisy.view((S * N,) + shape))
    assert torch.equal(fused, ref)
    with pytest.raises(Exception):
        p.wavedec_noisy(torch.randn((N, 2) + shape, device="cuda"), sigma, S, N, 2, seed=77)


@pytest.mark.parametrize("wav,shape,J,C", [("db4", (224, 224), 3, 3), ("haar", (224, 224), 3, 3),
                                           ("sym8", (128, 96), 2, 1), ("db6", (225, 223), 3, 3),
                                           ("db2", (64, 300), 2, 1), ("sym8", (512, 512), 5, 3),
                                           ("db4", (300, 302), 3, 1)])
def test_adjoint_maps_equals_adjoint_then_subband_maps(wam, wav, shape, J, C):
    p = wam.get_plan(2, shape, J, wav, "reflect", "cuda")
    assert p.caps & wam.CAP_ADJOINT_MAPS
    torch.manual_seed(7)
    G, N = 3, 4
    g = torch.randn((G * N * C,) + p.rec_shape, device="cuda")
    maps, bmax, full = p.adjoint_maps(g, G, N, C, full=True)
    cg = p.adjoint(g)
    rmaps, rbmax = wam.subband_maps(p, cg, G, N, C)
    assert torch.equal(full, cg)
    # the plane-resident kernel averages the channels BEFORE the (linear) adjoint; the per-level
    # kernels after it, in numpy's order: equal up to fp32 rounding of the reordered sums
    tol = 2e-6 * float(rbmax.max())
    assert float((maps - rmaps).abs().max()) <= tol
    assert float((bmax - rbmax).abs().max()) <= tol


@pytest.mark.parametrize("wav,shape,J,mode", [("db4", (224, 224), 3, "reflect"), ("haar", (224, 224), 3, "reflect"),
                                              ("db2", (64, 96), 4, "symmetric"), ("db3", (100, 84), 2, "zero"),
                                              ("db4", (224, 224), 1, "periodic"), ("sym4", (36, 252), 3, "constant")])
def test_plane_resident_equals_per_level(wam, wav, shape, J, mode):
    """All-levels-in-one-workgroup kernels vs the per-level row kernels (and the generic path)."""
    fast = wam.get_plan(2, shape, J, wav, mode, "cuda")
    ref = wam.get_plan(2, shape, J, wav, mode, "cuda", flags=wam.PLAN_NO_PLANE)
    gen = wam.get_plan(2, shape, J, wav, mode, "cuda", generic=True)
    torch.manual_seed(3)
    B = 37
    x = torch.randn((B,) + shape, device="cuda")
    a, b, c = fast.wavedec(x), ref.wavedec(x), gen.wavedec(x)
    assert float((a - c).abs().max()) < 1e-5 and float((b - c).abs().max()) < 1e-5
    g = torch.randn((B,) + fast.rec_shape, device="cuda")
    a, c = fast.adjoint(g), gen.adjoint(g)
    assert float((a - c).abs().max()) < 1e-5
    cf = gen.wavedec(x)
    a, b, c = fast.waverec(cf, B), ref.waverec(cf, B), gen.waverec(cf, B)
    assert torch.equal(a, b)  # same arithmetic order as the per-level synthesis kernel
    assert float((a - c).abs().max()) < 1e-5
    al = [0.0, 0.25, 1.0 / 3.0, 1.0]
    a, b = fast.waverec(cf, B, alphas=al), ref.waverec(cf, B, alphas=al)
    assert a.shape == (len(al), B) + fast.rec_shape and torch.equal(a, b)
    N, C = 5, 3
    xs = torch.randn((N, C) + shape, device="cuda")
    sigma = wam.item_sigma(xs, C * shape[0] * shape[1], C * shape[0] * shape[1], 0.25)
    S = 3
    if fast.caps & wam.CAP_NOISY_WAVEDEC and ref.caps & wam.CAP_NOISY_WAVEDEC:
        a = fast.wavedec_noisy(xs, sigma, S, N, C, seed=99, sample_base=4)
        b = ref.wavedec_noisy(xs, sigma, S, N, C, seed=99, sample_base=4)
        assert float((a - b).abs().max()) < 1e-5


def test_plane_maps_band_max_over_many_groups(wam):
    """maps / batch-global maxima of the plane kernel at the bench's WAM-group size (25 x 64)."""
    p = wam.get_plan(2, (224, 224), 3, "db4", "reflect", "cuda")
    torch.manual_seed(5)
    G, N, C = 25, 64, 3
    g = torch.randn((G * N * C, 224, 224), device="cuda")
    maps, bmax, _ = p.adjoint_maps(g, G, N, C, full=False)
    m = maps.view(G, N, p.coeff_numel)
    for b in range(p.nbands):
        lo, hi = p.band_offsets[b], p.band_offsets[b + 1]
        assert torch.equal(bmax[:, b], m[:, :, lo:hi].amax(dim=(1, 2)))
    # spot-check two images against adjoint + subband maps
    sel = torch.tensor([0, G * N - 1], device="cuda")
    gi = g.view(G * N, C, 224, 224)[sel].reshape(2 * C, 224, 224)
    rmaps, _ = wam.subband_maps(p, p.adjoint(gi), 1, 2, C)
    assert float((m.view(G * N, -1)[sel].reshape(-1) - rmaps).abs().max()) <= 2e-6 * float(bmax.max())


@pytest.mark.parametrize("wav,n,J,mode", [("db6", 80000, 5, "reflect"), ("haar", 4097, 3, "symmetric"),
                                          ("sym8", 1001, 4, "zero"), ("db6", 9000, 5, "constant"),
                                          ("db4", 37, 3, "reflect"), ("db2", 12345, 6, "symmetric"),
                                          ("coif2", 50000, 4, "reflect")])
def test_dwt1_tiles_equal_per_axis(wam, wav, n, J, mode):
    """Fused multi-level 1D tiles (all levels per signal tile in LDS) vs the per-axis kernels, for
    wavedec, waverec (with IG alphas) and the adjoint; the per-axis path is pinned to pywt above."""
    fast = wam.get_plan(1, (n,), J, wav, mode, "cuda")
    gen = wam.get_plan(1, (n,), J, wav, mode, "cuda", generic=True)
    torch.manual_seed(9)
    B = 6
    x = torch.randn(B, n, device="cuda")
    a, b = fast.wavedec(x), gen.wavedec(x)
    assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max())
    ra, rb = fast.waverec(b, B), gen.waverec(b, B)
    assert torch.equal(ra, rb)  # same per-sample accumulation order as k_synthesis_axis
    al = [0.0, 0.5, 1.0]
    assert torch.equal(fast.waverec(b, B, alphas=al), gen.waverec(b, B, alphas=al))
    g = torch.randn((B,) + fast.rec_shape, device="cuda")
    a, b = fast.adjoint(g), gen.adjoint(g)
    assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max())


@pytest.mark.parametrize("shape,J,mode", [((128, 128, 128), 2, "symmetric"), ((16, 12, 20), 1, "reflect"),
                                          ((8, 16, 24), 2, "zero")])
def test_haar3_blocks_equal_per_axis(wam, shape, J, mode):
    """Fused 3D Haar blocks (all levels per 2^J block in registers) vs the per-axis kernels:
    wavedec, waverec (with IG alphas) and the adjoint, bit-identical (same arithmetic order)."""
    fast = wam.get_plan(3, shape, J, "haar", mode, "cuda")
    gen = wam.get_plan(3, shape, J, "haar", mode, "cuda", generic=True)
    torch.manual_seed(10)
    B = 3
    x = torch.randn((B,) + shape, device="cuda")
    a, b = fast.wavedec(x), gen.wavedec(x)
    assert torch.equal(a, b)
    assert torch.equal(fast.waverec(b, B), gen.waverec(b, B))
    al = [0.25, 1.0]
    assert torch.equal(fast.waverec(b, B, alphas=al), gen.waverec(b, B, alphas=al))
    g = torch.randn((B,) + fast.rec_shape, device="cuda")
    assert torch.equal(fast.adjoint(g), gen.adjoint(g))


@pytest.mark.parametrize("wav,shape,J,mode", [("db4", (40, 36, 34), 2, "zero"), ("db2", (17, 23, 30), 2, "reflect"),
                                              ("sym4", (33, 16, 25), 2, "symmetric"), ("db3", (20, 21, 22), 2, "constant"),
                                              ("sym8", (48, 40, 36), 2, "reflect"), ("coif1", (19, 18, 17), 1, "periodic"),
                                              ("haar", (15, 14, 13), 2, "reflect"), ("db6", (64, 64, 64), 2, "symmetric"),
                                              ("db4", (128, 128, 128), 2, "reflect")])
def test_dwt3_tile_levels_equal_per_axis(wam, wav, shape, J, mode):
    """Fused 3D levels (dwt3_tile.hip: the footprint of a tile in LDS, W / H / D passes there, one
    launch per level; filters up to 8 taps) vs the per-axis kernels (three passes per level):
    wavedec3, waverec3 with IG alphas and the adjoint bit-identical (same axis order, taps and fma
    chains), odd sizes, every mode; the fused kernels must be the ones that ran (db6 / sym8 keep the
    per-axis path and are checked as a regression)."""
    fast = wam.get_plan(3, shape, J, wav, mode, "cuda")
    gen = wam.get_plan(3, shape, J, wav, mode, "cuda", generic=True)
    torch.manual_seed(14)
    B = 2
    x = torch.randn((B,) + shape, device="cuda")
    wam.timing_drain()
    wam.timing_enable(True)
    a = fast.wavedec(x)
    torch.cuda.synchronize()
    wam.timing_enable(False)
    names = {r[0] for r in wam.timing_drain()}
    b = gen.wavedec(x)
    assert torch.equal(a, b)
    from wam_amd.filters import get_wavelet
    fused = len(get_wavelet(wav).dec_lo) <= 8  # longer filters keep the per-axis kernels
    if fused and (wav != "haar" or any(n % 4 for n in shape)):
        assert "k_dwt3_ana_tile" in names, names
    al = [0.25, 1.0]
    wam.timing_drain()
    wam.timing_enable(True)
    r = fast.waverec(b, B, alphas=al)
    torch.cuda.synchronize()
    wam.timing_enable(False)
    names = {r_[0] for r_ in wam.timing_drain()}
    assert torch.equal(r, gen.waverec(b, B, alphas=al))
    assert torch.equal(fast.waverec(b, B), gen.waverec(b, B))
    if fused and wav != "haar":
        assert "k_dwt3_syn_tile" in names, names
    g = torch.randn((B,) + fast.rec_shape, device="cuda")
    assert torch.equal(fast.adjoint(g), gen.adjoint(g))


@pytest.mark.parametrize("wav,shape,J,mode", [("db4", (224, 224), 3, "reflect"), ("haar", (224, 224), 3, "reflect"),
                                              ("db2", (64, 96), 4, "symmetric"), ("db3", (100, 84), 2, "zero"),
                                              ("db4", (37, 52), 2, "reflect"), ("sym4", (36, 200), 3, "constant"),
                                              ("db4", (224, 224), 1, "periodic"), ("db4", (17, 16), 3, "reflect")])
def test_plane_coop_equals_wave_chunks(wam, wav, shape, J, mode):
    """Cooperative level-1 row stream (plan flag WAM_PLAN_FORCE_COOP) vs the wave-chunk form
    (WAM_PLAN_NO_COOP): the same taps in the same fma order, so wavedec, noisy wavedec and the
    maps epilogue are bit-identical."""
    plans = {"0": wam.get_plan(2, shape, J, wav, mode, "cuda", flags=wam.PLAN_NO_COOP),
             "1": wam.get_plan(2, shape, J, wav, mode, "cuda", flags=wam.PLAN_FORCE_COOP)}
    if not all(p.caps & wam.CAP_NOISY_WAVEDEC for p in plans.values()):
        pytest.skip("plane kernels do not cover this geometry")
    torch.manual_seed(11)
    N, C, S = 3, 3, 4
    x = torch.randn((N, C) + shape, device="cuda")
    sigma = wam.item_sigma(x, C * shape[0] * shape[1], C * shape[0] * shape[1], 0.25)
    g = torch.randn((S * N * C,) + plans["0"].rec_shape, device="cuda")
    out = {}
    for flag, p in plans.items():
        out[flag] = (p.wavedec(x.view(N * C, *shape)),
                     p.wavedec_noisy(x, sigma, S, N, C, seed=5, sample_base=2),
                     p.adjoint(g),
                     p.adjoint_maps(g, S, N, C, full=False)[:2] if p.caps & wam.CAP_ADJOINT_MAPS else ())
        torch.cuda.synchronize()
    for a, b in zip(out["0"][:3], out["1"][:3]):
        assert torch.equal(a, b)
    for a, b in zip(out["0"][3], out["1"][3]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("items,stride,length", [(64, 3 * 224 * 224, 3 * 224 * 224), (256, 80000, 80000),
                                                 (16, 128 ** 3, 128 ** 3), (3, 1001, 999), (5, 4096, 4096),
                                                 (1, 7, 7), (2, 40000, 37)])
def test_item_sigma_split_matches_torch(wam, items, stride, length):
    """Full-chip split sigma reduction (items x ranges workgroups, last arrival combines) vs the
    reference formula spread * (x.max() - x.min()) in fp32 (lib/wam_2D.py:396-399), at the c2, c3
    and c5 shapes and ragged ones; a NaN item propagates, a constant item gives 0; two calls on the
    same workspace agree (its arrival counters are reset)."""
    torch.manual_seed(23)
    x = torch.randn(items * stride, device="cuda") * 3.0
    xv = x.view(items, stride)[:, :length]
    if items >= 3:
        xv[1].fill_(0.75)                     # constant item
        xv[2, length // 2] = float("nan")     # NaN item
    spread = 0.15
    got = wam.item_sigma(x, stride, length, spread)
    ref = np.float32(spread) * (xv.amax(dim=1) - xv.amin(dim=1))
    if items >= 3:
        assert torch.isnan(got[2]) and torch.isnan(ref[2])
        assert float(got[1]) == 0.0
    ok = ~torch.isnan(ref)
    assert torch.equal(got[ok], ref[ok])
    again = wam.item_sigma(x, stride, length, spread)
    assert torch.equal(again[ok], got[ok])
