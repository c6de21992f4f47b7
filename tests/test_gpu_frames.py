"""The mosaic accumulation in coefficient order (wam_frame_accumulate_coef, the path the classes
use) vs the per-pixel gather form (wam_frame_accumulate): bit-identical fp64 frames (same per-pixel
sum order), for the legacy and native c2 mosaics, normalised and not."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wav,frame", [("db4", "native"), ("haar", "legacy"), ("haar", "native")])
@pytest.mark.parametrize("normalize", [True, False])
def test_coef_order_equals_gather(wav, frame, normalize):
    from wam_amd import frames, plan as P
    from wam_amd._lib import check, lib, ptr, stream_of
    p = P.get_plan(2, (224, 224), 3, wav, "reflect", "cuda")
    n, groups = 5, 11
    gmap, (rh, rw) = frames.smooth_frame(p, n, frame, "cuda")
    torch.manual_seed(4)
    maps = torch.rand(groups * n * p.coeff_numel, device="cuda")
    bmax = torch.rand(groups, p.nbands, device="cuda") + 0.5
    base = torch.randn(n, rh, rw, dtype=torch.float64, device="cuda")
    a, b = base.clone(), base.clone()
    P.frame_accumulate(groups, n, gmap, maps, p.coeff_numel, bmax, p.nbands, normalize, a)
    assert P._inverse_map(gmap, p.coeff_numel) is not None  # the classes' path is the coefficient order
    src, band = gmap
    check(lib.wam_frame_accumulate(groups, n, src.numel(), ptr(src), ptr(band), ptr(maps), p.coeff_numel, ptr(bmax),
                                   p.nbands, int(normalize), ptr(b), stream_of(b.device)))
    assert torch.equal(a, b)


@pytest.mark.parametrize("shape,wav,J", [(224, "db4", 3), (512, "sym8", 5)])
@pytest.mark.parametrize("normalize", [True, False])
@pytest.mark.parametrize("weighted", [False, True])
def test_trapz_coef_order_equals_gather(shape, wav, J, normalize, weighted):
    """wam_frame_trapz_coef (the IG path's trapezoid) vs the per-pixel wam_frame_trapz over two
    chained passes (k0 = 0, then k0 > 0 carrying prev), NaN / inf map values included: bit-identical
    fp32 acc and prev. 512^2 sym8 J=5 takes the runs-of-items branch (mosaic tables > 2 MB, n * K / 2^22 = 2)."""
    from wam_amd import frames, plan as P
    from wam_amd._lib import check, lib, ptr, stream_of
    p = P.get_plan(2, (shape, shape), J, wav, "reflect", "cuda")
    n = 6 if shape == 224 else 32  # 32 x 293 K coefficients: 2 items per thread (runs branch)
    _, gmap, (rh, rw) = frames.ig_frames(p, n, "native", "cuda")
    assert P._inverse_map(gmap, p.coeff_numel) is not None
    src, band = gmap
    torch.manual_seed(5)
    acc_a = torch.zeros(n * rh * rw, device="cuda")
    prev_a = torch.zeros_like(acc_a)
    acc_b, prev_b = acc_a.clone(), prev_a.clone()
    k0 = 0
    for groups in (11, 5):
        maps = torch.rand(groups * n * p.coeff_numel, device="cuda")
        maps[::997] = float("nan")
        maps[5::1999] = float("inf")
        bmax = torch.rand(groups, p.nbands, device="cuda") + 0.5
        w = torch.rand(groups, device="cuda") if weighted else None
        P.frame_trapz(groups, k0, n, gmap, maps, p.coeff_numel, bmax, p.nbands, normalize, prev_a, acc_a, w)
        check(lib.wam_frame_trapz(groups, k0, n, src.numel(), ptr(src), ptr(band), ptr(maps), p.coeff_numel,
                                  ptr(bmax), p.nbands, int(normalize), ptr(w), ptr(prev_b), ptr(acc_b),
                                  stream_of(acc_b.device)))
        k0 += groups
    torch.cuda.synchronize()
    assert torch.equal(acc_a, acc_b) and torch.equal(prev_a, prev_b)
    assert acc_a.abs().sum() > 0


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("groups", [1, 2, 5])
@pytest.mark.parametrize("cube", [4 * 3072, 4 * 3000])  # 3 x cube % 256 == 0: the strided form; else 4 consecutive
def test_cube_accumulate_vec4_equals_scalar(mode, groups, cube):
    """wam_cube_accumulate's four-voxel forms (16-byte aligned index / accumulator, cube_len % 4 == 0;
    strided over 256-voxel wave blocks when the work divides, the c5 path) vs its one-voxel form (the
    same index map handed over misaligned): bit-identical acc and prev in every mode -- legacy in-loop
    averaging, weighted sum, trapezoid over two chained passes with NaN / inf map values -- with
    voxels outside the mosaic (index -1) included."""
    from wam_amd import plan as P
    torch.manual_seed(7 + mode + groups + cube)
    n, items_len = 3, cube + 64
    src = torch.randperm(items_len, device="cuda")[:cube].to(torch.int32)
    src[::13] = -1
    buf = torch.empty(cube + 1, dtype=torch.int32, device="cuda")
    buf[1:] = src
    src_mis = buf[1:]  # 4-byte offset: the one-voxel kernel
    assert src.data_ptr() % 16 == 0 and src_mis.data_ptr() % 16 != 0
    acc_a = torch.rand(n * cube, device="cuda")
    prev_a = torch.rand(n * cube, device="cuda") if mode == 2 else None
    acc_b = acc_a.clone()
    prev_b = prev_a.clone() if prev_a is not None else None
    k0 = 0
    for _ in range(2):
        maps = torch.randn(groups * n * items_len, device="cuda")
        if mode == 2:
            maps[::997] = float("nan")
            maps[5::1999] = float("inf")
        w = torch.rand(groups, device="cuda") if mode == 1 else None
        P.cube_accumulate(groups, k0, n, src, maps, items_len, mode, 25.0, acc_a, prev=prev_a, weights=w)
        P.cube_accumulate(groups, k0, n, src_mis, maps, items_len, mode, 25.0, acc_b, prev=prev_b, weights=w)
        k0 += groups
    torch.cuda.synchronize()
    assert torch.equal(acc_a, acc_b)
    if mode == 2:
        assert torch.equal(prev_a, prev_b)
